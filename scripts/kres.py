"""Per-kernel register / LDS usage of one HIP source (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for f, r in rows.items():
    print(f"{f[:60]:60s} vgpr {r.get('VGPRs')} agpr {r.get('AGPRs')} vspill {r.get('VGPRs Spill')} "
          f"sspill {r.get('SGPRs Spill')} lds {r.get('LDS Size [bytes/block]')} occ {r.get('Occupancy [waves/SIMD]')}")
