#!/bin/bash
# C2 tiling sweep: JIT workgroup tile / halo and the arrival-tile shift
# (SH_JIT_TILE, SH_JIT_HALO, SH_TILE_SHIFT); one unverified bench per point
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for cfg in "256 256 19" "256 64 19" "512 128 19" "1024 256 19" "1024 64 19" "256 256 17" "256 256 21" "1024 128 20"; do
  set -- $cfg
  tag="t$1_h$2_s$3"
  SH_JIT_TILE=$1 SH_JIT_HALO=$2 SH_TILE_SHIFT=$3 timeout -k 10 240 python -u bench.py --steps 4 --warmup 1 \
      --cpu-sample 0 --no-verify > gpurun_out/sweep/$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -5 gpurun_out/sweep/$tag.log; exit $rc; fi
  python - "$tag" gpurun_out/sweep/$tag.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
j = json.loads(l)
print(sys.argv[1], "%.3f Gev/s" % (j["value"] / 1e9), "ms/step %.2f" % j["ms_per_step"],
      {k: round(v, 2) for k, v in j["phase_ms"].items()})
PY
done
