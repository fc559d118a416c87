"""Write the generated bucketed-matcher source (shb_match + shb_pmatch) of an app
(default C2) to a file and print each kernel's register / LDS / scratch use, from
an offline hipcc build of that source (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from siddhi_amd import abi, build, compiler, synth  # noqa: E402


def main(out="/tmp/shb_src.hip", app=synth.C2_QUERY):
    lib = abi.bind_product(C.CDLL(build.build()))
    d = compiler.compile_app(app).descriptor()
    h = C.c_void_p()
    assert lib.sh_compile(C.byref(d), C.byref(h)) == abi.SH_OK
    buf = C.create_string_buffer(1 << 22)
    rc = lib.shx_bucket_compile(h, buf, 1 << 22)
    src = buf.value.decode()
    lib.sh_destroy(h)
    assert rc == abi.SH_OK, rc
    # hipcc form: the hipRTC prelude's typedefs come from the HIP headers instead
    body = re.sub(r"^typedef __hip_internal::.*$|^typedef decltype\(sizeof\(0\)\) size_t;$|^#define INT(32|64)_MIN .*$",
                  "", src, flags=re.M)
    with open(out, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n#include <stdint.h>\n" + body)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-gpu-flush-denormals-to-zero", "--cuda-device-only", "-c", out, "-o", out + ".o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    for line in r.stderr.splitlines():
        if "remark" in line and any(k in line for k in ("Function Name", "VGPRs:", "SGPRs", "ScratchSize", "Occupancy",
                                                          "LDS Size", "AGPRs")):
            print(line.split("remark: ")[-1])
    if r.returncode:
        print(r.stderr[-4000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:2]))
