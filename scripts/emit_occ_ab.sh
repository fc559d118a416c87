#!/bin/bash
# emitter occupancy A/B on C2 (packed rows): 4 waves/SIMD (6 rows per lane) vs 5 (3) vs 6 (2, three workgroups per CU)
set -o pipefail
mkdir -p gpurun_out/emit_occ
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py -k packed \
    > gpurun_out/emit_occ/tests.log 2>&1 || exit 1
for occ in 4 6 5 4 6; do
  SH_EMIT_OCC=$occ timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
      >> gpurun_out/emit_occ/b_$occ.json 2>/dev/null || exit 1
done
SH_EMIT_OCC=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py -k packed \
    > gpurun_out/emit_occ/tests6.log 2>&1
