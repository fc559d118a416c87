#!/bin/bash
# C3 (raw rows, 3 values) emitter occupancy: SH_EMIT_OCC 4 vs 6, and the C3 GPU tests at the default
set -o pipefail
mkdir -p gpurun_out/c3_occ
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c3.py \
    > gpurun_out/c3_occ/tests.log 2>&1 || exit 1
for occ in 4 6 4 6; do
  SH_EMIT_OCC=$occ timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
      >> gpurun_out/c3_occ/b_$occ.json 2>/dev/null || exit 1
done
