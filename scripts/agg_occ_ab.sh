#!/bin/bash
# C2 + aggregates emitter (6 packed values): 4 waves x 4 rows vs 6 waves x 1 row (SH_EMIT_OCC=66)
set -o pipefail
mkdir -p gpurun_out/agg_occ
for occ in 4 66 4 66; do
  SH_EMIT_OCC=$occ timeout -k 10 300 python bench.py --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
      >> gpurun_out/agg_occ/b_$occ.json 2>/dev/null || exit 1
done
SH_EMIT_OCC=66 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_agg.py -k packed \
    > gpurun_out/agg_occ/tests.log 2>&1
