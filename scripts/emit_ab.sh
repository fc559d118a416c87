#!/bin/bash
# emitter change check: bucket tests (packed rows), C2 and C2 + aggregates step times
set -o pipefail
mkdir -p gpurun_out/emit_ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_agg.py \
    > gpurun_out/emit_ab/tests.log 2>&1 || exit 1
for agg in "" "--agg"; do
  timeout -k 10 300 python bench.py --config c2 $agg --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
      > gpurun_out/emit_ab/b${agg}.json 2>/dev/null || exit 1
done
