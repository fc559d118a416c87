#!/bin/bash
# k_bk_aggp: aggregate tests, step time, phase ticks (SH_BK_PROFILE)
set -o pipefail
mkdir -p gpurun_out/aggp_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_agg.py \
    > gpurun_out/aggp_ab/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
    > gpurun_out/aggp_ab/bench.json 2> gpurun_out/aggp_ab/bench.err || exit 1
SH_BK_PROFILE=1 timeout -k 10 300 python bench.py --config c2 --agg --steps 2 --warmup 1 --cpu-sample 0 \
    --no-verify > /dev/null 2> gpurun_out/aggp_ab/prof.err
