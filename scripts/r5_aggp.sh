#!/bin/bash
# C2 + aggregates with the parallel fixed-point carry (k_bk_aggp): tests, bench line, kernel split
set -o pipefail
mkdir -p gpurun_out/aggp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_agg.py \
    > gpurun_out/aggp/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 \
    > gpurun_out/aggp/bench.json 2> gpurun_out/aggp/bench.err &&
SH_BK_PROFILE=1 timeout -k 10 300 python bench.py --config c2 --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify \
    > gpurun_out/aggp/prof.json 2> gpurun_out/aggp/prof.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aggp/prof -o run -- python bench.py --config c2 --agg \
    --steps 10 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/aggp/rp.log 2>&1
