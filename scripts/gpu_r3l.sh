#!/bin/bash
# round 3: C4 on the SURVEY 8d workload (100M events, 10M users, 20/60/20, calls of 4,096), one pass with the
# >=1M-event CPU baseline; per-call kernel / copy summary on the first 3,000 calls
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r3l_c4prof -o run -- python -u bench.py --config c4 --c4-calls 3000 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/r3l_c4prof.json 2> gpurun_out/r3l_c4prof.err || { tail -20 gpurun_out/r3l_c4prof.err; exit 1; }
cat gpurun_out/r3l_c4prof.json
find gpurun_out/r3l_c4prof -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-140
timeout -k 10 1000 python -u bench.py --config c4 --steps 1 --warmup 0 > gpurun_out/r3l_c4.json 2> gpurun_out/r3l_c4.err || { tail -20 gpurun_out/r3l_c4.err; exit 1; }
cat gpurun_out/r3l_c4.json
