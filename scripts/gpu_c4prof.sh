#!/bin/bash
# C4 profile: kernel + HIP runtime statistics of a small streaming run
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4prof
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- \
    python -u bench.py --config c4 --keys 200000 --seconds 10 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4prof/log 2>&1 || { tail -5 gpurun_out/c4prof/log; exit 1; }
tail -n 1 gpurun_out/c4prof/log
