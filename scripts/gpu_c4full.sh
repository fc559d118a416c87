#!/bin/bash
# C4 at BASELINE size (10M users, 100 s of playback) on the streaming path
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 1000 python -u bench.py --config c4 --steps 1 --warmup 0 --cpu-sample 1000000 > gpurun_out/c4/bench_full.log 2>&1 || { tail -5 gpurun_out/c4/bench_full.log; exit 1; }
tail -n 2 gpurun_out/c4/bench_full.log
