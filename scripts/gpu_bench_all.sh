#!/bin/bash
# bench lines of every config (C2 default, C5 rules, C3 sequence+count)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 300 gpurun_out/bench_c2_small.log python -u bench.py --steps 2 --warmup 1 --events 2000000 --cpu-sample 100000 || exit $?
tail -n 1 gpurun_out/bench_c2_small.log
$S 600 gpurun_out/bench_c5.log python -u bench.py --config c5 --steps 3 --warmup 1 || exit $?
tail -n 2 gpurun_out/bench_c5.log
$S 600 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 1000000 || exit $?
tail -n 2 gpurun_out/bench_c3.log
