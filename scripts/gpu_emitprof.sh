#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SH_BK_PROFILE=1 scripts/gpu_step.sh 200 gpurun_out/bench_phase.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "clock ticks" gpurun_out/bench_phase.log | tail -2
