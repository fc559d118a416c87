#!/bin/bash
# quick perf iteration: bench (verified) + kernel-trace stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
scripts/gpu_step.sh 300 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 || exit $?
tail -1 gpurun_out/bench.log
bash scripts/gpu_prof.sh
