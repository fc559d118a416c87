#!/bin/bash
# end-of-session check at HEAD: smoke, default C2 bench (verified), kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final/prof
S=scripts/gpu_step.sh
$S 240 gpurun_out/final/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -n 2 gpurun_out/final/smoke.log
$S 600 gpurun_out/final/bench.log python -u bench.py || exit $?
grep "^{" gpurun_out/final/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/final/prof/log 2>&1 || exit $?
rm -f gpurun_out/final/prof/*trace.csv
