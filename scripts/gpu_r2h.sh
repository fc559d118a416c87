#!/bin/bash
# Re-entry evidence at HEAD: smoke, the whole -m gpu suite, C2 bench (verified), kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 240 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -n 2 gpurun_out/smoke.log
$S 600 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 3 gpurun_out/gpu_tests.log
$S 300 gpurun_out/bench_c2.log python -u bench.py --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/bench_c2.log | cut -c1-400
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
