#!/bin/bash
# full GPU session: smoke, all GPU parity tests, bench (verified + cpu baseline), kernel-trace profile
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 240 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 gpurun_out/smoke.log
$S 900 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -3 gpurun_out/gpu_tests.log
grep -q "failed\|error" gpurun_out/gpu_tests.log && exit 1
$S 600 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 2 || exit $?
tail -1 gpurun_out/bench.log
bash scripts/gpu_prof.sh
