#!/bin/bash
# HEAD check: smoke + every -m gpu test
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 240 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -n 2 gpurun_out/smoke.log
$S 800 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 3 gpurun_out/gpu_tests.log
