#!/bin/bash
# first-round GPU session: smoke, parity tests, bench, rocprof
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 180 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
$S 900 gpurun_out/gpu_tests.log python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -p no:cacheprovider
tail -5 gpurun_out/gpu_tests.log
$S 600 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 2
tail -3 gpurun_out/bench.log
