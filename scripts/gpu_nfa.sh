#!/bin/bash
# general-engine GPU parity: randomized apps + the fixtures on the device
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 600 gpurun_out/nfa_tests.log python -u -m pytest tests/test_gpu_nfa.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
tail -3 gpurun_out/nfa_tests.log
$S 600 gpurun_out/fx_tests.log python -u -m pytest tests/test_gpu_parity.py -k fixture -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
tail -3 gpurun_out/fx_tests.log
