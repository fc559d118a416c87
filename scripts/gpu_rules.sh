#!/bin/bash
# rule-engine (C5) GPU parity + a C5-size timing probe
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 900 gpurun_out/rules_tests.log python -u -m pytest tests/test_gpu_rules.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 5 gpurun_out/rules_tests.log
