#!/bin/bash
# rate limiter / selection / snapshot GPU parity, then the C3 PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 500 gpurun_out/rate_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
   tests/test_rate_limit.py tests/test_order_limit.py tests/test_having.py tests/test_gpu_snapshot.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/rate_tests.log
scripts/gpu_c3pmc.sh
