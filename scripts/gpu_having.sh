#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/having_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_having.py tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_range_partition.py || exit $?
tail -n 2 gpurun_out/having_tests.log
grep -E "^FAILED" gpurun_out/having_tests.log | head
