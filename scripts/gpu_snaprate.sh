#!/bin/bash
# snapshot/restore with output rate limiters
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 400 gpurun_out/snaprate_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread \
   tests/test_gpu_snapshot.py -p no:cacheprovider -k rate_limited || exit $?
tail -n 3 gpurun_out/snaprate_tests.log
