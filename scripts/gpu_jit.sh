#!/bin/bash
# window-engine parity (hipRTC + ahead-of-time kernels), C2 checks, then quick perf
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh 600 gpurun_out/jit_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "window_engine or c2_device_run or c2_full_size" || exit $?
tail -5 gpurun_out/jit_tests.log
grep -q " passed" gpurun_out/jit_tests.log && ! grep -q "FAILED\|Error" gpurun_out/jit_tests.log || exit 1
bash scripts/gpu_quick.sh
