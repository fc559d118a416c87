#!/bin/bash
# device tie-break of due keys: parity with the device path forced, the full GPU
# suite, then C4 at BASELINE size
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4d
S=scripts/gpu_step.sh
SH_TIEBREAK_MIN=1 $S 400 gpurun_out/c4d/tests_forced.log python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_nfa.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/c4d/tests_forced.log
grep -q " passed" gpurun_out/c4d/tests_forced.log && ! grep -q " failed" gpurun_out/c4d/tests_forced.log || exit 1
$S 600 gpurun_out/c4d/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/c4d/gpu_tests.log
grep -q " passed" gpurun_out/c4d/gpu_tests.log && ! grep -q " failed" gpurun_out/c4d/gpu_tests.log || exit 1
timeout -k 10 700 python -u bench.py --config c4 --steps 1 --warmup 0 --cpu-sample 1000000 > gpurun_out/c4d/bench_full.log 2>&1 || { tail -3 gpurun_out/c4d/bench_full.log; exit 1; }
grep "^{" gpurun_out/c4d/bench_full.log
