#!/bin/bash
# C3 on the rise-and-fall sequence engine: parity + bench + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c3
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
scripts/gpu_step.sh 900 gpurun_out/c3_tests.log $T tests/test_gpu_c3.py || exit $?
grep -E "passed|failed" gpurun_out/c3_tests.log | tail -2
scripts/gpu_step.sh 600 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/bench_c3.log | cut -c1-500
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof_c3/bench.log 2>&1
echo "prof rc=$?"
