#!/bin/bash
# order by / limit / offset GPU parity; round-2 numbers for C5 (1,000 rules, verified) and C4
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 400 gpurun_out/order_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
   tests/test_order_limit.py tests/test_having.py -p no:cacheprovider || exit $?
tail -3 gpurun_out/order_tests.log
$S 400 gpurun_out/bench_c5.log python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 8192 --cpu-threads 1 || exit $?
grep '^{' gpurun_out/bench_c5.log | cut -c1-400 || true
$S 400 gpurun_out/bench_c4.log python -u bench.py --config c4 --steps 1 --warmup 0 --c4-calls 3000 --cpu-sample 200000 || exit $?
grep '^{' gpurun_out/bench_c4.log | cut -c1-400 || true
