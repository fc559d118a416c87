#!/bin/bash
# XCD-ordered radix scatter tiles: parity (general engine, C3, C1 window) and A/B on C3 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof3
S=scripts/gpu_step.sh
$S 500 gpurun_out/xcd_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread \
   tests/test_gpu_c3.py tests/test_gpu_nfa.py tests/test_gpu_c1.py tests/test_gpu_rules.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/xcd_tests.log
for x in 1 0 1; do
SH_RADIX_XCD=$x $S 300 gpurun_out/bench_c3_x$x.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "C3 xcd=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3_x$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3_x$x.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3_x$x.log)"
SH_RADIX_XCD=$x $S 300 gpurun_out/bench_c5_x$x.log python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 0 --no-verify || exit $?
echo "C5 xcd=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c5_x$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c5_x$x.log)"
done
