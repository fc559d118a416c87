#!/bin/bash
# 10-bit radix passes for 17..20-bit key ranges: parity and A/B on C3 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 500 gpurun_out/r10_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread \
   tests/test_gpu_c3.py tests/test_gpu_nfa.py tests/test_gpu_c1.py tests/test_gpu_rules.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/r10_tests.log
for x in 1 0 1; do
SH_RADIX10=$x $S 300 gpurun_out/bench_c3_r$x.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "C3 r10=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3_r$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3_r$x.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3_r$x.log)"
SH_RADIX10=$x $S 300 gpurun_out/bench_c5_r$x.log python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 0 || exit $?
echo "C5 r10=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c5_r$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c5_r$x.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c5_r$x.log)"
done
