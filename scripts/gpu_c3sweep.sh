#!/bin/bash
# k_seq3 load-block sweep (SH_S3_U) on C3 + C5 with the new radix scatter
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 300 gpurun_out/c3_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c3.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/c3_tests.log
$S 300 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "U=8 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3.log)"
for u in 4 16; do
SH_S3_U=$u $S 300 gpurun_out/bench_c3_u$u.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "U=$u $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3_u$u.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3_u$u.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3_u$u.log)"
done
$S 300 gpurun_out/bench_c5.log python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 0 || exit $?
echo "C5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c5.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c5.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c5.log)"
