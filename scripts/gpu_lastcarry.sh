#!/bin/bash
# payload carried by the last radix pass only (SH_SEG_LASTCARRY=1): parity and A/B on C3 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
SH_SEG_LASTCARRY=1 $S 400 gpurun_out/lc_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread \
   tests/test_gpu_c3.py tests/test_gpu_rules.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/lc_tests.log
for x in 1 0 1; do
SH_SEG_LASTCARRY=$x $S 300 gpurun_out/bench_c3_lc$x.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "C3 lc=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3_lc$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3_lc$x.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3_lc$x.log)"
SH_SEG_LASTCARRY=$x $S 300 gpurun_out/bench_c5_lc$x.log python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 0 || exit $?
echo "C5 lc=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c5_lc$x.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c5_lc$x.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c5_lc$x.log)"
done
