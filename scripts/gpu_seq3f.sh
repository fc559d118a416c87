#!/bin/bash
# k_seq3 float fast path: C3 parity, A/B against the generic kernel
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S 300 gpurun_out/c3_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c3.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/c3_tests.log
for g in 0 1 0; do
if [ $g = 1 ]; then export SH_SEQ3_GENERIC=1; else unset SH_SEQ3_GENERIC; fi
$S 300 gpurun_out/bench_c3_g$g.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "C3 generic=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3_g$g.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3_g$g.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3_g$g.log)"
done
