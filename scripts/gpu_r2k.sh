#!/bin/bash
# C2: emit super-block size (G = 1, 2, 4) x scatter occupancy; kb-ballot ranking
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
for g in 2 4 1; do
  SH_BK_EMIT_G=$g $S 300 gpurun_out/bucket_tests_$g.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py || exit $?
  tail -n 1 gpurun_out/bucket_tests_$g.log
done
for sc in 1 4; do for g in 1 2 4; do
  SH_BK_SCAT=$sc SH_BK_EMIT_G=$g $S 200 gpurun_out/var_${sc}_${g}.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-verify || exit $?
  echo "scat=$sc G=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_${sc}_${g}.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/var_${sc}_${g}.log)"
done; done
SH_BK_PROFILE=1 $S 200 gpurun_out/bench_phase.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_phase.log | tail -1
