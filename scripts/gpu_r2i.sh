#!/bin/bash
# C2 tuning: scatter prefetch (occupancy variants) x emit (row- vs event-parallel), matcher phase clocks
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 300 gpurun_out/bucket_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py tests/test_range_partition.py || exit $?
tail -n 2 gpurun_out/bucket_tests.log
for sc in 1 4; do for em in 0 1; do
  SH_BK_SCAT=$sc SH_BK_EMIT=$em $S 200 gpurun_out/var_${sc}_${em}.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-verify || exit $?
  echo "scat=$sc emit=$em $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_${sc}_${em}.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/var_${sc}_${em}.log)"
done; done
SH_BK_PROFILE=1 $S 200 gpurun_out/bench_phase.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_phase.log | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
