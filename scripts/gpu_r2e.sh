#!/bin/bash
# C2 (word-flag fast walk, D=10) + C3 (blocked k_seq3, used columns only): parity + bench + traces
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/prof_c3
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
scripts/gpu_step.sh 600 gpurun_out/bucket_tests.log $T tests/test_gpu_bucket.py || exit $?
grep -E "passed|failed" gpurun_out/bucket_tests.log | tail -2
scripts/gpu_step.sh 900 gpurun_out/c3_tests.log $T tests/test_gpu_c3.py tests/test_gpu_nfa.py || exit $?
grep -E "passed|failed" gpurun_out/c3_tests.log | tail -2
SH_BK_PROFILE=1 scripts/gpu_step.sh 300 gpurun_out/bench_bucket_prof.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_bucket_prof.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof/bench_prof.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof_c3/bench.log 2>&1
echo "c3 prof rc=$?"
grep '^{' gpurun_out/prof_c3/bench.log | cut -c1-300
# PMC: calibration streams, then the C2 step (separate passes per counter)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_cal_$c -o cal -- python scripts/pmc_calib.py > gpurun_out/pmc_cal_$c.log 2>&1 || { echo "cal $c failed"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_c2_$c -o c2 -- python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_c2_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo "pmc done"
