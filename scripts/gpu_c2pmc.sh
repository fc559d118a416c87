#!/bin/bash
# C2: parity tests, verified bench, kernel stats, calibrated PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 300 gpurun_out/bucket_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py || exit $?
tail -n 1 gpurun_out/bucket_tests.log
$S 200 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_cal_$c -o cal -- python scripts/pmc_calib.py > gpurun_out/pmc_cal_$c.log 2>&1 || { echo "cal $c failed"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_c2_$c -o c2 -- python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_c2_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python scripts/pmc_traffic.py gpurun_out/pmc_c2_FETCH_SIZE gpurun_out/pmc_c2_WRITE_SIZE 1 100000000 10000 gpurun_out/pmc_c2.json c2 --calib gpurun_out/pmc_cal_FETCH_SIZE gpurun_out/pmc_cal_WRITE_SIZE 2147483648
