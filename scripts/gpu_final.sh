#!/bin/bash
# Round-end evidence: smoke, every -m gpu test, the default bench (verified + CPU
# baseline), kernel stats, calibrated PMC traffic of the C2 step
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 240 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -n 2 gpurun_out/smoke.log
$S 700 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 3 gpurun_out/gpu_tests.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_cal_$c -o cal -- python scripts/pmc_calib.py > gpurun_out/pmc_cal_$c.log 2>&1 || { echo "cal $c failed"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_c2_$c -o c2 -- python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_c2_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python scripts/pmc_traffic.py gpurun_out/pmc_c2_FETCH_SIZE gpurun_out/pmc_c2_WRITE_SIZE 1 100000000 10000 gpurun_out/pmc_c2.json c2 --calib gpurun_out/pmc_cal_FETCH_SIZE gpurun_out/pmc_cal_WRITE_SIZE 2147483648 || exit $?
mkdir -p profiles && cp gpurun_out/pmc_c2.json profiles/pmc_c2.json
$S 400 gpurun_out/bench_c2.log python -u bench.py --steps 10 --warmup 2 || exit $?
grep '^{' gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
$S 300 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 5 --warmup 1 || exit $?
grep '^{' gpurun_out/bench_c3.log | cut -c1-300
mkdir -p gpurun_out/prof3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- \
    python bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof3/bench_prof.log 2>&1
echo "prof3 rc=$?"
