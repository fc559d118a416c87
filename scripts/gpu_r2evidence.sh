#!/bin/bash
# Round-2 evidence: C3 verified bench + kernel stats, C1 bench, C2 PMC traffic (calibrated)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c3
S=scripts/gpu_step.sh
$S 400 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 1000000 || exit $?
grep '^{' gpurun_out/bench_c3.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof_c3/bench.log 2>&1 || exit $?
echo "c3 prof ok"
$S 300 gpurun_out/bench_c1.log python -u bench.py --config c1 --steps 5 --warmup 1 || exit $?
grep '^{' gpurun_out/bench_c1.log | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_cal_$c -o cal -- python scripts/pmc_calib.py > gpurun_out/pmc_cal_$c.log 2>&1 || { echo "cal $c failed"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_c2_$c -o c2 -- python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_c2_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python scripts/pmc_traffic.py gpurun_out/pmc_c2_FETCH_SIZE gpurun_out/pmc_c2_WRITE_SIZE 1 100000000 10000 gpurun_out/pmc_c2.json c2 --calib gpurun_out/pmc_cal_FETCH_SIZE gpurun_out/pmc_cal_WRITE_SIZE 2147483648
echo "pmc rc=$?"
