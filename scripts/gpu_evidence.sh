#!/bin/bash
# GPU evidence for the round: smoke, GPU parity tests, bench, kernel-trace stats,
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic figure.
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmc_f gpurun_out/pmc_w
S=scripts/gpu_step.sh
$S 240 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -n 2 gpurun_out/smoke.log
$S 900 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 3 gpurun_out/gpu_tests.log
$S 600 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 2 || exit $?
tail -n 2 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o f -- \
    python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_f/log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o w -- \
    python bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/pmc_w/log 2>&1 || exit $?
python scripts/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w 1 100000000 10000 gpurun_out/pmc_c2.json c2
