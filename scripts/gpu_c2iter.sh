#!/bin/bash
# C2 iteration: bucketed-engine parity tests, verified bench, matcher phase clocks, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 300 gpurun_out/bucket_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py || exit $?
tail -n 1 gpurun_out/bucket_tests.log
grep -E "FAIL|Error" gpurun_out/bucket_tests.log | head -5
$S 200 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench.log)"
SH_BK_PROFILE=1 $S 200 gpurun_out/bench_phase.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_phase.log | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
python scripts/show_prof.py gpurun_out/prof | head -6
