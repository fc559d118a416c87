#!/bin/bash
# C3 iteration (segment scatter + ordered placement): general-engine / C3 / window parity tests,
# verified C3 bench, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof3
S=scripts/gpu_step.sh
$S 500 gpurun_out/c3_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread \
   tests/test_gpu_c3.py tests/test_gpu_nfa.py tests/test_gpu_c1.py tests/test_gpu_parity.py -p no:cacheprovider || exit $?
tail -n 1 gpurun_out/c3_tests.log
grep -E "FAIL|Error" gpurun_out/c3_tests.log | head -5
$S 300 gpurun_out/bench_c3.log python -u bench.py --config c3 --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c3.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench_c3.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench_c3.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- \
    python bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof3/bench_prof.log 2>&1
echo "prof rc=$?"
python scripts/show_prof.py gpurun_out/prof3 | head -12
