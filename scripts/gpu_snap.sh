#!/bin/bash
# snapshot/restore GPU tests, bucketed-engine parity, C2 bench
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 400 gpurun_out/snap_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_snapshot.py || exit $?
tail -n 1 gpurun_out/snap_tests.log
grep -E "^FAILED|Error|assert" gpurun_out/snap_tests.log | head -8
$S 300 gpurun_out/bucket_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py -k "c2_bucket_vs_oracle" || exit $?
tail -n 1 gpurun_out/bucket_tests.log
$S 200 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/bench.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/bench.log)"
