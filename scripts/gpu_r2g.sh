#!/bin/bash
# C2: wave-contiguous scatter ranking + arrival-order match-stream writes
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
scripts/gpu_step.sh 600 gpurun_out/bucket_tests.log $T tests/test_gpu_bucket.py tests/test_gpu_shard.py || exit $?
grep -E "passed|failed" gpurun_out/bucket_tests.log | tail -2
SH_BK_PROFILE=1 scripts/gpu_step.sh 300 gpurun_out/bench_bucket_prof.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_bucket_prof.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof/bench_prof.log | cut -c1-300
