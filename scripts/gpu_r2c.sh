#!/bin/bash
# C2 bucketed engine perf + sharded path kernels and virtual-rank step
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
scripts/gpu_step.sh 600 gpurun_out/bucket_tests.log $T tests/test_gpu_bucket.py || exit $?
grep -E "passed|failed" gpurun_out/bucket_tests.log | tail -2
scripts/gpu_step.sh 600 gpurun_out/shard_tests.log $T tests/test_gpu_shard.py || exit $?
grep -E "passed|failed" gpurun_out/shard_tests.log | tail -2
SH_BK_PROFILE=1 scripts/gpu_step.sh 300 gpurun_out/bench_bucket_prof.log python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify || exit $?
grep "shb_match clock" gpurun_out/bench_bucket_prof.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof/bench_prof.log | cut -c1-400
scripts/gpu_step.sh 600 gpurun_out/c1_tests.log $T tests/test_gpu_c1.py || exit $?
grep -E "passed|failed" gpurun_out/c1_tests.log | tail -2
scripts/gpu_step.sh 600 gpurun_out/bench_c1.log python -u bench.py --config c1 --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/bench_c1.log | cut -c1-600
scripts/gpu_step.sh 900 gpurun_out/c4_tests.log $T tests/test_gpu_c4.py || exit $?
grep -E "passed|failed" gpurun_out/c4_tests.log | tail -2
mkdir -p gpurun_out/prof_c4
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- \
    python bench.py --config c4 --steps 1 --warmup 0 --cpu-sample 0 --c4-calls 3000 > gpurun_out/prof_c4/bench_c4.log 2>&1
echo "c4 prof rc=$?"
grep '^{' gpurun_out/prof_c4/bench_c4.log | cut -c1-400
