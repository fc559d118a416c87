#!/bin/bash
# C4 on the GPU: parity tests, a probe bench at 1M users, the full 10M-user bench
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
S=scripts/gpu_step.sh
$S 400 gpurun_out/c4/tests.log python -u -m pytest tests/test_gpu_c4.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 5 gpurun_out/c4/tests.log
grep -q " passed" gpurun_out/c4/tests.log || exit 1
timeout -k 10 300 python -u bench.py --config c4 --keys 1000000 --seconds 20 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4/probe.log 2>&1 || { tail -5 gpurun_out/c4/probe.log; exit 1; }
tail -n 3 gpurun_out/c4/probe.log
timeout -k 10 700 python -u bench.py --config c4 --steps 1 --warmup 0 --cpu-sample 1000000 > gpurun_out/c4/bench.log 2>&1 || { tail -5 gpurun_out/c4/bench.log; exit 1; }
tail -n 3 gpurun_out/c4/bench.log
