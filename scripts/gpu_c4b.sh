#!/bin/bash
# C4 after pinned staging: parity (C4 + general engine), 200k-user probe, kernel
# stats of the first 600 calls at 10M users
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4b
S=scripts/gpu_step.sh
$S 500 gpurun_out/c4b/tests.log python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_nfa.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 2 gpurun_out/c4b/tests.log
grep -q " passed" gpurun_out/c4b/tests.log && ! grep -q " failed" gpurun_out/c4b/tests.log || exit 1
timeout -k 10 200 python -u bench.py --config c4 --keys 200000 --seconds 10 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4b/probe.log 2>&1 || { tail -5 gpurun_out/c4b/probe.log; exit 1; }
grep "^{" gpurun_out/c4b/probe.log | cut -c1-330
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4b/prof -o c4 -- \
    python -u bench.py --config c4 --c4-calls 600 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4b/prof.log 2>&1 || { tail -5 gpurun_out/c4b/prof.log; exit 1; }
grep "^{" gpurun_out/c4b/prof.log | cut -c1-330
