#!/bin/bash
# round 3: key-sharded C4 (virtual ranks) + regressions of the timer path; C5 sharded-share probe
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard_stream.py tests/test_gpu_c4.py tests/test_gpu_nfa.py tests/test_gpu_snapshot.py tests/test_abi.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3f_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3f_tests.log | head -20; tail -40 gpurun_out/r3f_tests.log; exit 1; }
timeout -k 10 400 python -u scripts/c5_shard_probe.py > gpurun_out/r3f_c5probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/r3f_c5probe.log | grep -v amdgpu.ids
