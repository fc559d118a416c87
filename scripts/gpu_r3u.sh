#!/bin/bash
# round 3: one staging copy and one row copy per streaming call (streaming-path parity: C4, snapshot, fixtures, random
# apps, sharded streaming, selection features); C5 with the whole rule image; C4 full workload
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_snapshot.py tests/test_gpu_parity.py tests/test_gpu_nfa.py tests/test_gpu_shard_stream.py tests/test_rate_limit.py tests/test_group_by.py tests/test_gpu_rules.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3u_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3u_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3u_tests.log | head -20; tail -40 gpurun_out/r3u_tests.log; exit 1; }
SH_HOST_PROF=1 timeout -k 10 600 python -u bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/r3u_c4.json 2> gpurun_out/r3u_c4.err || { tail -20 gpurun_out/r3u_c4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3u_c4.json').read()); print('c4', round(d['ms_per_step'],1), d['value'], d['cpu_baseline']['value'])"
grep "sh host profile" gpurun_out/r3u_c4.err | tail -1
