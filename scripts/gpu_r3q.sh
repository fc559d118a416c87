#!/bin/bash
# round 3: counter block + column-image cache on the push path (C4, snapshot, sharded streaming, fixtures, rules);
# in-lane aggregates of the rise-and-fall kernel (C3 agg parity + bench); C4 full workload again
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_agg.py tests/test_gpu_c3.py tests/test_gpu_snapshot.py tests/test_gpu_c4.py tests/test_gpu_shard_stream.py tests/test_gpu_parity.py tests/test_gpu_nfa.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3q_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3q_tests.log | head -20; tail -40 gpurun_out/r3q_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --agg --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3q_c3agg.json 2> gpurun_out/r3q_c3agg.err || { tail -20 gpurun_out/r3q_c3agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3q_c3agg.json').read()); print('c3 agg', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'])"
timeout -k 10 300 python -u bench.py --agg --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3q_c2agg.json 2> gpurun_out/r3q_c2agg.err || { tail -20 gpurun_out/r3q_c2agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3q_c2agg.json').read()); print('c2 agg', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'])"
SH_HOST_PROF=1 timeout -k 10 600 python -u bench.py --config c4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/r3q_c4.json 2> gpurun_out/r3q_c4.err || { tail -20 gpurun_out/r3q_c4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3q_c4.json').read()); print('c4', round(d['ms_per_step'],1), d['value'])"
grep "sh host profile" gpurun_out/r3q_c4.err | tail -1
