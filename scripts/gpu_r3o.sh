#!/bin/bash
# round 3: C3 (no key-state reset, one-line record gathers) parity + bench; general-engine push path with fewer
# syncs (C4, snapshot, sharded streaming, fixtures); C5 rule scan over an LDS image of the rule set (A/B);
# C4 on the full SURVEY 8d workload
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_agg.py tests/test_gpu_snapshot.py tests/test_gpu_c4.py tests/test_gpu_shard_stream.py tests/test_gpu_parity.py tests/test_gpu_rules.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3o_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3o_tests.log | head -20; tail -40 gpurun_out/r3o_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r3o_c3.json 2> gpurun_out/r3o_c3.err || { tail -20 gpurun_out/r3o_c3.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3o_c3.json').read()); print('c3', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3o_c5.json 2> gpurun_out/r3o_c5.err || { tail -20 gpurun_out/r3o_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3o_c5.json').read()); print('c5', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'])"
SH_RULES_IMG=0 timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/r3o_c5b.json 2> gpurun_out/r3o_c5b.err || { tail -20 gpurun_out/r3o_c5b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3o_c5b.json').read()); print('c5 no image', round(d['ms_per_step'],3), d['phase_ms'])"
SH_HOST_PROF=1 timeout -k 10 900 python -u bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/r3o_c4.json 2> gpurun_out/r3o_c4.err || { tail -20 gpurun_out/r3o_c4.err; exit 1; }
cat gpurun_out/r3o_c4.json
grep "sh host profile" gpurun_out/r3o_c4.err | tail -1
