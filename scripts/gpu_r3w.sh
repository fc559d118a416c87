#!/bin/bash
# round 3: rule engine with the direct-mapped rule index and the walked runs (keys kernel finds each
# consuming event's run; long runs fall back to the per-event run scan): rule, aggregate, sharding and
# streaming parity, then C5 bench walked vs scanned runs
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_rules.py tests/test_gpu_agg.py tests/test_gpu_shard.py tests/test_gpu_shard_stream.py tests/test_gpu_c3.py -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3w_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3w_tests.log | head -20; tail -40 gpurun_out/r3w_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3w_c5.json 2> gpurun_out/r3w_c5.err || { tail -20 gpurun_out/r3w_c5.err; exit 1; }
SH_RULES_RUNSCAN=1 timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3w_c5_scan.json 2> gpurun_out/r3w_c5_scan.err || { tail -20 gpurun_out/r3w_c5_scan.err; exit 1; }
python -c "
import json
for f in ('r3w_c5', 'r3w_c5_scan'):
    d = json.loads(open('gpurun_out/%s.json' % f).read()); print(f, round(d['ms_per_step'], 3), d['value'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w_prof -o run -- python -u bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3w_prof.json 2> gpurun_out/r3w_prof.err || { tail -20 gpurun_out/r3w_prof.err; exit 1; }
find gpurun_out/r3w_prof -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-140
