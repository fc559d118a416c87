#!/bin/bash
# round 3: the whole -m gpu suite and smoke() after the radix scatter's padding-tile fix, then C5 / C3 benches
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3y_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3y_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3y_tests.log | head -20; tail -40 gpurun_out/r3y_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3y_smoke.log 2>&1 || { tail -20 gpurun_out/r3y_smoke.log; exit 1; }
tail -1 gpurun_out/r3y_smoke.log
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3y_c5.json 2> gpurun_out/r3y_c5.err || { tail -20 gpurun_out/r3y_c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r3y_c2.json 2> gpurun_out/r3y_c2.err || { tail -20 gpurun_out/r3y_c2.err; exit 1; }
python -c "
import json
for f in ('r3y_c5', 'r3y_c2'):
    d = json.loads(open('gpurun_out/%s.json' % f).read()); print(f, round(d['ms_per_step'], 3), d['value'], d['roofline']['frac'], d.get('verified_vs_restatement'))"
