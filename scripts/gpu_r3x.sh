#!/bin/bash
# round 3: radix scatter with 16 KB LDS staging (8-byte columns in two halves) and 4 workgroups per CU; rule image
# without the index-implied terms (two 1024-thread workgroups per CU): C5 (A/B) and C3 benches with rocprof kernel
# stats, then the whole -m gpu suite
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3x_c5.json 2> gpurun_out/r3x_c5.err || { tail -20 gpurun_out/r3x_c5.err; exit 1; }
SH_RULES_IXTERM=1 SH_RULES_OCC2=0 timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3x_c5_old.json 2> gpurun_out/r3x_c5_old.err || { tail -20 gpurun_out/r3x_c5_old.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3x_c3.json 2> gpurun_out/r3x_c3.err || { tail -20 gpurun_out/r3x_c3.err; exit 1; }
python -c "
import json
for f in ('r3x_c5', 'r3x_c5_old', 'r3x_c3'):
    d = json.loads(open('gpurun_out/%s.json' % f).read()); print(f, round(d['ms_per_step'], 3), d['value'], d['roofline']['frac'], d.get('verified_vs_restatement'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3x_prof5 -o run -- python -u bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/r3x_prof5.json 2> gpurun_out/r3x_prof5.err || { tail -20 gpurun_out/r3x_prof5.err; exit 1; }
find gpurun_out/r3x_prof5 -name "*kernel_stats.csv" | head -1 | xargs head -4 | cut -c1-60,180-260
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3x_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3x_tests.log | head -20; tail -40 gpurun_out/r3x_tests.log; exit 1; }
exit 0
