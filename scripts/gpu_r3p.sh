#!/bin/bash
# round 3 evidence: the whole -m gpu suite, smoke(), the default bench line (C2) with its rocprof kernel summary,
# and the aggregate variants of C2 / C3
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3p_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3p_tests.log | head -20; tail -40 gpurun_out/r3p_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3p_smoke.log 2>&1 || { tail -20 gpurun_out/r3p_smoke.log; exit 1; }
tail -3 gpurun_out/r3p_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err || { tail -20 gpurun_out/r3p_bench.err; exit 1; }
cat gpurun_out/r3p_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof -o run -- python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3p_prof.json 2> gpurun_out/r3p_prof.err || { tail -20 gpurun_out/r3p_prof.err; exit 1; }
find gpurun_out/r3p_prof -name "*kernel_stats.csv" | head -1 | xargs head -10 | cut -c1-140
timeout -k 10 300 python -u bench.py --agg --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3p_c2agg.json 2> gpurun_out/r3p_c2agg.err || { tail -20 gpurun_out/r3p_c2agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3p_c2agg.json').read()); print('c2 agg', round(d['ms_per_step'],3), d['verified_vs_restatement'])"
timeout -k 10 300 python -u bench.py --config c3 --agg --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3p_c3agg.json 2> gpurun_out/r3p_c3agg.err || { tail -20 gpurun_out/r3p_c3agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3p_c3agg.json').read()); print('c3 agg', round(d['ms_per_step'],3), d['verified_vs_restatement'])"
