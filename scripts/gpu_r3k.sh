#!/bin/bash
# round 3: C3 with the LDS-staged sequence kernel and no timestamp carry (parity + bench + kernel stats);
# C5 bench with the >=1M-event CPU baseline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_agg.py tests/test_gpu_nfa.py tests/test_rate_limit.py tests/test_gpu_rules.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3k_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3k_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3k_tests.log | head -20; tail -40 gpurun_out/r3k_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r3k_c3.json 2> gpurun_out/r3k_c3.err || { tail -20 gpurun_out/r3k_c3.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3k_c3.json').read()); print('c3', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'], d['roofline']['frac'])"
SH_S3_STAGED=0 timeout -k 10 400 python -u bench.py --config c3 --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/r3k_c3_old.json 2> gpurun_out/r3k_c3_old.err || { tail -20 gpurun_out/r3k_c3_old.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3k_c3_old.json').read()); print('c3 unstaged', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3k_c3prof -o run -- python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3k_c3prof.json 2> gpurun_out/r3k_c3prof.err || { tail -20 gpurun_out/r3k_c3prof.err; exit 1; }
find gpurun_out/r3k_c3prof -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-140
timeout -k 10 400 python -u bench.py --config c3 --agg --steps 5 --warmup 2 > gpurun_out/r3k_c3agg.json 2> gpurun_out/r3k_c3agg.err || { tail -20 gpurun_out/r3k_c3agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3k_c3agg.json').read()); print('c3 agg', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'])"
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/r3k_c5.json 2> gpurun_out/r3k_c5.err || { tail -20 gpurun_out/r3k_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3k_c5.json').read()); print('c5', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'], d['cpu_baseline'])"
timeout -k 10 300 python -u bench.py --columns --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r3k_cols.json 2> gpurun_out/r3k_cols.err || { tail -20 gpurun_out/r3k_cols.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3k_cols.json').read()); print('c2 cols', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'])"
