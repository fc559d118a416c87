#!/bin/bash
# round 3: C3 with the round-robin LDS-staged sequence kernel + compact records (parity, bench, A/B, kernel
# stats); C5 with the LDS rule index (bench with the >=1M-event CPU baseline); C2 typed-column A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_agg.py tests/test_gpu_rules.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3m_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3m_tests.log | head -20; tail -40 gpurun_out/r3m_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r3m_c3.json 2> gpurun_out/r3m_c3.err || { tail -20 gpurun_out/r3m_c3.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3m_c3.json').read()); print('c3', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'], d['roofline']['frac'], d['cpu_baseline'])"
for v in "SH_S3_COMPACT=0" "SH_S3_STAGED=0"; do
  env $v timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/r3m_c3_ab.json 2> gpurun_out/r3m_c3_ab.err || { tail -20 gpurun_out/r3m_c3_ab.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3m_c3_ab.json').read()); print('c3 $v', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m_c3prof -o run -- python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3m_c3prof.json 2> gpurun_out/r3m_c3prof.err || { tail -20 gpurun_out/r3m_c3prof.err; exit 1; }
find gpurun_out/r3m_c3prof -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-140
timeout -k 10 400 python -u bench.py --config c3 --agg --steps 5 --warmup 2 > gpurun_out/r3m_c3agg.json 2> gpurun_out/r3m_c3agg.err || { tail -20 gpurun_out/r3m_c3agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3m_c3agg.json').read()); print('c3 agg', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'])"
timeout -k 10 300 python -u bench.py --columns --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r3m_cols.json 2> gpurun_out/r3m_cols.err || { tail -20 gpurun_out/r3m_cols.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3m_cols.json').read()); print('c2 cols', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'])"
timeout -k 10 700 python -u bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/r3m_c5.json 2> gpurun_out/r3m_c5.err || { tail -20 gpurun_out/r3m_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3m_c5.json').read()); print('c5', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'], d['cpu_baseline'])"
