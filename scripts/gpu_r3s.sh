#!/bin/bash
# round 3: C5 rule scan with two workgroups per CU (parity + bench + kernel stats); C3 segment with 10-bit digits (A/B)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rules.py tests/test_gpu_agg.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3s_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3s_tests.log | head -20; tail -40 gpurun_out/r3s_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3s_c5.json 2> gpurun_out/r3s_c5.err || { tail -20 gpurun_out/r3s_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3s_c5.json').read()); print('c5', round(d['ms_per_step'],3), d['phase_ms'], d['verified_vs_restatement'])"
for v in "SH_RADIX10=0" "SH_RADIX10=1"; do
  env $v timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/r3s_c3.json 2> gpurun_out/r3s_c3.err || { tail -20 gpurun_out/r3s_c3.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3s_c3.json').read()); print('c3 $v', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_c5prof -o run -- python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3s_c5prof.json 2> gpurun_out/r3s_c5prof.err || { tail -20 gpurun_out/r3s_c5prof.err; exit 1; }
find gpurun_out/r3s_c5prof -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-140
