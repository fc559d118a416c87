#!/bin/bash
# round 3: List outputs on the GPU (fixtures, random apps, snapshot), sharded C5 probe, C2 typed-column A/B, agg post-pass stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_snapshot.py tests/test_rate_limit.py tests/test_gpu_parity.py tests/test_gpu_nfa.py tests/test_abi.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3h_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3h_tests.log | head -20; tail -40 gpurun_out/r3h_tests.log; exit 1; }
timeout -k 10 500 python -u scripts/c5_shard_probe2.py > gpurun_out/r3h_c5probe2.log 2>&1; echo "probe2 rc=$?"; grep -v amdgpu.ids gpurun_out/r3h_c5probe2.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h_cols -o run -- python -u bench.py --columns --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3h_cols.json 2> gpurun_out/r3h_cols.err || { tail -20 gpurun_out/r3h_cols.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3h_cols.json').read()); print('cols', d['ms_per_step'], d['phase_ms'], d['verified_vs_restatement'])"
find gpurun_out/r3h_cols -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h_agg -o run -- python -u bench.py --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3h_agg.json 2> gpurun_out/r3h_agg.err || { tail -20 gpurun_out/r3h_agg.err; exit 1; }
find gpurun_out/r3h_agg -name "*kernel_stats.csv" | head -1 | xargs head -16 | cut -c1-140
