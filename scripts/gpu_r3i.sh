#!/bin/bash
# round 3: C2 dynamic walk parity + A/B; selection features on the GPU (Lists, all-per-N, group by, snapshot);
# sharded C5 probe; C2 typed-column A/B; aggregate post-pass stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_bucket.py tests/test_group_by.py tests/test_gpu_snapshot.py tests/test_rate_limit.py tests/test_gpu_parity.py tests/test_gpu_nfa.py tests/test_abi.py -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3i_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3i_tests.log | head -20; tail -40 gpurun_out/r3i_tests.log; exit 1; }
for d in 0 1; do
  SH_BK_DYN=$d timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r3i_c2_dyn$d.json 2> gpurun_out/r3i_c2_dyn$d.err || { tail -20 gpurun_out/r3i_c2_dyn$d.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3i_c2_dyn$d.json').read()); print('dyn$d', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, d['verified_vs_restatement'])"
done
SH_BK_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3i_c2_prof.json 2> gpurun_out/r3i_c2_prof.err || { tail -20 gpurun_out/r3i_c2_prof.err; exit 1; }
grep "clock ticks" gpurun_out/r3i_c2_prof.err | tail -1
timeout -k 10 500 python -u scripts/c5_shard_probe2.py > gpurun_out/r3i_c5probe2.log 2>&1; echo "probe2 rc=$?"; grep -v amdgpu.ids gpurun_out/r3i_c5probe2.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_cols -o run -- python -u bench.py --columns --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3i_cols.json 2> gpurun_out/r3i_cols.err || { tail -20 gpurun_out/r3i_cols.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3i_cols.json').read()); print('cols', d['ms_per_step'], d['phase_ms'], d['verified_vs_restatement'])"
find gpurun_out/r3i_cols -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_agg -o run -- python -u bench.py --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3i_agg.json 2> gpurun_out/r3i_agg.err || { tail -20 gpurun_out/r3i_agg.err; exit 1; }
find gpurun_out/r3i_agg -name "*kernel_stats.csv" | head -1 | xargs head -16 | cut -c1-140
