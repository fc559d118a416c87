#!/bin/bash
# round 3: sharded C5 probe (virtual ranks, full size), C2 typed-column emit A/B, aggregate post-pass kernel stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u scripts/c5_shard_probe2.py > gpurun_out/r3g_c5probe2.log 2>&1; echo "probe2 rc=$?"; grep -v amdgpu.ids gpurun_out/r3g_c5probe2.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g_cols -o run -- python -u bench.py --columns --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3g_cols.json 2> gpurun_out/r3g_cols.err || { tail -20 gpurun_out/r3g_cols.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3g_cols.json').read()); print('cols', d['ms_per_step'], d['phase_ms'], d['verified_vs_restatement'])"
find gpurun_out/r3g_cols -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g_agg -o run -- python -u bench.py --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3g_agg.json 2> gpurun_out/r3g_agg.err || { tail -20 gpurun_out/r3g_agg.err; exit 1; }
find gpurun_out/r3g_agg -name "*kernel_stats.csv" | head -1 | xargs head -16 | cut -c1-140
