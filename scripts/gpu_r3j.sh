#!/bin/bash
# round 3: full GPU suite after the default-stream fix; C5 sharded rehearsal (2 ranks on one GPU);
# aggregate post-pass after the workgroup reduction (rocprof stats); C2 headline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3j_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3j_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3j_tests.log | head -20; tail -40 gpurun_out/r3j_tests.log; exit 1; }
SH_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --config c5 --gpus 2 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r3j_rehearse_c5.json 2> gpurun_out/r3j_rehearse_c5.err || { tail -20 gpurun_out/r3j_rehearse_c5.err; exit 1; }
cat gpurun_out/r3j_rehearse_c5.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j_agg -o run -- python -u bench.py --agg --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3j_agg.json 2> gpurun_out/r3j_agg.err || { tail -20 gpurun_out/r3j_agg.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3j_agg.json').read()); print('agg', d['ms_per_step'], d['phase_ms'], d['verified_vs_restatement'])"
find gpurun_out/r3j_agg -name "*kernel_stats.csv" | head -1 | xargs head -16 | cut -c1-140
timeout -k 10 300 python -u bench.py --agg --steps 10 --warmup 3 > gpurun_out/r3j_agg_v.json 2> gpurun_out/r3j_agg_v.err || { tail -20 gpurun_out/r3j_agg_v.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3j_agg_v.json').read()); print('agg verified', d['ms_per_step'], d['phase_ms'], d['verified_vs_restatement'])"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3j_c2.json 2> gpurun_out/r3j_c2.err || { tail -20 gpurun_out/r3j_c2.err; exit 1; }
cat gpurun_out/r3j_c2.json
