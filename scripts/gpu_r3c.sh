#!/bin/bash
# round 3: aggregate post-pass tests, restore rollback, rehearsal, C2 profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py tests/test_gpu_snapshot.py tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/r3c_tests.log | head -60
[ $rc -ne 0 ] && { tail -40 gpurun_out/r3c_tests.log; exit 1; }
SH_BK_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3c_c2_prof.json 2> gpurun_out/r3c_c2_prof.err || { tail -20 gpurun_out/r3c_c2_prof.err; exit 1; }
grep "clock ticks" gpurun_out/r3c_c2_prof.err | tail -1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof -o c2 -- python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3c_c2.json 2> gpurun_out/r3c_c2.err || { tail -20 gpurun_out/r3c_c2.err; exit 1; }
cat gpurun_out/r3c_c2.json
find gpurun_out/r3c_prof -name "*kernel_stats.csv" | head -1 | xargs head -14
for c in c3 c5; do
  SH_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --config $c --gpus 2 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r3c_rehearse_$c.json 2> gpurun_out/r3c_rehearse_$c.err || { tail -20 gpurun_out/r3c_rehearse_$c.err; exit 1; }
  cat gpurun_out/r3c_rehearse_$c.json
done
