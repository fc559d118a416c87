#!/bin/bash
# round 3: sharded C2/C3/C5 (virtual ranks), rule run ids, then a 2-rank gloo rehearsal of the sharded bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_rules.py tests/test_gpu_c3.py tests/test_gpu_snapshot.py tests/test_range_partition.py tests/test_gpu_nfa.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -5 gpurun_out/r3a_tests.log
for c in c3 c5; do
  SH_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --config $c --gpus 2 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r3a_rehearse_$c.json 2> gpurun_out/r3a_rehearse_$c.err || { tail -20 gpurun_out/r3a_rehearse_$c.err; exit 1; }
  cat gpurun_out/r3a_rehearse_$c.json
done
