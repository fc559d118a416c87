#!/bin/bash
# rehearsal of the key-sharded C2 step with 2 and 4 ranks sharing the one GPU
# (gloo through host memory: RCCL refuses duplicate devices)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
SH_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 2 --warmup 1 --events 20000000 \
    > gpurun_out/rehearse$n.log 2>&1
rc=$?
echo "n=$n rc=$rc"
grep '^{' gpurun_out/rehearse$n.log | cut -c1-300
grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/rehearse$n.log
[ $rc -ne 0 ] && { grep -A3 "Error\|Traceback" gpurun_out/rehearse$n.log | head -20; exit $rc; }
done
exit 0
