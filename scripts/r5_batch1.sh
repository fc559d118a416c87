# round 5: C5 live-bitmap check (verified line + rule tests), C3 / C5 per-rank sizes,
# a 2-rank weak-scaling rehearsal of C2 on one GPU
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b1
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 > $O/c5.json 2> $O/c5.log || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rules.py > $O/rules.log 2>&1 || exit 1
SH_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 2 --config c2 --steps 5 --warmup 2 --cpu-sample 0 > $O/weak_c2_2r.json 2> $O/weak_c2_2r.log || exit 1
SCALE_CFGS="c3 c5" bash scripts/scale_predict.sh
