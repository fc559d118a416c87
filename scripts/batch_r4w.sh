R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
scripts/gpu.sh bench r4w_c2agg --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 \
&& scripts/gpu.sh bench r4w_c4 --config c4 --steps 1 --warmup 0 \
&& SH_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --master-port 29533 bench.py --gpus 2 --config c2 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r4w_reh_c2.json 2> gpurun_out/r4w_reh_c2.err \
&& tail -c 1500 gpurun_out/r4w_reh_c2.json \
&& SH_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --master-port 29534 bench.py --gpus 2 --config c4 --c4-calls 3000 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/r4w_reh_c4.json 2> gpurun_out/r4w_reh_c4.err \
&& tail -c 2500 gpurun_out/r4w_reh_c4.json
