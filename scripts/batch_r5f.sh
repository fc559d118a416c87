B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5h_m1 --config c2 --steps 20 --warmup 3 --cpu-sample 0 \
&& SH_BK_MWARM=0 scripts/gpu.sh bench r5h_m0 $B \
&& scripts/gpu.sh bench r5h_m1b $B \
&& SH_BK_MWARM=0 scripts/gpu.sh bench r5h_m0b $B \
&& scripts/gpu.sh test r5h_bucket tests/test_gpu_bucket.py tests/test_gpu_agg.py tests/test_gpu_shard.py
