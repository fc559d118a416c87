B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5f_w1 --config c2 --steps 20 --warmup 3 --cpu-sample 0 \
&& SH_BK_WARM=0 scripts/gpu.sh bench r5f_w0 $B \
&& scripts/gpu.sh bench r5f_w1b $B \
&& SH_BK_WARM=0 scripts/gpu.sh bench r5f_w0b $B \
&& scripts/gpu.sh test r5f_bucket tests/test_gpu_bucket.py tests/test_gpu_agg.py
