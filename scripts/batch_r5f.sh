B="--config c3 --steps 10 --warmup 2 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5k_w1 --config c3 --steps 10 --warmup 2 --cpu-sample 0 \
&& SH_S3B_WARM=0 scripts/gpu.sh bench r5k_w0 $B \
&& scripts/gpu.sh bench r5k_w1b $B \
&& SH_S3B_WARM=0 scripts/gpu.sh bench r5k_w0b $B \
&& scripts/gpu.sh test r5k_t tests/test_gpu_c3.py tests/test_gpu_nfa.py
