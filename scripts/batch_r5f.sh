B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5i_w64 --config c2 --steps 20 --warmup 3 \
&& SH_BK_WARM=0 scripts/gpu.sh bench r5i_w0 $B \
&& scripts/gpu.sh bench r5i_w64b $B \
&& SH_BK_WARM=0 scripts/gpu.sh bench r5i_w0b $B \
&& scripts/gpu.sh pmc r5i_c2f FETCH_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r5i_c2w WRITE_SIZE --config c2 $A \
&& scripts/gpu.sh test r5i_bucket tests/test_gpu_bucket.py tests/test_gpu_c3.py
