B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r4z_ru6 --config c2 --steps 20 --warmup 3 --cpu-sample 0 \
&& SH_BK_RU=4 scripts/gpu.sh bench r4z_ru4 $B \
&& scripts/gpu.sh bench r4z_ru6b $B \
&& SH_BK_RU=4 scripts/gpu.sh bench r4z_ru4b $B \
&& scripts/gpu.sh test r4z_bucket tests/test_gpu_bucket.py tests/test_gpu_c3.py tests/test_gpu_agg.py \
&& scripts/gpu.sh prof r4z_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify
