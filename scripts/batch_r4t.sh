scripts/gpu.sh test r4t_tests tests/test_gpu_bucket.py tests/test_gpu_agg.py tests/test_abi.py \
&& scripts/gpu.sh bench r4t_c2 --config c2 --steps 20 --warmup 3 \
&& scripts/gpu.sh bench r4t_c2raw --config c2 --steps 20 --warmup 3 --cpu-sample 0 --layout raw \
&& scripts/gpu.sh bench r4t_c2b --config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh prof r4t_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify
