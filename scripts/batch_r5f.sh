timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5j_smoke.log 2>&1 && tail -1 gpurun_out/r5j_smoke.log \
&& scripts/gpu.sh bench r5j_c2 --config c2 --steps 20 --warmup 3 \
&& scripts/gpu.sh bench r5j_c3 --config c3 --steps 10 --warmup 2 \
&& scripts/gpu.sh prof r5j_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh test r5j_t tests/test_gpu_bucket.py tests/test_gpu_c3.py tests/test_gpu_agg.py tests/test_gpu_shard.py tests/test_gpu_parity.py
