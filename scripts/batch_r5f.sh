A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5g_c2 --config c2 --steps 20 --warmup 3 \
&& scripts/gpu.sh bench r5g_c3 --config c3 --steps 10 --warmup 2 \
&& SH_BK_WARM=0 scripts/gpu.sh bench r5g_c3w0 --config c3 --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh prof r5g_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh pmc r5g_c2f FETCH_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r5g_c2w WRITE_SIZE --config c2 $A \
&& timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g_smoke.log 2>&1 && tail -1 gpurun_out/r5g_smoke.log \
&& scripts/gpu.sh test r5g_all tests -m gpu -rs
