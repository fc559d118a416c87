A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh pmc r4v_c5f FETCH_SIZE --config c5 $A \
&& scripts/gpu.sh pmc r4v_c5w WRITE_SIZE --config c5 $A \
&& scripts/gpu.sh bench r4v_c2agg --config c2 --agg --steps 10 --warmup 2 \
&& scripts/gpu.sh bench r4v_c2agg_raw --config c2 --agg --layout raw --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
&& SH_BK_AGGC=1 SH_BK_PROFILE=1 scripts/gpu.sh bench r4v_c2aggc --config c2 --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh prof r4v_c2aggprof --config c2 --agg --steps 3 --warmup 1 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh pmc r4v_c2af FETCH_SIZE --config c2 --agg $A \
&& scripts/gpu.sh pmc r4v_c2aw WRITE_SIZE --config c2 --agg $A
