A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
SH_SPARSE_XCD=1 scripts/gpu.sh bench r4x_c5x1 --config c5 --steps 5 --warmup 2 --cpu-sample 0 \
&& SH_SPARSE_XCD=0 scripts/gpu.sh bench r4x_c5x0 --config c5 --steps 5 --warmup 2 --cpu-sample 0 --no-verify \
&& SH_SPARSE_XCD=1 scripts/gpu.sh bench r4x_c5x1b --config c5 --steps 5 --warmup 2 --cpu-sample 0 --no-verify \
&& SH_SPARSE_XCD=0 scripts/gpu.sh bench r4x_c5x0b --config c5 --steps 5 --warmup 2 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh test r4x_rules tests/test_gpu_rules.py \
&& scripts/gpu.sh pmc r4x_c2af FETCH_SIZE --config c2 --agg $A \
&& scripts/gpu.sh pmc r4x_c2aw WRITE_SIZE --config c2 --agg $A \
&& SH_SPARSE_XCD=1 scripts/gpu.sh pmc r4x_c5f FETCH_SIZE --config c5 $A
