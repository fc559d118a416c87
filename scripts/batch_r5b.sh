A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench r5b_c2 --config c2 --steps 20 --warmup 3 \
&& scripts/gpu.sh prof r5b_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh pmc r5b_c2f FETCH_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r5b_c2w WRITE_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r5b_c3f FETCH_SIZE --config c3 $A \
&& scripts/gpu.sh pmc r5b_c3w WRITE_SIZE --config c3 $A \
&& scripts/gpu.sh pmc r5b_c2sq SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES --config c2 $A \
&& scripts/gpu.sh test r5b_tests tests/test_gpu_bucket.py tests/test_gpu_c3.py tests/test_gpu_agg.py tests/test_gpu_shard.py
