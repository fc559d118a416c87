A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh pmc r4u_c2sq SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES --config c2 $A \
&& (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4u_calf -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) \
&& (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4u_calw -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) \
&& scripts/gpu.sh pmc r4u_c2f FETCH_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r4u_c2w WRITE_SIZE --config c2 $A \
&& scripts/gpu.sh pmc r4u_c3f FETCH_SIZE --config c3 $A \
&& scripts/gpu.sh pmc r4u_c3w WRITE_SIZE --config c3 $A \
&& scripts/gpu.sh prof r4u_c3prof --config c3 --steps 5 --warmup 1 --cpu-sample 0 --no-verify
