S="SH_BK_SPAN=3072 SH_BK_CH=2048 SH_BK_CT=56 SH_BK_MINB=6"
scripts/gpu.sh bench r4s_c2a --config c2 --steps 20 --warmup 3 \
&& env $S scripts/gpu.sh bench r4s_c2b --config c2 --steps 20 --warmup 3 --cpu-sample 0 \
&& scripts/gpu.sh bench r4s_c2c --config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify \
&& env $S scripts/gpu.sh bench r4s_c2d --config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh prof r4s_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4s_calf -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) \
&& (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4s_calw -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) \
&& scripts/gpu.sh pmc r4s_c2f FETCH_SIZE --config c2 --steps 1 --warmup 0 --cpu-sample 0 --no-verify \
&& scripts/gpu.sh pmc r4s_c2w WRITE_SIZE --config c2 --steps 1 --warmup 0 --cpu-sample 0 --no-verify
