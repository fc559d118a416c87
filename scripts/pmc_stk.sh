cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES --output-format csv -d $R/gpurun_out/stk_sq1 -o run -- python3 $R/scripts/stk_debug.py 20000000 10000 > $R/gpurun_out/stk_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_LDS,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_INST_CYCLES_VMEM_RD --output-format csv -d $R/gpurun_out/stk_sq2 -o run -- python3 $R/scripts/stk_debug.py 20000000 10000 > $R/gpurun_out/stk_sq2.log 2>&1
echo rc=$?
python3 $R/scripts/pmc_table.py $R/gpurun_out/stk_sq1 $R/gpurun_out/stk_sq2 | head
