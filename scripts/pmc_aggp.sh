#!/bin/bash
# SQ counters of the C2+agg step (k_bk_aggp and the rest), two passes of <= 8 SQ counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --config c2 --agg --steps 2 --warmup 1 --cpu-sample 0 --no-verify"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES --output-format csv -d $R/gpurun_out/agg_sq1 -o run -- $B > $R/gpurun_out/agg_sq1.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_LDS,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_INST_CYCLES_VMEM_RD --output-format csv -d $R/gpurun_out/agg_sq2 -o run -- $B > $R/gpurun_out/agg_sq2.log 2>&1 &&
python3 $R/scripts/pmc_table.py $R/gpurun_out/agg_sq1 $R/gpurun_out/agg_sq2 > $R/gpurun_out/agg_sq.txt
