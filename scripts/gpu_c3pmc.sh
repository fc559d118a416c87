#!/bin/bash
# C3 PMC passes (one counter group per run): SQ wave-state counters, fabric bytes, L2 hit rate
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/c3pmc_$i -o c3 -- \
      python bench.py --config c3 --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/c3pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  echo "pass $i done"
done
python scripts/pmc_table.py gpurun_out/c3pmc_1 gpurun_out/c3pmc_2 gpurun_out/c3pmc_3 gpurun_out/c3pmc_4 > gpurun_out/c3pmc_table.txt
cat gpurun_out/c3pmc_table.txt
