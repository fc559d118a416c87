#!/bin/bash
# C5 kernel stats + one SQ / one L2 PMC pass (round-3 planning)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- \
    python bench.py --config c5 --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof5/bench_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof done"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/c5pmc_$i -o c5 -- \
      python bench.py --config c5 --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/c5pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  echo "pass $i done"
done
python scripts/pmc_table.py gpurun_out/c5pmc_1 gpurun_out/c5pmc_2 > gpurun_out/c5pmc_table.txt
head -8 gpurun_out/c5pmc_table.txt
