#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 4 6 8 12; do
  SH_BK_WALK=$d scripts/gpu_step.sh 200 gpurun_out/walk_$d.log python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 || exit $?
  echo "D=$d $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/walk_$d.log) $(grep -o '"phase_ms": {[^}]*}' gpurun_out/walk_$d.log) $(grep -o '"verified_vs_restatement": [a-z]*' gpurun_out/walk_$d.log)"
done
