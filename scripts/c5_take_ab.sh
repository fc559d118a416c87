#!/bin/bash
# C5 k_sparse_take: 1,024-thread workgroups (one per CU) vs 512 at <= 80 VGPRs (SH_TAKE_512=1)
set -o pipefail
mkdir -p gpurun_out/c5_take
SH_TAKE_512=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rules.py \
    > gpurun_out/c5_take/tests.log 2>&1 || exit 1
for t in 0 1 0 1; do
  SH_TAKE_512=$t timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
      >> gpurun_out/c5_take/b_$t.json 2>/dev/null || exit 1
done
SH_TAKE_512=1 bash scripts/gpu.sh prof c5take512 --config c5 --steps 5 --warmup 1 --cpu-sample 0 --no-verify
