#!/bin/bash
# emitter workgroups per CU (LDS padding) on C2 + aggregates and plain C2: step times
set -o pipefail
mkdir -p gpurun_out/emit_pad
for pad in 0 12288; do
  for agg in "--agg" ""; do
    SH_EMIT_LDS_PAD=$pad timeout -k 10 300 python bench.py --config c2 $agg --steps 10 --warmup 2 --cpu-sample 0 --no-verify \
        > gpurun_out/emit_pad/b_${pad}${agg}.json 2>/dev/null || exit 1
  done
done
