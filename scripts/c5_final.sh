#!/bin/bash
# C5 line, kernel summary and PMC passes at the current build (round-6 close)
set -o pipefail
A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench c5 --config c5 --steps 5 --warmup 2 \
&& scripts/gpu.sh prof c5prof --config c5 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& for ctr in FETCH_SIZE WRITE_SIZE; do scripts/gpu.sh pmc c5_$ctr $ctr --config c5 $A || exit 1; done
