#!/bin/bash
# C3 line, kernel summary and PMC passes at the current build (round-6 close)
set -o pipefail
A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench c3 --config c3 --steps 10 --warmup 2 \
&& scripts/gpu.sh prof c3prof --config c3 --steps 5 --warmup 1 --cpu-sample 0 --no-verify \
&& for ctr in FETCH_SIZE WRITE_SIZE; do scripts/gpu.sh pmc c3_$ctr $ctr --config c3 $A || exit 1; done
