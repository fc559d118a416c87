#!/bin/bash
# HBM traffic of the C2 + aggregates step (packed rows, k_bk_aggp): FETCH_SIZE / WRITE_SIZE passes + calibration
set -o pipefail
A="--steps 2 --warmup 1 --cpu-sample 0 --no-verify"
for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
        -d $GRAFT_REPO_ROOT/gpurun_out/cal_$ctr -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) || exit 1
    scripts/gpu.sh pmc c2agg_$ctr $ctr --config c2 --agg $A || exit 1
done
scripts/gpu.sh prof c2aggprof --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 --no-verify
