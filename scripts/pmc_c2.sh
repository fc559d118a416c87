#!/bin/bash
# HBM traffic of the C2 step (packed rows): FETCH_SIZE / WRITE_SIZE passes + calibration
set -o pipefail
A="--steps 2 --warmup 1 --cpu-sample 0 --no-verify"
for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
        -d $GRAFT_REPO_ROOT/gpurun_out/cal_$ctr -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) || exit 1
    scripts/gpu.sh pmc c2_$ctr $ctr --config c2 $A || exit 1
done
