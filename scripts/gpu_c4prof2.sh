#!/bin/bash
# kernel + HIP API statistics of C4 at 10M users, first 12k send calls
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4p2
timeout -k 10 500 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d gpurun_out/c4p2 -o c4 -- \
    python -u bench.py --config c4 --c4-calls 12000 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4p2/log 2>&1 || { tail -5 gpurun_out/c4p2/log; exit 1; }
grep "^{" gpurun_out/c4p2/log | cut -c1-300; rm -f gpurun_out/c4p2/*trace.csv
