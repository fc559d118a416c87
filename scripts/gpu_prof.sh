#!/bin/bash
# kernel-trace profile of the bench (separate from PMC passes)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1
rc=$?
echo "rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
