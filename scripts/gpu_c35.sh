#!/bin/bash
# C3 and C5 benches at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c35
timeout -k 10 400 python -u bench.py --config c3 --steps 2 --warmup 1 > gpurun_out/c35/c3.log 2>&1 || { tail -3 gpurun_out/c35/c3.log; exit 1; }
grep "^{" gpurun_out/c35/c3.log | cut -c1-250
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c35/c5.log 2>&1 || { tail -3 gpurun_out/c35/c5.log; exit 1; }
grep "^{" gpurun_out/c35/c5.log | cut -c1-250
