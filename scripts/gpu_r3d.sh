#!/bin/bash
# round 3 re-entry: whole -m gpu suite at HEAD (skip reasons listed), smoke, C2 bench line
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r3d_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAIL|ERROR" gpurun_out/r3d_tests.log | head -20; tail -40 gpurun_out/r3d_tests.log; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r3d_smoke.log 2>&1 || { tail -20 gpurun_out/r3d_smoke.log; exit 1; }
tail -1 gpurun_out/r3d_smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3d_c2.json 2> gpurun_out/r3d_c2.err || { tail -20 gpurun_out/r3d_c2.err; exit 1; }
cat gpurun_out/r3d_c2.json
