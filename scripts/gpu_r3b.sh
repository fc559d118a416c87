#!/bin/bash
# round 3: failed-restore test, C2 phase clocks, C2 kernel stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_snapshot.py -x -q -k "failed_restore or refuses" --timeout 200 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1; echo "tests rc=$?"; tail -30 gpurun_out/r3b_tests.log | grep -E "Error|assert|passed|failed"
SH_BK_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3b_c2_prof.json 2> gpurun_out/r3b_c2_prof.err || { tail -20 gpurun_out/r3b_c2_prof.err; exit 1; }
grep "clock ticks" gpurun_out/r3b_c2_prof.err | tail -2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof -o c2 -- python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3b_c2.json 2> gpurun_out/r3b_c2.err || { tail -20 gpurun_out/r3b_c2.err; exit 1; }
cat gpurun_out/r3b_c2.json
find gpurun_out/r3b_prof -name "*kernel_stats.csv" | head -1 | xargs head -12
