#!/bin/bash
# window-engine parity (consumer-side walk), then the C2 bench and kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
S=scripts/gpu_step.sh
$S 600 gpurun_out/ext_tests.log python -u -m pytest tests/test_gpu_parity.py -k "window or c2" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -n 3 gpurun_out/ext_tests.log
grep -q "failed" gpurun_out/ext_tests.log && exit 1
$S 600 gpurun_out/bench.log python -u bench.py --steps 5 --warmup 2 --cpu-sample 200000 || exit $?
tail -n 1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof/bench_prof.log 2>&1 || exit $?
python scripts/show_prof.py
