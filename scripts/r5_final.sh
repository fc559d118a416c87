#!/bin/bash
# round-5 closing batch, part 1 (tests) or 2 (bench lines + kernel summaries)
set -o pipefail
mkdir -p gpurun_out/final
if [ "$1" = tests ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
      > gpurun_out/final/gpu_tests.log 2>&1
  exit $?
fi
for c in c2 c3 c5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/final/bench_$c.json 2> gpurun_out/final/bench_$c.err || exit 1
done
timeout -k 10 400 python -u bench.py --config c2 --agg > gpurun_out/final/bench_c2_agg.json 2> gpurun_out/final/bench_c2_agg.err || exit 1
bash scripts/gpu.sh prof final_c2prof --config c2 --steps 5 --warmup 1 --cpu-sample 0 --no-verify &&
bash scripts/gpu.sh prof final_c3prof --config c3 --steps 5 --warmup 1 --cpu-sample 0 --no-verify
