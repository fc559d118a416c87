#!/bin/bash
# round 3: smoke, C2 line, aggregate-select lines (C2 / C3), C2 phase clocks + kernel stats, 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3e_smoke.log 2>&1 || { tail -20 gpurun_out/r3e_smoke.log; exit 1; }
tail -1 gpurun_out/r3e_smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3e_c2.json 2> gpurun_out/r3e_c2.err || { tail -20 gpurun_out/r3e_c2.err; exit 1; }
cat gpurun_out/r3e_c2.json
timeout -k 10 300 python -u bench.py --agg --steps 10 --warmup 3 --cpu-sample 500000 > gpurun_out/r3e_c2agg.json 2> gpurun_out/r3e_c2agg.err || { tail -20 gpurun_out/r3e_c2agg.err; exit 1; }
cat gpurun_out/r3e_c2agg.json
timeout -k 10 400 python -u bench.py --config c3 --agg --steps 5 --warmup 2 --cpu-sample 500000 > gpurun_out/r3e_c3agg.json 2> gpurun_out/r3e_c3agg.err || { tail -20 gpurun_out/r3e_c3agg.err; exit 1; }
cat gpurun_out/r3e_c3agg.json
SH_BK_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3e_c2_prof.json 2> gpurun_out/r3e_c2_prof.err || { tail -20 gpurun_out/r3e_c2_prof.err; exit 1; }
grep "clock ticks" gpurun_out/r3e_c2_prof.err | tail -1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e_prof -o c2 -- python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/r3e_c2p.json 2> gpurun_out/r3e_c2p.err || { tail -20 gpurun_out/r3e_c2p.err; exit 1; }
find gpurun_out/r3e_prof -name "*kernel_stats.csv" | head -1 | xargs head -12
for c in c3 c5; do
  SH_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --config $c --gpus 2 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r3e_rehearse_$c.json 2> gpurun_out/r3e_rehearse_$c.err || { tail -20 gpurun_out/r3e_rehearse_$c.err; exit 1; }
  cat gpurun_out/r3e_rehearse_$c.json
done
