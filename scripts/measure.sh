#!/bin/bash
# The round's measurement recipes (run under gpurun from the repo root, one step per
# call of scripts/gpu.sh, each with its own time limit; steps chained with &&):
#   scripts/measure.sh bench     C2 / C3 / C5 / C2+agg lines and the whole C4 stream
#   scripts/measure.sh prof      rocprofv3 kernel summaries (C2, C3, C5, C2+agg)
#   scripts/measure.sh pmc       FETCH_SIZE / WRITE_SIZE passes (+ calibration) and C2 SQ counters
#   scripts/measure.sh rehearse  2 ranks sharing one GPU over gloo (C2, C4 first 3,000 calls)
#   scripts/measure.sh tests     smoke + the whole -m gpu suite with skip reasons
# Outputs land in gpurun_out/; scripts/pmc_traffic.py turns the PMC passes into
# profiles/pmc_<variant>.json.
set -o pipefail
A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
case $1 in
bench)
    scripts/gpu.sh bench c2 --config c2 --steps 20 --warmup 3 \
    && scripts/gpu.sh bench c3 --config c3 --steps 10 --warmup 2 \
    && scripts/gpu.sh bench c5 --config c5 --steps 5 --warmup 2 \
    && scripts/gpu.sh bench c2agg --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 \
    && scripts/gpu.sh bench c4 --config c4 --steps 1 --warmup 0
    ;;
prof)
    for c in c2 c3 c5; do scripts/gpu.sh prof ${c}prof --config $c --steps 5 --warmup 1 --cpu-sample 0 --no-verify || exit 1; done
    scripts/gpu.sh prof c2aggprof --config c2 --agg --steps 3 --warmup 1 --cpu-sample 0 --no-verify
    ;;
pmc)
    for ctr in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
            -d $GRAFT_REPO_ROOT/gpurun_out/cal_$ctr -o run -- python3 $GRAFT_REPO_ROOT/scripts/pmc_calib.py) || exit 1
        for c in c2 c3 c5; do scripts/gpu.sh pmc ${c}_$ctr $ctr --config $c $A || exit 1; done
        scripts/gpu.sh pmc c2agg_$ctr $ctr --config c2 --agg $A || exit 1
    done
    scripts/gpu.sh pmc c2sq SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES --config c2 $A
    ;;
rehearse)
    R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
    SH_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --master-port 29533 bench.py --gpus 2 --config c2 --steps 5 --warmup 1 \
        --cpu-sample 0 > gpurun_out/reh_c2.json 2> gpurun_out/reh_c2.err \
    && SH_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --master-port 29534 bench.py --gpus 2 --config c4 --c4-calls 3000 \
        --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/reh_c4.json 2> gpurun_out/reh_c4.err
    ;;
tests)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    && scripts/gpu.sh test all tests -m gpu -rs
    ;;
*) echo "usage: scripts/measure.sh bench|prof|pmc|rehearse|tests"; exit 2 ;;
esac
