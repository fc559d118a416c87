# One-GPU timings of C2 / C3 / C5 at the per-rank sizes of N = 1, 2, 4, 8: a rank
# of an N-GPU key-sharded step matches ~1/N of the events over 1/N of the keys at
# 1/N of the rate (the per-key rate and window density stay those of the whole
# stream). Each size runs bench.py under rocprofv3 --kernel-trace --stats; the
# JSON lines and kernel summaries land in gpurun_out/scale/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/scale
mkdir -p $O
run() {  # name, bench args
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run -- python3 $R/bench.py --steps 5 --warmup 2 \
        --cpu-sample 0 --no-verify "$@" > $O/$name.json 2> $O/$name.log || return 1
    echo "$name done"
}
CFGS=${SCALE_CFGS:-"c2 c3 c5"}
case " $CFGS " in *" c2 "*) for N in 1 2 4 8; do
    run c2_n$N --config c2 --events $((100000000 / N)) --keys $((10000 / N)) --rate $((100 / N)) || exit 1
done ;; esac
case " $CFGS " in *" c3 "*) for N in 1 2 4 8; do
    run c3_n$N --config c3 --events $((100000000 / N)) --keys $((1000000 / N)) --rate $((1000 / N)) || exit 1
done ;; esac
case " $CFGS " in *" c5 "*) for N in 1 2 4 8; do
    run c5_n$N --config c5 --events $((100000000 / N)) --keys $((1000000 / N)) --rate $((100 / N)) || exit 1
done ;; esac
