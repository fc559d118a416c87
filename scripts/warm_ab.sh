# C2 emitter L2 warming A/B on one box: alternating runs with the warming on
# (SH_BK_WARM=1) and off (SH_BK_WARM=0), 20 timed steps each, verification off
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/warm
mkdir -p $O
for i in 1 2 3; do
    SH_BK_WARM=1 timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 3 --cpu-sample 0 --no-verify > $O/on_$i.json 2> $O/on_$i.log || exit 1
    SH_BK_WARM=0 timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 3 --cpu-sample 0 --no-verify > $O/off_$i.json 2> $O/off_$i.log || exit 1
done
