# C4: the speculative due pass (one sync for the event launch and the first due pass)
# A/B on the first 3,000 calls, alternating arms in one call, then the C4 tests
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c4
mkdir -p $O
cd $R
for i in 1 2; do
    SH_SPEC_DUE=0 timeout -k 10 300 python3 bench.py --config c4 --c4-calls 3000 --steps 1 --warmup 1 --cpu-sample 0 > $O/off_$i.json 2> $O/off_$i.log || exit 1
    SH_SPEC_DUE=1 timeout -k 10 300 python3 bench.py --config c4 --c4-calls 3000 --steps 1 --warmup 1 --cpu-sample 0 > $O/on_$i.json 2> $O/on_$i.log || exit 1
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4.py tests/test_gpu_snapshot.py \
    tests/test_gpu_shard_stream.py > $O/tests.log 2>&1
