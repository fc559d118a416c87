# C5 check: verified line + kernel summary + rule tests
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c5
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --cpu-sample 0 > $O/c5.json 2> $O/c5.log || exit 1
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --config c5 \
    --steps 3 --warmup 1 --cpu-sample 0 --no-verify > $O/c5p.json 2> $O/c5p.log) || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rules.py > $O/rules.log 2>&1
