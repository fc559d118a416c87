# C3: k_s3b2 (two workgroups per bucket) vs k_s3b in one call, then the C3 tests
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c3
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0 > $O/sub.json 2> $O/sub.log || exit 1
SH_S3B_SUB=0 timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0 --no-verify > $O/one.json 2> $O/one.log || exit 1
SH_BK_PROFILE=1 timeout -k 10 300 python3 bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --no-verify > $O/prof.json 2> $O/prof.log || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c3.py > $O/tests.log 2>&1
