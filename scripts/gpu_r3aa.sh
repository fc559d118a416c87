#!/bin/bash
# round 3: C2 matcher launch bound A/B (SH_BK_MINB: minimum workgroups per CU the registers are sized for;
# its LDS holds two), with the walk block size at the larger register budget
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r3aa_$name.json 2> gpurun_out/r3aa_$name.err || { tail -20 gpurun_out/r3aa_$name.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r3aa_$name.json').read()); print('$name', round(d['ms_per_step'], 3), d.get('verified_vs_restatement'), {k: round(v, 3) for k, v in d.get('phase_ms', {}).items()})"
}
run minb4 X=0
run minb2 SH_BK_MINB=2
run minb3 SH_BK_MINB=3
run minb2_w6 SH_BK_MINB=2 SH_BK_WALK=6
run minb2_w8 SH_BK_MINB=2 SH_BK_WALK=8
SH_BK_MINB=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_bucket.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3aa_bucket_minb2.log 2>&1 || { tail -30 gpurun_out/r3aa_bucket_minb2.log; exit 1; }
tail -1 gpurun_out/r3aa_bucket_minb2.log
