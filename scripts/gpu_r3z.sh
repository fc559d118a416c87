#!/bin/bash
# round 3: segment variants on C5 / C3 after the scatter's LDS cut: 8-bit digits (default), two 10-bit passes
# (SH_RADIX10=1), columns carried by the last pass only (SH_SEG_LASTCARRY=1)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, config, env...
    local name=$1 cfg=$2; shift 2
    env "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/r3z_$name.json 2> gpurun_out/r3z_$name.err || { tail -20 gpurun_out/r3z_$name.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r3z_$name.json').read()); print('$name', round(d['ms_per_step'], 3), d.get('verified_vs_restatement'), d.get('phase_ms'))"
}
run c5_base c5 X=0
run c5_r10 c5 SH_RADIX10=1
run c5_last c5 SH_SEG_LASTCARRY=1
run c3_base c3 X=0
run c3_r10 c3 SH_RADIX10=1
