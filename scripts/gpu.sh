#!/bin/bash
# GPU-box helper (run under gpurun from the repo root), one step per call:
#   scripts/gpu.sh bench NAME [bench.py args]    -> gpurun_out/NAME.json (+ .err)
#   scripts/gpu.sh test NAME [pytest args]       -> gpurun_out/NAME.log
#   scripts/gpu.sh prof NAME [bench.py args]     -> rocprofv3 kernel-trace stats in gpurun_out/NAME/
#   scripts/gpu.sh pmc NAME COUNTER [bench.py args] -> one PMC pass in gpurun_out/NAME/
# Every step has its own time limit; chain steps with && so a failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cmd=$1; name=$2; shift 2
case $cmd in
bench)
    timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err \
        || { tail -30 gpurun_out/$name.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'], 3), 'ms', round(d['value']/1e9, 3), 'Gev/s', 'frac', round(d['roofline']['frac'], 4), 'verified', d.get('verified_vs_restatement'), d.get('phase_ms'))"
    ;;
test)
    timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1 \
        || { tail -60 gpurun_out/$name.log; exit 1; }
    tail -3 gpurun_out/$name.log
    ;;
prof)
    export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o run -- python3 -u bench.py "$@" \
        > gpurun_out/$name.out 2> gpurun_out/$name.err || { tail -30 gpurun_out/$name.err; exit 1; }
    db=$(find gpurun_out/$name -name "*.db" | head -1)
    python scripts/prof_db.py "$db" gpurun_out/$name.kernel_stats.csv
    head -12 gpurun_out/$name.kernel_stats.csv | cut -c1-160
    ;;
pmc)
    ctr=$1; shift
    export TMPDIR=/tmp
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/$name -o run -- python3 -u bench.py "$@" \
        > gpurun_out/$name.out 2> gpurun_out/$name.err || { tail -30 gpurun_out/$name.err; exit 1; }
    echo "pmc $name $ctr done"
    ;;
*) echo "unknown step $cmd"; exit 2 ;;
esac
