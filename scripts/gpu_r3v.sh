#!/bin/bash
# round 3 final evidence: the whole -m gpu suite, smoke(), the default bench line (C2) with its rocprof kernel
# summary and calibrated PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes), and C4's `every` variant
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3v_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3v_tests.log | head -20; tail -40 gpurun_out/r3v_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3v_smoke.log 2>&1 || { tail -20 gpurun_out/r3v_smoke.log; exit 1; }
tail -1 gpurun_out/r3v_smoke.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3v_prof -o run -- python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3v_prof.json 2> gpurun_out/r3v_prof.err || { tail -20 gpurun_out/r3v_prof.err; exit 1; }
find gpurun_out/r3v_prof -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-140
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3v_fetch -o run -- python -u bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/r3v_fetch.json 2> gpurun_out/r3v_fetch.err || { tail -20 gpurun_out/r3v_fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3v_write -o run -- python -u bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify > gpurun_out/r3v_write.json 2> gpurun_out/r3v_write.err || { tail -20 gpurun_out/r3v_write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3v_cfetch -o run -- python -u scripts/pmc_calib.py > gpurun_out/r3v_cfetch.log 2>&1 || { tail -20 gpurun_out/r3v_cfetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3v_cwrite -o run -- python -u scripts/pmc_calib.py > gpurun_out/r3v_cwrite.log 2>&1 || { tail -20 gpurun_out/r3v_cwrite.log; exit 1; }
python scripts/pmc_traffic.py gpurun_out/r3v_fetch gpurun_out/r3v_write 1 100000000 10000 gpurun_out/r3v_pmc_c2.json c2 --calib gpurun_out/r3v_cfetch gpurun_out/r3v_cwrite 2147483648 > gpurun_out/r3v_pmc.log 2>&1 || { tail -20 gpurun_out/r3v_pmc.log; exit 1; }
tail -5 gpurun_out/r3v_pmc.log
timeout -k 10 600 python -u bench.py --config c4 --c4-every --steps 1 --warmup 1 > gpurun_out/r3v_c4every.json 2> gpurun_out/r3v_c4every.err || { tail -20 gpurun_out/r3v_c4every.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3v_c4every.json').read()); print('c4 every', round(d['ms_per_step'],1), d['value'], d['config']['matches_total'], d['cpu_baseline']['value'])"
