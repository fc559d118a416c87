#!/bin/bash
# Same-call A/B of an environment switch on one bench config (run under gpurun):
#   scripts/env_ab.sh NAME "ENV_A" "ENV_B" [bench.py args]
# Arms alternate A B A B; arm B's first run verifies the output. Lines land in
# gpurun_out/NAME/; the summary prints ms/step and the phase split per run.
set -o pipefail
name=$1; ea=$2; eb=$3; shift 3
mkdir -p gpurun_out/$name
for r in 1 2; do
  for arm in A B; do
    e=$ea; [ $arm = B ] && e=$eb
    v="--no-verify"; [ $arm = B ] && [ $r = 1 ] && v=""
    env $e timeout -k 10 300 python -u bench.py --cpu-sample 0 $v "$@" \
        > gpurun_out/$name/$arm$r.json 2> gpurun_out/$name/$arm$r.err || { tail -20 gpurun_out/$name/$arm$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/$name/$arm$r.json').read().strip().splitlines()[-1]); p=d.get('phase_ms') or {}; print('$arm$r', '$e', round(d['ms_per_step'],3), 'verified', d.get('verified_vs_restatement'), {k: round(v,3) for k,v in p.items() if v})"
  done
done
