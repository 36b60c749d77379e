#!/bin/bash
# consensus knob A/B on one box: each setting (";"-separated env assignments in CONFIGS) runs
# the default bench (no CPU baseline, 2 worst-case steps); prints value, consensus, worst case
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra CFG <<< "${CONFIGS:-X=0}"
for r in 1 2; do
for c in "${CFG[@]}"; do
  F=gpurun_out/knob_$(echo "$c" | tr ' =' '__')_$r.json
  env $c timeout -k 10 400 python bench.py --no-cpu-baseline --steps 6 --warmup 2 --hard-steps 0 --worst-steps 2 > $F 2> $F.err || { tail -20 $F.err; exit 1; }
  python -c "
import json;d=json.loads(open('$F').read().strip().splitlines()[-1]);s=d['stages_ms_serial_step'];w=d.get('worst_case') or {}
print('$c', round(d['value']), round(d['ms_per_step'],2), 'cons', round(s['consensus_bounds']+s['consensus_refine']+s['consensus_select']+s['consensus_rows']+s['consensus_final'],2), 'worst', round(w.get('value',0)), d.get('exact'))"
done; done
