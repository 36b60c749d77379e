#!/bin/bash
# same-box bench A/B: VARIANTS = "name=lib[,ctx_option=value...]" (lib: scripts/dev/libs/<lib>),
# ROUNDS alternating 10-step benches, one summary line each (pairs/s, ms per step, exact, the
# serial stage times of gram / sampler / consensus / filter).
#   TAG=r06ah VARIANTS="base=base gpad=gpad t1=base,gram_tiles=1" bash scripts/dev/gpu_bench_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-ab}; ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do for spec in $VARIANTS; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; opts=""
  [ "$rest" != "$lib" ] && for o in $(echo "${rest#*,}" | tr ',' ' '); do opts="$opts --ctx-option $o"; done
  ERP_LIB_PATH=scripts/dev/libs/$lib/liberp_match.so timeout -k 10 400 python bench.py --no-cpu-baseline \
    --steps ${STEPS:-10} --warmup 3 --hard-steps 0 --worst-steps ${WORST_STEPS:-0} $opts > gpurun_out/ab_${TAG}_$name$r.json \
    2> gpurun_out/ab_${TAG}_$name$r.err || { tail -20 gpurun_out/ab_${TAG}_$name$r.err; exit 1; }
  echo "$name$r $(python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_$name$r.json'));s=d['stages_ms_serial_step'];print(round(d['value']), round(d['ms_per_step'],2), d['exact'], 'gram', round(s.get('gram',0),3), 'sampler', round(s.get('sampler',0),3), 'cons', round(sum(v for k,v in s.items() if k.startswith('consensus')),3), 'filter', round(s['knn2_filter'],3), 'rescore', round(s['knn2_rescore'],3), 'worst', (d.get('worst_case') or {}).get('value'))")"
done; done
echo done
