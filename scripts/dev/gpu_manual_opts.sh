#!/bin/bash
# configs[4] (one 100k-iteration find, K ~ 89k rows) under route options: the pruning stages
# added for the 128-pair configs[1] launches (gradient references, flat-pair route, hinted
# refine windows, second stage) against their single-pair cost.  One bench line per arm.
#   TAG=r06h bash scripts/dev/gpu_manual_opts.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r06h}
ARMS=${ARMS:-"default lipg=0 flat_refs=0 refine_hint=0 lip2=0 flat_refs=0,refine_hint=0"}
for a in $ARMS; do
  OPTS=""
  if [ "$a" != default ]; then for kv in $(echo "$a" | tr ',' ' '); do OPTS="$OPTS --ctx-option $kv"; done; fi
  F=gpurun_out/manual_${TAG}_$(echo "$a" | tr ',=' '_-')
  timeout -k 10 300 python bench.py --workload manual --steps 10 --warmup 2 $OPTS > $F.json 2> $F.err \
    || { tail -20 $F.err; exit 1; }
  python -c "import json;d=json.load(open('$F.json'));s=d['stages_ms_rank0'];print('$a', round(d['ms_per_step'],3), d['check']['same_as_unsharded'], {k:round(v,3) for k,v in s.items() if v>0.05})"
done
