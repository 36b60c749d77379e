#!/bin/bash
# Step-shape sweep on one box: the default bench (no CPU baseline, no hard / worst batches) at
# several (pairs per step, streams) shapes; prints value and ms per step for each.
#   CONFIGS="768:4 1024:4 1536:4 768:6" bash scripts/gpu_step_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CONFIGS:-768:4 1024:4}; do
  P=${C%%:*}; S=${C##*:}
  F=gpurun_out/sweep_${P}x${S}
  echo "== pairs $P streams $S" && timeout -k 10 400 python bench.py --no-cpu-baseline --hard-steps 0 --worst-steps 0 --steps ${STEPS:-8} --warmup 2 --pairs $P --streams $S > $F.json 2> $F.err || { tail -20 $F.err; exit 1; }
  python -c "import json;d=json.loads(open('$F.json').read().strip().splitlines()[-1]);print(round(d['value']), round(d['ms_per_step'],2), d['overlap'])"
done
