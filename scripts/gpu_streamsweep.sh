#!/bin/bash
# throughput vs batch size and sub-batch streams (configs[1] shape)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in ${CFGS:-128:1}; do
  set -- ${cfg/:/ }
  timeout -k 10 400 python bench.py --steps ${STEPS:-4} --warmup 2 --pairs $1 --streams $2 --no-cpu-baseline --hard-steps 0 > gpurun_out/ss_$1_$2.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ss_$1_$2.log').read().strip().splitlines()[-1]);print('$1 $2', round(d['value']), round(d['ms_per_step'],2))"
done
