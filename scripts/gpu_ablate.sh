#!/bin/bash
# timing ablations (ERP_DEBUG_MODE): stage times only, results invalid for modes != 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 0 1 2 3; do
  echo "== mode $m"
  ERP_DEBUG_MODE=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ablate_$m.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ablate_$m.log').read().strip().splitlines()[-1]);print({k:round(v,3) for k,v in d['stages_ms_serial_step'].items()})"
done
