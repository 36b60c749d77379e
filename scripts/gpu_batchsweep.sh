#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in 8 16 32; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --pairs $b --no-cpu-baseline > gpurun_out/sweep_$b.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/sweep_$b.log').read().strip().splitlines()[-1]);print($b, round(d["value"]), d["check"]["consensus_survivors"], {k:round(v,3) for k,v in d["stages_ms_serial_step"].items() if v>0.05})"
done
