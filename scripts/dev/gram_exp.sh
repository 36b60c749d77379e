#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for GB in 8 6 4 2; do
  ERP_GRAM_B=$GB timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pairs 8 > gpurun_out/gram_b$GB.log 2>&1 || exit 1
  echo "GB=$GB $(tail -1 gpurun_out/gram_b$GB.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms_per_step"]; print(round(d["value"]), s["gram"], s["eigen"])')"
done
