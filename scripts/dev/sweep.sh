#!/bin/bash
# batch-size x stream-count sweep of bench.py (no CPU baseline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "8 1" "8 2" "16 1" "16 2" "32 1" "32 2" "32 4" "64 1" "64 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --pairs $1 --streams $2 > gpurun_out/sweep_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/sweep_$1_$2.log; exit 1; }
  echo "B=$1 S=$2 $(tail -1 gpurun_out/sweep_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')"
done
