#!/bin/bash
# batch-size x stream-count sweep of bench.py (no CPU baseline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-"8 1" "32 1" "64 1" "64 2" "128 1" "128 2"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --pairs $1 --streams $2 > gpurun_out/sweep_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/sweep_$1_$2.log; exit 1; }
  echo "B=$1 S=$2 $(tail -1 gpurun_out/sweep_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), {k:round(v,2) for k,v in d["stages_ms_per_step"].items() if v > 0.1*d["ms_per_step"]})')"
done
