#!/bin/bash
# PMC passes (kernel trace only, one --pmc pass per counter group) over a short bench run.
# usage: gpu_pmc.sh TAG "COUNTERS A" ["COUNTERS B" ...]   (extra bench args via BENCH_ARGS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
i=0
for grp in "$@"; do
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  i=$((i+1))
done
echo done
