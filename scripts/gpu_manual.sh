#!/bin/bash
# configs[4]: the sharded-hypothesis tests + the manual-regime bench at N=1 (100k iterations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01f}
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "== manual bench" && timeout -k 10 300 python bench.py --workload manual --steps 3 --warmup 1 > gpurun_out/manual_${TAG}.json 2> gpurun_out/manual_${TAG}.err || { tail -20 gpurun_out/manual_${TAG}.err; exit 1; }
cut -c1-2500 gpurun_out/manual_${TAG}.json
