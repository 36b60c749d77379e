#!/bin/bash
# whole GPU test suite, then the end-to-end pipeline bench (do_all + find from 5376 x 2688 images)
# and a rocprofv3 kernel-stats pass over it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01h}
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "== e2e" && timeout -k 10 300 python bench.py --workload e2e --steps 8 --warmup 2 --iters 10000 > gpurun_out/e2e_${TAG}.json 2> gpurun_out/e2e_${TAG}.err || { tail -20 gpurun_out/e2e_${TAG}.err; exit 1; }
cat gpurun_out/e2e_${TAG}.json
echo "== e2e prof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e_${TAG} -o e2e --output-format csv -- python3 bench.py --workload e2e --steps 4 --warmup 1 --iters 10000 > gpurun_out/prof_e2e_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_e2e_${TAG}.log; exit 1; }
find gpurun_out/prof_e2e_${TAG} -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -25'
