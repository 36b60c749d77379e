#!/bin/bash
# SURF parity tests, the SURF timing probe under rocprofv3 (kernel stats), the e2e bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s}
echo "== surf tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_surf.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_surf.log 2>&1 || { tail -40 gpurun_out/pytest_surf.log; exit 1; }
tail -1 gpurun_out/pytest_surf.log
echo "== surf prof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof_${TAG} -o sp --output-format csv -- python3 scripts/dev/surf_prof.py > gpurun_out/sprof_${TAG}.log 2>&1 || { tail -20 gpurun_out/sprof_${TAG}.log; exit 1; }
grep "surf 8 bands" gpurun_out/sprof_${TAG}.log
f=$(find gpurun_out/sprof_${TAG} -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-150 | head -14
echo "== e2e" && timeout -k 10 300 python bench.py --workload e2e --steps 8 --warmup 2 --iters 10000 > gpurun_out/e2e_${TAG}.json 2> gpurun_out/e2e_${TAG}.err || { tail -20 gpurun_out/e2e_${TAG}.err; exit 1; }
cat gpurun_out/e2e_${TAG}.json
