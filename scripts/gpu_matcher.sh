#!/bin/bash
# configs[3] matcher comparison: matcher parity tests on both methods, the batch test with the
# VALU matcher, the dense 16k bench (both methods) and a rocprofv3 kernel-trace of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01f}
echo "== matcher tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "== dense bench" && timeout -k 10 300 python bench.py --workload dense --steps 5 --warmup 2 > gpurun_out/dense_${TAG}.json 2> gpurun_out/dense_${TAG}.err || { tail -20 gpurun_out/dense_${TAG}.err; exit 1; }
cat gpurun_out/dense_${TAG}.json | cut -c1-1500
echo "== pairs bench, valu matcher" && timeout -k 10 300 python bench.py --matcher valu --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pairs_valu_${TAG}.json 2> gpurun_out/pairs_valu_${TAG}.err || { tail -20 gpurun_out/pairs_valu_${TAG}.err; exit 1; }
cut -c1-300 gpurun_out/pairs_valu_${TAG}.json
echo "== rocprof dense" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dense_${TAG} -o run --output-format csv -- python3 bench.py --workload dense --steps 5 --warmup 2 > gpurun_out/prof_dense_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_dense_${TAG}.log; exit 1; }
find gpurun_out/prof_dense_${TAG} -name "*kernel_stats.csv"
