#!/bin/bash
# GPU parity tests, the default bench, and a rocprofv3 kernel trace of OVERLAPPED steps (the
# timed region's 4 streams), so scripts/overlap_report.py can show which kernels co-execute.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03a}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_${TAG}.log
fi
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
tail -c 400 gpurun_out/bench_${TAG}.json
echo "== overlapped kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --hard-steps 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/trace_${TAG}.log 2>&1 || { tail -20 gpurun_out/trace_${TAG}.log; exit 1; }
find gpurun_out/trace_${TAG} -name "*.csv"
