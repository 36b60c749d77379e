#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== bench full" && timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1; rc=$?; tail -2 gpurun_out/bench_full.log; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== rocprof" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1; rc=$?; tail -3 gpurun_out/rocprof.log; echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
