#!/bin/bash
# quick GPU loop: parity tests (fail-fast) + full-size bench without the CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== bench" && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?; tail -2 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc
