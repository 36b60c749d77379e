#!/bin/bash
# quick GPU loop: parity tests (fail-fast) + full-size bench (B=8 and B=32) without the CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for B in 8 32; do
  echo "== bench B=$B" && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pairs $B > gpurun_out/bench_b$B.log 2>&1; rc=$?; tail -1 gpurun_out/bench_b$B.log | cut -c1-200; echo "bench rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
