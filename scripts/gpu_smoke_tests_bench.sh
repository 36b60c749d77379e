#!/bin/bash
# first GPU pass: smoke, parity tests, a small bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== bench small" && timeout -k 10 300 python bench.py --pairs 2 --iters 2000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1; rc=$?; tail -3 gpurun_out/bench_small.log; echo "bench rc=$rc"
exit $rc
