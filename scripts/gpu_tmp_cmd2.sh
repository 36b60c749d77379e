#!/bin/bash
# one-off GPU call: the bench (with the CPU baseline and parity) plus rocprof stats and the two
# PMC passes under TAG, without the test suite (run on the same code by the previous call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03n}
echo "== bench" && timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
tail -c 300 gpurun_out/bench_${TAG}.json
echo "== rocprofv3 kernel-trace stats" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
echo "== pmc FETCH_SIZE" && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
echo "== pmc WRITE_SIZE" && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/pmc_write_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
echo done
