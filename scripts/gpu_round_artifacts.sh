#!/bin/bash
# Round artifacts on one MI355X: GPU parity tests, the default bench (with the CPU baseline),
# a rocprofv3 kernel-trace --stats run of the bench workload, and two PMC passes (FETCH_SIZE,
# WRITE_SIZE; separate passes, kernel trace only) for the HBM traffic per kernel.  The profiled
# runs use --steps 0 --warmup 2: bench.py then runs only its serial profile pass (the default
# step's 3 sub-batches one after the other), so rocprof sees exactly the launches whose
# durations bench.py measures with HIP events for the roofline (the timed step overlaps them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "== bench (default, with cpu baseline)" && timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
tail -c 600 gpurun_out/bench_${TAG}.json
echo "== rocprofv3 kernel-trace stats" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
echo "== pmc FETCH_SIZE" && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
echo "== pmc WRITE_SIZE" && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 > gpurun_out/pmc_write_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} gpurun_out/pmc_fetch_${TAG} gpurun_out/pmc_write_${TAG} -name "*.csv" | head -20
# then, in the container: python scripts/pmc_summarize.py --tag $TAG --stats gpurun_out/prof_$TAG \
#   --fetch gpurun_out/pmc_fetch_$TAG --write gpurun_out/pmc_write_$TAG   (-> profiles/)
