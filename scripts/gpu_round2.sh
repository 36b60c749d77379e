#!/bin/bash
# Round-2 artifacts on one MI355X: GPU parity tests, the default bench (CPU baseline + parity of
# the timed workload), rocprofv3 kernel-trace --stats of the bench's serial profile pass, PMC
# passes for HBM bytes (FETCH_SIZE, WRITE_SIZE) and one SQ pass (VALU / LDS instruction counts
# per kernel), each in its own run.  Summaries: scripts/pmc_summarize.py in the container.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02c}
PROF="python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 ${BENCH_ARGS}"
if [ -z "$SKIP_TESTS" ]; then
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
fi
echo "== bench" && timeout -k 10 600 python bench.py --profile-tag ${TAG} ${BENCH_ARGS} ${BENCH_CPU} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
tail -c 400 gpurun_out/bench_${TAG}.json
echo "== rocprofv3 kernel-trace stats" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- ${PROF} > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
[ -n "$SKIP_PMC" ] && exit 0
echo "== pmc FETCH_SIZE" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv -- ${PROF} > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
echo "== pmc WRITE_SIZE" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run --output-format csv -- ${PROF} > gpurun_out/pmc_write_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
echo "== pmc SQ" && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmc_sq_${TAG} -o run --output-format csv -- ${PROF} > gpurun_out/pmc_sq_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_sq_${TAG}.log; exit 1; }
echo done
