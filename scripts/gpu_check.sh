#!/bin/bash
# GPU suite, then the default bench line, then (N > 1 rehearsal) the 2-rank bench on one device.
#   TAG=r06c bash scripts/gpu_check.sh    (SKIP_TESTS=1 / SKIP_BENCH=1 / SKIP_RANKS=1; TEST_K=<-k expr>)
# ERP_PARITY_OUT: the tests' measured parity deviations -> gpurun_out/parity_$TAG.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r06c}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== gpu tests" && ERP_PARITY_OUT=gpurun_out/parity_${TAG}.json timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
    || { tail -40 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_${TAG}.log
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json \
    2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}.json'));print(d['value'],d['ms_per_step'],d['exact'],{k:round(v,2) for k,v in d['stages_ms_serial_step'].items() if v>0.1})"
fi
if [ "${SKIP_RANKS:-0}" != "1" ]; then
  TAG=$TAG bash scripts/gpu_ranks_on_one.sh || exit 1
fi
echo done
