#!/bin/bash
# GPU parity tests, then an A/B of the standalone sampler + Gram kernels (ERP_FUSE_SAMPLER=0)
# against the fused sampler_gram kernel on one box: the bench and a rocprofv3 kernel trace of
# OVERLAPPED steps for each (scripts/overlap_report.py shows which kernels co-execute).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03a}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${TEST_ARGS:-} > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_${TAG}.log
fi
for F in ${FUSE_LIST:-0 1}; do
  echo "== bench fuse=$F" && ERP_FUSE_SAMPLER=$F timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}_f$F.json 2> gpurun_out/bench_${TAG}_f$F.err || { tail -20 gpurun_out/bench_${TAG}_f$F.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_f$F.json'));print(d['value'], d['ms_per_step'], d['overlap'], d['check']['parity'] and d['check']['parity']['all_equal'])"
  echo "== overlapped kernel trace fuse=$F" && ERP_FUSE_SAMPLER=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_f$F -o run --output-format csv -- python3 bench.py --no-cpu-baseline --hard-steps 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/trace_${TAG}_f$F.log 2>&1 || { tail -20 gpurun_out/trace_${TAG}_f$F.log; exit 1; }
done
