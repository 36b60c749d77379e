#!/bin/bash
# A/B on one box: optional GPU test subset (TEST_K), then the default bench (no CPU baseline) once
# per value in VALUES of a context route option OPT (bench.py --ctx-option, erp_ctx_set_option)
# or of an environment variable KNOB (the Python side's ERP_LIB_PATH: a variant library);
# prints value, step, stages.
#   TAG=r06x OPT=lip2 VALUES="1 0" TEST_K="consensus" bash scripts/gpu_ab.sh
#   TAG=r06y KNOB=ERP_LIB_PATH VALUES="a.so b.so" bash scripts/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "${TEST_K:-}" ]; then
  echo "== gpu tests -k $TEST_K" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "$TEST_K" > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_${TAG}.log
fi
N=0
for V in ${VALUES:-0 1}; do
  N=$((N + 1))
  F=gpurun_out/bench_${TAG}_${N}_$(echo "$V" | tr '/' '_')
  if [ -n "${OPT:-}" ]; then PRE=""; ARM="--ctx-option $OPT=$V"; else PRE="$KNOB=$V"; ARM=""; fi
  echo "== bench ${OPT:-$KNOB}=$V" && env $PRE timeout -k 10 400 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 $ARM ${BENCH_ARGS:-} > $F.json 2> $F.err || { tail -20 $F.err; exit 1; }
  python scripts/bench_summary.py $F.json 2>/dev/null || python -c "import json;d=json.load(open('$F.json'));print(d['value'], d['ms_per_step'], {k:round(v,2) for k,v in d['stages_ms_serial_step'].items() if v>0.3})"
done
