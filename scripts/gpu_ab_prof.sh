#!/bin/bash
# scripts/gpu_ab.sh, then a rocprofv3 kernel-trace --stats pass of the bench's serial profile
# step (--steps 0) per knob value, so per-kernel times can be compared between the arms.
#   TAG=r06x OPT=lip2 VALUES="1 0" TEST_K="consensus" bash scripts/gpu_ab_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_ab.sh || exit 1
for V in ${VALUES:-0 1}; do
  W=$(echo "$V" | tr '/' '_')  # (path-valued knobs: ERP_LIB_PATH variant libraries)
  if [ -n "${OPT:-}" ]; then PRE=""; ARM="--ctx-option $OPT=$V"; else PRE="$KNOB=$V"; ARM=""; fi
  echo "== rocprofv3 ${OPT:-$KNOB}=$V" && env $PRE timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$W -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 $ARM ${BENCH_ARGS:-} > gpurun_out/prof_${TAG}_$W.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_$W.log; exit 1; }
done
find gpurun_out -path "*prof_${TAG}_*" -name "*kernel_stats.csv" | head
