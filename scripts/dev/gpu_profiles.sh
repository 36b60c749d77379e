#!/bin/bash
# the profile half of scripts/gpu_round_artifacts.sh alone (kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate passes, kernel trace only):  TAG=r05f bash scripts/dev/gpu_profiles.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:?TAG}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 --profile-tag $T > gpurun_out/prof_$T.log 2>&1 \
  || { tail -20 gpurun_out/prof_$T.log; exit 1; }
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  d=$([ $c = FETCH_SIZE ] && echo fetch || echo write)
  timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/pmc_${d}_$T -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 --profile-tag $T > gpurun_out/pmc_${d}_$T.log 2>&1 \
    || { tail -20 gpurun_out/pmc_${d}_$T.log; exit 1; }
  echo "$c ok"
done
