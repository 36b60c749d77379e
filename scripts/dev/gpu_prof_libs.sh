#!/bin/bash
# rocprofv3 kernel-stats pass of the bench's serial profile step per development library
# (scripts/dev/libs/<name>): for timing ablations whose results are wrong (no tests, no bench).
#   TAG=r06r LIBS="base gabl" bash scripts/dev/gpu_prof_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${LIBS:-base}; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/prof_${TAG}_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline \
    --steps 0 --warmup 2 > gpurun_out/prof_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_$v.log; exit 1; }
done
echo done
