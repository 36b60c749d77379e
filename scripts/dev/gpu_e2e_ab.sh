#!/bin/bash
# SURF / e2e A/B of development libraries: the SURF + do_all GPU tests on the in-tree library,
# then per library ROUNDS e2e bench lines and one rocprofv3 kernel-stats pass.
#   TAG=r06ae LIBS="base icol" bash scripts/dev/gpu_e2e_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r06ae}; LIBS=${LIBS:-base}; ROUNDS=${ROUNDS:-2}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "${TEST_K:-surf or do_all or e2e or real}" > gpurun_out/pytest_e2e_${TAG}.log 2>&1 \
  || { tail -30 gpurun_out/pytest_e2e_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_e2e_${TAG}.log
for r in $(seq 1 $ROUNDS); do for v in $LIBS; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 300 python bench.py --workload e2e --steps 8 \
    --warmup 2 > gpurun_out/e2e_${TAG}_$v$r.json 2> gpurun_out/e2e_${TAG}_$v$r.err || { tail -20 gpurun_out/e2e_${TAG}_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/e2e_${TAG}_$v$r.json'));print(round(d['value'],1), round(d['ms_per_step'],3))")"
done; done
for v in $LIBS; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/prof_e2e_${TAG}_$v -o run --output-format csv -- python3 bench.py --workload e2e --steps 4 \
    --warmup 1 > gpurun_out/prof_e2e_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/prof_e2e_${TAG}_$v.log; exit 1; }
done
echo done
