#!/bin/bash
# The consensus list kernels' grids and the folded memsets: GPU tests on the in-tree library,
# then, per development library (scripts/dev/libs/<name>), a rocprofv3 kernel-stats pass of the
# bench's serial profile step and ROUNDS alternating short benches.
#   TAG=r06m LIBS="base cap fold" bash scripts/dev/gpu_list_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r06m}; LIBS=${LIBS:-"base cap fold"}; ROUNDS=${ROUNDS:-2}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  ERP_PARITY_OUT=gpurun_out/parity_${TAG}.json timeout -k 10 900 python -u -m pytest tests -x -v -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_${TAG}.log
fi
for v in $LIBS; do
  L=scripts/dev/libs/$v/liberp_match.so
  ERP_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$v -o run \
    --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 \
    > gpurun_out/prof_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_$v.log; exit 1; }
done
for r in $(seq 1 $ROUNDS); do for v in $LIBS; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 400 python bench.py --no-cpu-baseline \
    --steps 10 --warmup 3 --hard-steps 0 --worst-steps ${WORST_STEPS:-0} > gpurun_out/ab_${TAG}_$v$r.json \
    2> gpurun_out/ab_${TAG}_$v$r.err || { tail -20 gpurun_out/ab_${TAG}_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_$v$r.json'));s=d['stages_ms_serial_step'];w=d.get('worst_case') or {};print(round(d['value']), round(d['ms_per_step'],2), d['exact'], 'cons', round(sum(v for k,v in s.items() if k.startswith('consensus')),3), 'bounds', round(s['consensus_bounds'],3), 'filter', round(s['knn2_filter'],3), 'worst', w.get('value'))")"
done; done
echo done
