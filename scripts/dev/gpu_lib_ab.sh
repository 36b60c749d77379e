#!/bin/bash
# in-tree library (B) against scripts/dev/libs/base (A): matcher tests on B, bench stage times
# (two rounds) and the matcher kernels' FETCH / WRITE (separate PMC passes, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=scripts/dev/libs/base/liberp_match.so
B=erp_match_eightpoint_test_amd/lib/liberp_match.so
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TEST_K:-match or knn or filter or fixture or full}" > gpurun_out/pytest_ab.log 2>&1 || { tail -20 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for r in 1 2; do for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  ERP_LIB_PATH=$L timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --hard-steps 0 --worst-steps 0 > gpurun_out/bench_ab_$v$r.json 2> gpurun_out/bench_ab_$v$r.err || { tail -20 gpurun_out/bench_ab_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/bench_ab_$v$r.json'));s=d['stages_ms_serial_step'];print(round(d['value']), round(d['ms_per_step'],2), 'filter', s['knn2_filter'], 'rescore', s['knn2_rescore'])")"
done; done
for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    ERP_LIB_PATH=$L timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_ab_${v}_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 1 --pairs 128 --streams 1 > gpurun_out/pmc_ab_${v}_$c.log 2>&1 || { tail -5 gpurun_out/pmc_ab_${v}_$c.log; exit 1; }
  done
done
echo done
