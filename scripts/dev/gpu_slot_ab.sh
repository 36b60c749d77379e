#!/bin/bash
# round 5: candidate slot layout A/B -- (interleaved, tile-index array) vs ([list][slot], embedded
# index): matcher tests on the variant, bench stage times (two rounds) and the matcher kernels'
# FETCH / WRITE (separate PMC passes, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=erp_match_eightpoint_test_amd/lib/liberp_match.so
B=scripts/dev/libs/li0/liberp_match.so
ERP_LIB_PATH=$B ERP_CAND_TILE_ARRAY=0 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k 'match or knn or filter or fixture' > gpurun_out/pytest_li0.log 2>&1 || { tail -20 gpurun_out/pytest_li0.log; exit 1; }
tail -1 gpurun_out/pytest_li0.log
for r in 1 2; do
for v in A B; do
  if [ $v = A ]; then L=$A; T=1; else L=$B; T=0; fi
  ERP_LIB_PATH=$L ERP_CAND_TILE_ARRAY=$T timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --hard-steps 0 --worst-steps 0 > gpurun_out/bench_li_$v$r.json 2> gpurun_out/bench_li_$v$r.err || { tail -20 gpurun_out/bench_li_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/bench_li_$v$r.json'));s=d['stages_ms_serial_step'];print(round(d['value']), s['knn2_filter'], s['knn2_rescore'])")"
done
done
for v in A B; do
  if [ $v = A ]; then L=$A; T=1; else L=$B; T=0; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    ERP_LIB_PATH=$L ERP_CAND_TILE_ARRAY=$T timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_li_${v}_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 1 --pairs 128 --streams 1 > gpurun_out/pmc_li_${v}_$c.log 2>&1 || { tail -5 gpurun_out/pmc_li_${v}_$c.log; exit 1; }
  done
done
echo done
