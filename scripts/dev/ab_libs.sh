#!/bin/bash
# same-box A/B of development libraries (scripts/dev/libs/<name>/liberp_match.so, built with
# _build.build(lib_path=..., defines=[...])): the GPU tests matching TEST_K on each variant, then
# ROUNDS alternating default benches reporting one stage's serial time.
#   LIBS="base ring4" STAGE=gram TEST_K="find or gram" bash scripts/dev/ab_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
LIBS=${LIBS:-base}; STAGE=${STAGE:-gram}; ROUNDS=${ROUNDS:-2}
for v in $LIBS; do
  [ "$v" = base ] && continue
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TEST_K:-find}" > gpurun_out/ab_t_$v.log 2>&1 \
    || { tail -20 gpurun_out/ab_t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab_t_$v.log)"
done
for r in $(seq 1 $ROUNDS); do for v in $LIBS; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 \
    --warmup 2 --hard-steps 0 --worst-steps 0 > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err \
    || { tail -20 gpurun_out/ab_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));s=d['stages_ms_serial_step'];print(round(d['value']), round(d['ms_per_step'],2), '$STAGE', round(s['$STAGE'],3), 'rescore', round(s['knn2_rescore'],3))")"
done; done
