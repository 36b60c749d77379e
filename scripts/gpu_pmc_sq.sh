#!/bin/bash
# SQ counters per kernel for one short bench run (one --pmc pass, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS} \
  -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pairs ${1:-8} > gpurun_out/pmc_sq.log 2>&1
rc=$?
tail -3 gpurun_out/pmc_sq.log
find gpurun_out/pmc_sq -name "*.csv" | head
exit $rc
