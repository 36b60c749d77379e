#!/bin/bash
# SQ counters per kernel over the bench's profile-only run (one --pmc pass, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS} \
  -d gpurun_out/pmc_k -o run --output-format csv -- python3 bench.py --steps 0 --warmup 1 --pairs 128 --streams 1 --no-cpu-baseline > gpurun_out/pmc_k.log 2>&1
rc=$?
tail -2 gpurun_out/pmc_k.log
exit $rc
