#!/bin/bash
# SQ counters: the single-pair latency path (two passes) and the 128-pair serial profile pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05n}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  -d gpurun_out/sqlat_a_$TAG -o run --output-format csv -- python3 scripts/latency_probe.py --runs 5 > gpurun_out/sqlat_a_$TAG.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/sqlat_b_$TAG -o run --output-format csv -- python3 scripts/latency_probe.py --runs 5 > gpurun_out/sqlat_b_$TAG.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
  -d gpurun_out/sqk_$TAG -o run --output-format csv -- python3 bench.py --steps 0 --warmup 1 --pairs 128 --streams 1 --no-cpu-baseline > gpurun_out/sqk_$TAG.log 2>&1 || exit 1
find gpurun_out/sqlat_a_$TAG gpurun_out/sqlat_b_$TAG gpurun_out/sqk_$TAG -name "*.csv"
