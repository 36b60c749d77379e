#!/bin/bash
# SQ counters of the remap kernels (one --pmc pass, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES \
  -d gpurun_out/pmc_remap_sq -o run --output-format csv -- python3 bench.py --workload remap --steps 2 --warmup 1 \
  > gpurun_out/pmc_remap_sq.log 2>&1 || { tail -5 gpurun_out/pmc_remap_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY \
  -d gpurun_out/pmc_remap_sq2 -o run --output-format csv -- python3 bench.py --workload remap --steps 2 --warmup 1 \
  > gpurun_out/pmc_remap_sq2.log 2>&1 || { tail -5 gpurun_out/pmc_remap_sq2.log; exit 1; }
echo done
