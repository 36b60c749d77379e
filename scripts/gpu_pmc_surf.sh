#!/bin/bash
# SQ / LDS / fetch counters per SURF kernel over the SURF timing probe (separate --pmc passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES FETCH_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc_surf$i -o run --output-format csv -- python3 scripts/dev/surf_prof.py > gpurun_out/pmc_surf$i.log 2>&1 || { tail -5 gpurun_out/pmc_surf$i.log; exit 1; }
done
