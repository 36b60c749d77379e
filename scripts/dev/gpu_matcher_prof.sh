#!/bin/bash
# matcher probe + correctness probe + SQ / TCC counters of the filter kernel (dev)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-mp}
timeout -k 10 100 ./scripts/dev/matcher_probe 128 4096 > gpurun_out/mprobe_${TAG}.txt 2>&1 && timeout -k 10 60 ./scripts/dev/matcher_probe 1 16384 >> gpurun_out/mprobe_${TAG}.txt 2>&1 && cat gpurun_out/mprobe_${TAG}.txt || exit 1
[ -n "$NO_DBG" ] || { timeout -k 10 200 python scripts/dev/matcher_debug.py > gpurun_out/mdbg_${TAG}.txt 2>&1; tail -2 gpurun_out/mdbg_${TAG}.txt; }
[ -n "$NO_PMC" ] && exit 0
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/mpmc_sq_${TAG} -o run --output-format csv -- ./scripts/dev/matcher_probe 128 4096 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum -d gpurun_out/mpmc_b_${TAG} -o run --output-format csv -- ./scripts/dev/matcher_probe 128 4096 > /dev/null 2>&1 || echo "pmc pass b failed"
echo done
