#!/bin/bash
# one-off GPU call: round artifacts (tests, bench, rocprof stats, FETCH/WRITE PMC), the SQ
# counters of every kernel of a 192-pair step, and configs[2]'s whole workload on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03e bash scripts/gpu_round_artifacts.sh || exit 1
echo "== SQ pass" && PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM" timeout -k 10 400 bash scripts/gpu_pmc_kernel.sh || exit 1
echo "== configs[2]: 1024 pairs x 2048 kpts" && timeout -k 10 600 python bench.py --kpts 2048 --pairs 1024 --steps 3 --warmup 1 --hard-steps 0 --worst-steps 0 > gpurun_out/bench_r03e_configs2.json 2> gpurun_out/bench_r03e_configs2.err || { tail -20 gpurun_out/bench_r03e_configs2.err; exit 1; }
tail -c 400 gpurun_out/bench_r03e_configs2.json
