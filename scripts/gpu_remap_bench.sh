#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01f}
echo "== remap bench" && timeout -k 10 300 python bench.py --workload remap --steps 5 --warmup 2 > gpurun_out/remap_${TAG}.json 2> gpurun_out/remap_${TAG}.err || { tail -20 gpurun_out/remap_${TAG}.err; exit 1; }
cat gpurun_out/remap_${TAG}.json
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_remap_${TAG} -o run --output-format csv -- python3 bench.py --workload remap --steps 3 --warmup 1 > gpurun_out/prof_remap_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_remap_${TAG}.log; exit 1; }
echo "== pmc" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_remap_fetch_${TAG} -o run --output-format csv -- python3 bench.py --workload remap --steps 2 --warmup 1 > gpurun_out/pmc_remap_f.log 2>&1 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_remap_write_${TAG} -o run --output-format csv -- python3 bench.py --workload remap --steps 2 --warmup 1 > gpurun_out/pmc_remap_w.log 2>&1
