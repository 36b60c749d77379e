#!/bin/bash
# sampler split replay: the GPU suite, the sampler / end-to-end tests with the split forced on
# (ERP_SAMPLER_SPLIT=1, every launch whose bitmaps fit), single-pair latency + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05s}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
ERP_SAMPLER_SPLIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sampler or sample or full or find or overlap or fixture" > gpurun_out/pytest_split_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_split_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_split_$TAG.log
for v in 0 1; do
  ERP_SAMPLER_SPLIT=$v timeout -k 10 120 python scripts/latency_probe.py --runs 30 > gpurun_out/lat_split${v}_$TAG.json || exit 1
  ERP_SAMPLER_SPLIT=$v timeout -k 10 120 python scripts/latency_probe.py --runs 30 --graph > gpurun_out/lat_split${v}g_$TAG.json || exit 1
  echo "split=$v $(cat gpurun_out/lat_split${v}_$TAG.json) $(cat gpurun_out/lat_split${v}g_$TAG.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lat_$TAG -o run --output-format csv -- python3 scripts/latency_probe.py --runs 20 > gpurun_out/lat_$TAG.log 2>&1 || exit 1
python scripts/latency_probe.py --report $(find gpurun_out/lat_$TAG -name "*kernel_trace.csv" | head -1) --runs 20 > gpurun_out/latency_trace_$TAG.json || exit 1
head -c 1200 gpurun_out/latency_trace_$TAG.json
