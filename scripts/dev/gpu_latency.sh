#!/bin/bash
# round 5: GPU suite, then single-pair latency with and without the small-batch route, and a
# kernel trace of the default
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05e}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -8 | tee gpurun_out/pytest_gpu_$TAG.log || exit 1
fi
timeout -k 10 300 python scripts/latency_probe.py --runs 20 > gpurun_out/latency_host_$TAG.json 2> gpurun_out/latency_$TAG.err && cat gpurun_out/latency_host_$TAG.json &&
ERP_SMALL_BATCH=0 timeout -k 10 300 python scripts/latency_probe.py --runs 20 > gpurun_out/latency_host_prune_$TAG.json 2>> gpurun_out/latency_$TAG.err && cat gpurun_out/latency_host_prune_$TAG.json &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lat_$TAG -o run --output-format csv -- python3 scripts/latency_probe.py --runs 20 > gpurun_out/lat_$TAG.log 2>&1 &&
python scripts/latency_probe.py --report $(find gpurun_out/lat_$TAG -name "*kernel_trace.csv" | head -1) --runs 20 > gpurun_out/latency_trace_$TAG.json && head -c 2500 gpurun_out/latency_trace_$TAG.json
