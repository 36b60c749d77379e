#!/bin/bash
# single-pair latency: GPU suite (SKIP_TESTS=1 skips it), then the latency per sampler latency mode
# (--ctx-option sampler_lat = 0 / 1 / 2; host-timed) and a kernel trace of each:  TAG=r05x bash scripts/dev/gpu_latency.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05p}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -8 | tee gpurun_out/pytest_gpu_$TAG.log || exit 1
fi
for m in 0 1 2; do
  timeout -k 10 300 python scripts/latency_probe.py --runs 20 --ctx-option sampler_lat=$m > gpurun_out/latency_host_${TAG}_lat$m.json 2>> gpurun_out/latency_$TAG.err || exit 1
  echo "lat$m $(cat gpurun_out/latency_host_${TAG}_lat$m.json)"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lat_${TAG}_$m -o run --output-format csv -- python3 scripts/latency_probe.py --runs 20 --ctx-option sampler_lat=$m > gpurun_out/lat_${TAG}_$m.log 2>&1 || exit 1
  python scripts/latency_probe.py --report $(find gpurun_out/lat_${TAG}_$m -name "*kernel_trace.csv" | head -1) --runs 20 > gpurun_out/latency_trace_${TAG}_$m.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/latency_trace_${TAG}_$m.json'));print('span',d['span_us_median'],'sampler',d['kernels_us_in_median_run'].get('sampler_kernel'))"
done
