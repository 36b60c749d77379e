#!/bin/bash
# quick loop: all GPU tests, the configs[4] bench and the default bench (no CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "== manual" && timeout -k 10 300 python bench.py --workload manual --steps 3 --warmup 1 > gpurun_out/manual.json 2> gpurun_out/manual.err || { tail -20 gpurun_out/manual.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/manual.json'));print(round(d['ms_per_step'],3), d['check'], {k:round(v,3) for k,v in d['stages_ms_rank0'].items()})"
echo "== pairs" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pairs.json 2> gpurun_out/pairs.err || { tail -20 gpurun_out/pairs.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pairs.json'));print(round(d['value']), d['latency'], d['check']['all_status_ok'], {k:round(v/3,3) for k,v in sorted(d['stages_ms_serial_step'].items(),key=lambda x:-x[1])})"
