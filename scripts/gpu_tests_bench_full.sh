#!/bin/bash
# GPU parity tests (all), then the default bench WITH the CPU baseline + parity check
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r02}
echo "== gpu tests" && timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_${TAG}.log
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
print("roofline", d["roofline"])
print("cpu", d["cpu_baseline"])
print("parity", d["check"]["parity"])
print("stages", {k: round(v, 3) for k, v in d["stages_ms_serial_step"].items()})
PY
