#!/bin/bash
# GPU parity tests, then the default bench without the CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "== bench" && timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_dev.json 2> gpurun_out/bench_dev.err || { tail -20 gpurun_out/bench_dev.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_dev.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
print("roofline", d["roofline"])
print("stages", {k: round(v, 3) for k, v in d["stages_ms_serial_step"].items()})
print("check", {k: d["check"][k] for k in ("all_status_ok", "mean_abs_euler_err_deg_max", "K_mean")})
PY
