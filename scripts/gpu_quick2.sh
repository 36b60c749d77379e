#!/bin/bash
# quick loop: a subset of GPU tests (PYTEST_K) then the default bench without the CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
echo "== gpu tests ($PYTEST_K)" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "${PYTEST_K:-parity}" > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -50 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3))
r = d["roofline"]; print("roofline", r["kernel"], round(r["frac"], 3), round(r["avg_launch_ms"], 3))
print("stages", {k: round(v, 3) for k, v in sorted(d["stages_ms_serial_step"].items(), key=lambda kv: -kv[1])})
print("fracs", {k: round(v["frac"], 3) for k, v in d["roofline_stages"].items()})
PY
