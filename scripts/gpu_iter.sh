#!/bin/bash
# iteration loop on one MI355X: GPU parity tests (fail-fast), then the default bench without the
# CPU baseline; prints the per-stage times.  Extra args go to bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== bench" && timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_iter.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_iter.log; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_iter.log").read().strip().splitlines()[-1])
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3), "roof", d["roofline"] and {k: d["roofline"][k] for k in ("kernel", "frac")})
print({k: round(v, 3) for k, v in sorted(d["stages_ms_serial_step"].items(), key=lambda kv: -kv[1])})
c = d["check"]; print("ok", c["all_status_ok"], "err", c["mean_abs_euler_err_deg_max"], "surv max", max(c["consensus_survivors"]))
PY
