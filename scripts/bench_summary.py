#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (value, roofline, stage times, fractions)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"] and round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3))
r = d.get("roofline") or {}
print("roofline", r.get("kernel"), r.get("frac") and round(r["frac"], 3), r.get("avg_launch_ms") and round(r["avg_launch_ms"], 3))
print("stages", {k: round(v, 3) for k, v in sorted(d.get("stages_ms_serial_step", {}).items(), key=lambda kv: -kv[1]) if v})
print("fracs", {k: round(v["frac"], 3) for k, v in d.get("roofline_stages", {}).items()})
c = d.get("cpu_baseline")
if c:
    print("cpu", round(c["value"], 3), c["unit"], "1core", round(c.get("value_1core", 0), 3))
print("parity", (d.get("check") or {}).get("parity"), "latency", d.get("latency"))
