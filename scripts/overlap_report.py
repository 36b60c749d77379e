#!/usr/bin/env python3
"""Which kernels of an OVERLAPPED bench step actually co-execute: reads a rocprofv3
--kernel-trace CSV of `bench.py --steps K --warmup W` (scripts/gpu_overlap_trace.sh).

Phases are split at GPU idle gaps (host synchronisations): the warmup step, the timed steps
(one phase), each sub-batch of the serial profile pass.  Per phase:
  span      first kernel start -> last kernel end (ms)
  sum       the sum of the step's kernel durations (ms): span ~ sum means serial execution
  busy      the union of the kernel intervals (ms): span - busy = GPU idle gaps
  overlap   per pair of kernel names, the time both ran at once (ms), largest first

    python scripts/overlap_report.py gpurun_out/trace_r03a [--json profiles/r03a_overlap.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)", "anon")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    n = n.split("::")[-1]
    return n.replace("_kernel", "")


def load(path: str):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"]), r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    rows.sort(key=lambda x: x[1])
    return rows


def union_ns(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def step_report(rows):
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    ksum = sum(r[2] - r[1] for r in rows)
    busy = union_ns([(r[1], r[2]) for r in rows])
    # pairwise overlap by kernel name (sweep over the sorted events)
    ov = defaultdict(int)
    for i, a in enumerate(rows):
        for b in rows[i + 1:]:
            if b[1] >= a[2]:
                break
            o = min(a[2], b[2]) - max(a[1], b[1])
            if o > 0:
                ov[tuple(sorted((a[0], b[0])))] += o
    # per kernel name: its total time and the part of it during which some other kernel ran
    per = defaultdict(lambda: [0, 0])
    for i, a in enumerate(rows):
        others = [(max(a[1], b[1]), min(a[2], b[2])) for j, b in enumerate(rows)
                  if j != i and b[1] < a[2] and b[2] > a[1]]
        per[a[0]][0] += a[2] - a[1]
        per[a[0]][1] += union_ns(others)
    return {"span_ms": (t1 - t0) / 1e6, "kernel_sum_ms": ksum / 1e6, "busy_ms": busy / 1e6,
            "launches": len(rows),
            "overlap_ms": {f"{a} | {b}": v / 1e6 for (a, b), v in
                           sorted(ov.items(), key=lambda kv: -kv[1])[:25]},
            "per_kernel_ms": {k: {"total": v[0] / 1e6, "co_running": v[1] / 1e6}
                              for k, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}


def phases(rows, gap_ns):
    """split the trace at GPU idle gaps longer than gap_ns (host synchronisations: the warmup
    step, the timed steps, each serial sub-batch, ... become separate phases)"""
    out, cur, end = [], [], 0
    for r in rows:
        if cur and r[1] - end > gap_ns:
            out.append(cur)
            cur = []
        end = r[2] if not cur else max(end, r[2])
        cur.append(r)
    if cur:
        out.append(cur)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--json")
    ap.add_argument("--gap-us", type=float, default=100.0, help="idle gap that splits phases")
    ap.add_argument("--min-launches", type=int, default=20)
    a = ap.parse_args()
    rows = load(a.trace_dir)
    out = {"trace": a.trace_dir, "phases": []}
    for k, ph in enumerate(phases(rows, a.gap_us * 1e3)):
        if len(ph) < a.min_launches:
            continue
        rep = step_report(ph)
        rep["phase"] = k
        out["phases"].append(rep)
        print(f"phase {k}: span {rep['span_ms']:.2f} ms, kernel sum {rep['kernel_sum_ms']:.2f}, "
              f"busy {rep['busy_ms']:.2f}, {rep['launches']} launches")
        for kname, v in list(rep["per_kernel_ms"].items())[:10]:
            print(f"    {kname:28s} {v['total']:7.2f} ms, {v['co_running']:7.2f} with others")
        for pair, v in list(rep["overlap_ms"].items())[:8]:
            print(f"    overlap {pair:44s} {v:7.3f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
