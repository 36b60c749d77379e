#!/usr/bin/env python3
"""Single-pair latency of the batch pipeline (configs[1] "Single ERP pair": one 4096 x 4096
pair, 10k iterations, a batch of 1 through erp_pair_batch_run), host-timed with a sync around
each run -- and, under `rocprofv3 --kernel-trace`, the trace of the same runs, which
latency_report() splits into kernel time, the gaps between kernels and the host time around them.

    python scripts/latency_probe.py [--runs 20] [--graph]         (on the GPU box)
    rocprofv3 --kernel-trace -d gpurun_out/lat -o run --output-format csv -- \
        python3 scripts/latency_probe.py --runs 20
    python scripts/latency_probe.py --report gpurun_out/lat/.../run_kernel_trace.csv --runs 20
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def probe(runs: int, kpts: int, iters: int, seed: int, graphs: bool = False, opts=None) -> dict:
    import torch

    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, synth
    dev = torch.device("cuda:0")
    p = synth.make_pair(seed, n_kpts=kpts)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    args = (t(p["desc_l"]), t(p["desc_r"]), t(p["kp_l"]), t(p["kp_r"]),
            t(np.array([0, kpts], np.int64)), t(np.array([0, kpts], np.int64)),
            t(np.array([p["W"]], np.int32)), t(np.array([p["H"]], np.int32)), kpts, kpts)
    ctx = Context(0)
    for kv in opts or []:  # --ctx-option name=value (erp_ctx_set_option)
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ctx.set_graphs(graphs)  # erp_ctx_set_graphs: replay the captured launch sequence
    run = PairBatchRunner(ctx=ctx, iters=iters, reuse_outputs=True)
    st = torch.cuda.Stream(dev)  # (graphs need a capturable, non-NULL stream)
    run.reserve(1, kpts, kpts)
    for _ in range(3):
        run.run(*args, stream=st.cuda_stream)
    torch.cuda.synchronize()
    host, enq = [], []
    for _ in range(runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.run(*args, stream=st.cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        host.append(t2 - t0)
    return {"single_pair_ms_median": float(np.median(host)) * 1e3,
            "enqueue_ms_median": float(np.median(enq)) * 1e3, "runs": runs, "kpts": kpts,
            "iters": iters, "hip_graph": graphs}


def _short(n: str) -> str:
    m = re.search(r"namespace\)::([A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:40]


def latency_report(trace_csv: str, runs: int) -> dict:
    """the last `runs` pipeline runs of the trace (a run = the dispatches from knn2_split to
    consensus_final): per run the span first-start -> last-end, the kernel time inside it and
    the gaps; medians over the runs, plus the kernels by total time in the median run"""
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(_short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
           for r in rows]
    starts = [i for i, x in enumerate(seq) if x[0] == "knn2_split_kernel"]
    ends = [i for i, x in enumerate(seq) if x[0] == "consensus_final_kernel"]
    out = []
    for s in starts[-runs:]:
        e = next(i for i in ends if i > s)
        part = seq[s:e + 1]
        span = (part[-1][2] - part[0][1]) / 1e3
        busy = sum(b - a for _, a, b in part) / 1e3
        out.append({"span_us": span, "kernel_us": busy, "gaps_us": span - busy,
                    "dispatches": len(part), "kernels": part})
    med = sorted(out, key=lambda r: r["span_us"])[len(out) // 2]
    by = {}
    for n, a, b in med["kernels"]:
        by[n] = by.get(n, 0.0) + (b - a) / 1e3
    return {"runs": len(out), "span_us_median": med["span_us"],
            "kernel_us_median": med["kernel_us"], "gaps_us_median": med["gaps_us"],
            "dispatches": med["dispatches"],
            "gap_per_dispatch_us": med["gaps_us"] / max(med["dispatches"] - 1, 1),
            "kernels_us_in_median_run": dict(sorted(by.items(), key=lambda kv: -kv[1]))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--kpts", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=20200423)
    ap.add_argument("--graph", action="store_true", help="erp_ctx_set_graphs: HIP-graph replay")
    ap.add_argument("--ctx-option", action="append", default=[],
                    help="name=value: erp_ctx_set_option on the context (e.g. sampler_lat=1)")
    ap.add_argument("--report", default=None, help="rocprofv3 run_kernel_trace.csv to split")
    ap.add_argument("--host-json", default=None, help="merge this probe() record into --report")
    a = ap.parse_args()
    if a.report:
        r = latency_report(a.report, a.runs)
        if a.host_json and os.path.exists(a.host_json):
            r["host"] = json.load(open(a.host_json))
        print(json.dumps(r, indent=1))
        return
    print(json.dumps(probe(a.runs, a.kpts, a.iters, a.seed, a.graph, a.ctx_option)))


if __name__ == "__main__":
    main()
