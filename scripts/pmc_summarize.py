#!/usr/bin/env python3
"""Turn rocprofv3 outputs of one round into the committed summaries under profiles/.

  python scripts/pmc_summarize.py --tag r01c --stats gpurun_out/prof_r01c \
      --fetch gpurun_out/pmc_fetch_r01c --write gpurun_out/pmc_write_r01c

* copies the `--kernel-trace --stats` kernel table to profiles/<tag>_kernel_stats.csv;
* from the two separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (kernel trace only) it
  writes profiles/<tag>_pmc.json (mean per dispatch, every kernel) and, for every pipeline
  stage, profiles/<tag>_pmc_<stage>.json with `hbm_bytes_per_launch`, which bench.py reports as
  roofline.traffic.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]": rocprofv3's FETCH_SIZE and
WRITE_SIZE are kilobytes (counter_defs.yaml: ".../1024"); on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so bytes = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# pipeline stage -> kernel symbol (short name; since r02 the matcher has one MFMA pass)
STAGE_KERNEL = {
    "knn2_filter": "knn2_filter_kernel",
    "knn2_rescore": "knn2_rescore_kernel", "knn2_merge": "knn2_merge_kernel",
    "jump_prep": "jump_prep_kernel",
    "windows": "sampler_window_kernel", "sampler": "sampler_kernel<0>", "gram": "gram_mfma_kernel<2>",
    "eigen": "estimate_lite_kernel<false>", "valid_compact": "valid_place_kernel",
    "consensus_bounds": "consensus_bounds_kernel", "consensus_select": "consensus_select_kernel",
    "consensus_refine": "consensus_refine_kernel", "consensus_rows": "consensus_rows_kernel",
    "consensus_final": "consensus_final_kernel",
}


def short(name: str) -> str:
    """'erp::(anonymous namespace)::knn2_filter_kernel<1>(float const*, ...)' or its mangled form
    '_ZN3erp12_GLOBAL__N_118knn2_filter_kernelILi1EEEv...' -> 'knn2_filter_kernel<1>'"""
    m = re.search(r"([a-z][a-z0-9_]*_kernel)(?:IL([ib])(\d+)E)?", name) if name.startswith("_Z") else None
    if m:
        if not m.group(2):
            return m.group(1)
        v = m.group(3) if m.group(2) == "i" else ("true" if m.group(3) == "1" else "false")
        return f"{m.group(1)}<{v}>"
    m = re.search(r"([A-Za-z0-9_]+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0].split("::")[-1]


def find_csv(d: str, suffix: str) -> str | None:
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    return hits[0] if hits else None


def per_kernel_counter(d: str, counter: str) -> dict:
    path = find_csv(d, "counter_collection.csv")
    if path is None:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(float))  # kernel -> dispatch -> value
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq", help="dir of an SQ counter pass -> profiles/<tag>_sq.txt")
    ap.add_argument("--draws", type=float, default=0.0,
                    help="rand() draws per sampler launch (per-draw VALU / LDS in the SQ table)")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    if a.stats:
        src = find_csv(a.stats, "kernel_stats.csv")
        if src is None:
            raise SystemExit(f"no kernel_stats.csv under {a.stats}")
        shutil.copy(src, os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
        print("stats ->", os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    if a.fetch and a.write:
        fetch = per_kernel_counter(a.fetch, "FETCH_SIZE")
        write = per_kernel_counter(a.write, "WRITE_SIZE")
        table = {}
        for k in sorted(set(fetch) | set(write)):
            fk, nf = fetch.get(k, (0.0, 0))
            wk, nw = write.get(k, (0.0, 0))
            table[k] = {"fetch_size_kb_mean": fk, "write_size_kb_mean": wk,
                        "dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
                        "hbm_bytes_per_launch": 2 * 1024 * fk + 1024 * wk}
        note = ("bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (KB counters; gfx950 FETCH_SIZE "
                "halving, MI355X_MICROARCH.md 'HBM [CDNA4]'); separate --pmc passes, kernel "
                "trace only; mean over the dispatches of each pass")
        with open(os.path.join(prof, f"{a.tag}_pmc.json"), "w") as f:
            json.dump({"note": note, "kernels": table}, f, indent=1)
        for stage, kern in STAGE_KERNEL.items():
            if kern in table:
                with open(os.path.join(prof, f"{a.tag}_pmc_{stage}.json"), "w") as f:
                    json.dump({"stage": stage, "kernel": kern, "note": note, **table[kern]}, f,
                              indent=1)
        for k, v in sorted(table.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
            print(f"{k:40s} {v['hbm_bytes_per_launch'] / 1e6:10.3f} MB/launch")
    if a.sq:
        path = find_csv(a.sq, "counter_collection.csv")
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row["Dispatch_Id"])
        lines = ["# SQ counters per kernel: mean per dispatch (rocprofv3 --pmc, one pass, kernel trace",
                 "# only; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles, SQ_INSTS_* in",
                 "# wave-instructions, summed over the chip)"]
        for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            if k.startswith("__amd"):
                continue
            n = len(disp[k])
            lines.append(f"{k:36s} dispatches={n:3d} " +
                         " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items())))
        smp = acc.get("sampler_kernel<0>")
        if smp and a.draws > 0:
            n = len(disp["sampler_kernel<0>"])
            wd = a.draws / 64.0  # wave-level draws per launch
            lines.append(f"# sampler: {a.draws:.4g} draws per launch -> "
                         f"{smp['SQ_INSTS_VALU'] / n / wd:.2f} VALU and "
                         f"{smp['SQ_INSTS_LDS'] / n / wd:.2f} LDS wave-instructions per draw")
        with open(os.path.join(prof, f"{a.tag}_sq.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
        print("\n".join(lines[-3:]))


if __name__ == "__main__":
    main()
