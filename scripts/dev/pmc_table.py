#!/usr/bin/env python3
"""Per-kernel mean counter values of rocprofv3 --pmc output dirs (dev)."""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_summarize import short  # noqa: E402

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            k = short(row["Kernel_Name"])
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row["Dispatch_Id"])
    for k, v in sorted(acc.items(), key=lambda kv: -max(kv[1].values())):
        if k.startswith("__amd"):
            continue
        n = len(disp[k])
        print(f"{k:32s} n={n:3d} " + " ".join(f"{c}={x / n:.3g}" for c, x in sorted(v.items())))
