#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 counter_collection.csv files (sum per dispatch, mean over
dispatches).  usage: pmc_table.py DIR [DIR ...] [--kernels substr,substr]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
filt = None
for a in sys.argv[1:]:
    if a.startswith("--kernels="):
        filt = a.split("=", 1)[1].split(",")
acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for d in args:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            m = re.search(r"([A-Za-z0-9_]+_kernel(?:<[^>]*>)?)", row["Kernel_Name"])
            k = m.group(1) if m else row["Kernel_Name"][:40]
            acc[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
for k, cs in sorted(acc.items()):
    if filt and not any(f in k for f in filt):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v.values()) / len(v):16.4g}")
