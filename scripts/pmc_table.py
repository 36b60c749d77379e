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
            nm = row["Kernel_Name"]
            m = re.search(r"([a-z][a-z0-9_]*_kernel)(?:IL([ib])(\d+)E)?", nm) if nm.startswith("_Z") else None
            if m:
                v = "" if not m.group(2) else (m.group(3) if m.group(2) == "i" else ("true" if m.group(3) == "1" else "false"))
                k = m.group(1) + (f"<{v}>" if v else "")
            else:
                m = re.search(r"([A-Za-z0-9_]+_kernel(?:<[^>]*>)?)", nm)
                k = m.group(1) if m else nm[:40]
            acc[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
for k, cs in sorted(acc.items()):
    if filt and not any(f in k for f in filt):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v.values()) / len(v):16.4g}")
