#!/usr/bin/env python3
"""Print the kernel sequence of one sub-batch from a rocprofv3 kernel trace (run_kernel_trace.csv):
name, duration, VGPRs, LDS bytes, grid -- starting at the last dispatch whose name contains START.
    python scripts/trace_seq.py gpurun_out/prof_x/run_kernel_trace.csv valid_scatter 40
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
start = sys.argv[2] if len(sys.argv) > 2 else "valid_scatter"
count = int(sys.argv[3]) if len(sys.argv) > 3 else 40


def short(n):
    m = re.search(r"namespace\)::([A-Za-z0-9_]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
        r["VGPR_Count"], r["LDS_Block_Size"], r["Grid_Size_X"], r["Grid_Size_Y"]) for r in rows]
idx = [i for i, x in enumerate(seq) if start in x[0]]
s = idx[-1] if idx else 0
for n, d, v, l, gx, gy in seq[s:s + count]:
    print(f"{n:40s} {d:8.1f} us  vgpr {v:>4} lds {l:>6} grid {gx}x{gy}")
