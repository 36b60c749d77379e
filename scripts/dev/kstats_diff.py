"""Per-kernel time per step of two rocprofv3 kernel_stats.csv files (A/B), normalised by the
sampler's launch count (one launch per sub-batch; 6 sub-batches per step)."""
import csv
import re
import sys


def load(f):
    d = {}
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("erp::(anonymous namespace)::", "").replace("void ", "")
        n = re.sub(r"\(.*", "", n)
        t, c = d.get(n, (0.0, 0))
        d[n] = (t + float(r["TotalDurationNs"]) / 1e6, c + int(r["Calls"]))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
subs = int(sys.argv[3]) if len(sys.argv) > 3 else 6
na = a[next(k for k in a if k.startswith("sampler_kernel"))][1] / subs
nb = b[next(k for k in b if k.startswith("sampler_kernel"))][1] / subs
ta = tb = 0.0
for k in sorted(set(a) | set(b), key=lambda k: -b.get(k, (0, 0))[0]):
    x, y = a.get(k, (0, 0)), b.get(k, (0, 0))
    ta += x[0] / na
    tb += y[0] / nb
    if max(x[0] / na, y[0] / nb) >= 0.01:
        print(f"{k[:44]:44s} A {x[0] / na:7.3f} ms/step ({x[1]:4d})  B {y[0] / nb:7.3f} ms/step ({y[1]:4d})")
print(f"{'sum':44s} A {ta:7.3f}                B {tb:7.3f}")
