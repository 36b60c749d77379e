"""Probe: the bench step's sub-batches on S contexts / streams at once (bench.py call()) against
the same sub-batches one after the other: which pairs / fields of the records differ."""
import os
import sys

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy  # noqa: E402
from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE  # noqa: E402

S, B = 6, 768
pairs = bench.make_batch(0, B, 4096, 20200423)
same = os.environ.get("SAME") == "1"  # every sub-batch the same 128 pairs
subs = []
for i in range(S):
    j = 0 if same else i
    b = bench.to_device(pairs[j * B // S:(j + 1) * B // S], "cuda")
    ctx = Context(0)
    # SAMPLERS: one sampler per sub-batch (comma list), else SAMPLER for all
    smp = os.environ.get("SAMPLERS")
    sv = int(smp.split(",")[i]) if smp else int(os.environ.get("SAMPLER", "0"))
    subs.append(dict(b=b, run=PairBatchRunner(ctx=ctx, iters=10000, sampler=sv),
                     st=torch.cuda.Stream()))


def run_one(sb):
    b = sb["b"]
    with torch.cuda.stream(sb["st"]):
        o = sb["run"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"],
                          b["width"], b["height"], b["max_nq"], b["max_nt"],
                          stream=sb["st"].cuda_stream)
        return o["results"].clone()


def overlapped():
    outs = [run_one(sb) for sb in subs]
    torch.cuda.synchronize()
    return results_to_numpy(torch.cat(outs))


def serial():
    outs = []
    for sb in subs:
        outs.append(run_one(sb))
        torch.cuda.synchronize()
    return results_to_numpy(torch.cat(outs))


r = {"ser0": serial(), "ovl0": overlapped(), "ovl1": overlapped(), "ser1": serial()}
for k in ("ovl0", "ovl1", "ser1"):
    bad = []
    for f in RESULT_DTYPE.names:
        a, c = r["ser0"][f], r[k][f]
        ne = np.nonzero(np.any((a != c).reshape(len(a), -1), axis=1))[0]
        if len(ne):
            bad.append(f)
            print(f"{k}: field {f} differs on pairs {ne[:10].tolist()}: {a[ne[:3]].tolist()} vs {c[ne[:3]].tolist()}")
    print(k, "identical to ser0:", not bad)
for k in ("ovl0", "ovl1"):
    br0, br1 = r["ser0"]["binned_rows"].reshape(S, -1), r[k]["binned_rows"].reshape(S, -1)
    print(k, "sub-batches whose records differ from their serial run:",
          [i for i in range(S) if not np.array_equal(br0[i], br1[i])])
if same:
    for k in ("ser0", "ovl0", "ovl1"):
        br = r[k]["binned_rows"].reshape(S, -1)
        print(k, "sub-batches with binned_rows unlike sub-batch 0:",
              [i for i in range(1, S) if not np.array_equal(br[i], br[0])])
