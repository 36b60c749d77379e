"""Probe: run a bench batch (bench.make_batch, default seeds) several times through one
PairBatchRunner per run and report the pairs / fields whose records differ between runs."""
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

B = int(os.environ.get("B", "128"))
pairs = bench.make_batch(0, B, 4096, 20200423)
b = bench.to_device(pairs, "cuda")
args = (b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
        b["height"], b["max_nq"], b["max_nt"])
runs = []
reuse = os.environ.get("REUSE", "1") == "1"  # one context for every run, as bench.py's steps
run0 = PairBatchRunner(ctx=Context(0), iters=10000)
for it in range(3):
    o = (run0 if reuse else PairBatchRunner(ctx=Context(0), iters=10000)).run(*args)
    torch.cuda.synchronize()
    runs.append(results_to_numpy(o["results"]).copy())
for it in (1, 2):
    for f in RESULT_DTYPE.names:
        a, c = runs[0][f], runs[it][f]
        ne = np.nonzero(np.any((a != c).reshape(len(a), -1), axis=1))[0]
        if len(ne):
            print(f"run {it}: field {f} differs on pairs {ne[:12].tolist()}: "
                  f"{a[ne[:4]].tolist()} vs {c[ne[:4]].tolist()}")
    print(f"run {it}: identical = {np.array_equal(runs[0].view(np.uint8), runs[it].view(np.uint8))}")
print("survivors", runs[0]["survivors"][:40].tolist())
print("binned", runs[0]["binned_rows"][:40].tolist())
