#!/usr/bin/env python3
"""Run the pair pipeline several times on one batch and report which result-record fields
differ between runs (the records must be byte-identical: nothing is cached, every kernel's
output is a function of its inputs).  python scripts/dev/determinism.py [pairs] [runs] [twin]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy, synth  # noqa: E402
import bench  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 64
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
twin = len(sys.argv) > 3 and sys.argv[3] == "twin"
if twin:
    seeds = json.load(open(os.path.join(ROOT, "scripts", "twin_seeds.json")))["seeds"][:P]
    pairs = [synth.make_pair(s, inlier_frac=0.98) for s in seeds]
else:
    pairs = bench.make_batch(0, P, 4096, 20200423)
dev = torch.device("cuda:0")
b = bench.to_device(pairs, dev)
ctx = Context(0)
r = PairBatchRunner(ctx=ctx, iters=10000)
r.reserve(P, b["max_nq"], b["max_nt"])
outs = []
for k in range(runs):
    o = r.run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
              b["height"], b["max_nq"], b["max_nt"])
    torch.cuda.synchronize()
    outs.append(results_to_numpy(o["results"].clone()))
ref = outs[0]
for k in range(1, runs):
    diff = {f: int(np.sum(ref[f] != outs[k][f])) for f in ref.dtype.names
            if not np.array_equal(ref[f], outs[k][f])}
    print(f"run {k} vs 0: differing fields (pairs): {diff}")
print("survivors run0:", ref["survivors"][:16].tolist())
