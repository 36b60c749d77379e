"""Probe: are the consensus bounds (phase 1: erp_consensus_hyps_shard_dev, 1 shard -- the flat
route included) byte-identical run to run on a two-cluster pair, and is the finish phase?
Prints the rows whose lb / ub / bsel differ between two runs."""
import json
import os
import sys

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle as O  # noqa: E402  (the matcher for the keypoint lists only)
from erp_match_eightpoint_test_amd import Context, synth  # noqa: E402
from erp_match_eightpoint_test_amd.capi import HYP_DTYPE, RESULT_DTYPE  # noqa: E402
from erp_match_eightpoint_test_amd.dist import CapiShardBackend  # noqa: E402

seeds = json.load(open(os.path.join(ROOT, "scripts", "twin_seeds.json")))["seeds"]
p = synth.make_pair(seeds[0], n_kpts=4096, inlier_frac=0.98)
mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=16)
kl = torch.from_numpy(np.ascontiguousarray(p["kp_l"][mt["queryIdx"]])).cuda()
kr = torch.from_numpy(np.ascontiguousarray(p["kp_r"][mt["trainIdx"]])).cuda()
iters = 10000
ctx = Context(0)
be = CapiShardBackend(ctx, p["W"], p["H"], kl, kr, len(mt), {})
hy = torch.zeros((iters, HYP_DTYPE.itemsize), dtype=torch.uint8, device="cuda")
be.hyps(0, iters, hy)
parts, ress = [], []
for it in range(3):
    c2 = Context(0)
    b2 = CapiShardBackend(c2, p["W"], p["H"], kl, kr, len(mt), {})
    part = torch.zeros((3, 2 * iters), dtype=torch.float64, device="cuda")
    b2.shard(hy, iters, 0, 1, part)
    res = torch.zeros(RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    b2.finish(hy, iters, part.clone(), res)
    torch.cuda.synchronize()
    parts.append(part.cpu().numpy())
    ress.append(res.cpu().numpy().view(RESULT_DTYPE)[0])
print("rows with a NaN ub:", int(np.isnan(parts[0][1, :]).sum()), "nan lb:", int(np.isnan(parts[0][0, :]).sum()))
for it in (1, 2):
    d = np.nonzero(np.any(parts[it].view(np.uint64) != parts[0].view(np.uint64), axis=0))[0]
    print(f"run {it} vs 0: rows with different lb/ub/bsel: {len(d)} {d[:20].tolist()}")
    for r in d[:8]:
        print("   row", r, "lb", parts[0][0, r], parts[it][0, r], "ub", parts[0][1, r], parts[it][1, r],
              "bsel", parts[0][2].view(np.int32)[2 * r:2 * r + 2], parts[it][2].view(np.int32)[2 * r:2 * r + 2])
    print("  results", [(int(x["min_idx"]), int(x["survivors"]), int(x["binned_rows"])) for x in ress])
