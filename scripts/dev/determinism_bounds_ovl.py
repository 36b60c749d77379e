"""Probe: the consensus bounds phase (erp_consensus_hyps_shard_dev, 1 shard) of one configs[1]
pair on S contexts / streams at once: do lb / ub / bsel agree, and for the rows that differ,
how.  (A pair of the default bench batch.)"""
import os
import sys

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import oracle as O  # noqa: E402  (the matcher for the keypoint lists only)
from erp_match_eightpoint_test_amd import Context  # noqa: E402
from erp_match_eightpoint_test_amd.capi import HYP_DTYPE  # noqa: E402
from erp_match_eightpoint_test_amd.dist import CapiShardBackend  # noqa: E402

S = 6
p = bench.make_batch(0, 10, 4096, 20200423)[int(os.environ.get("PAIR", "6"))]
mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=16)
kl = torch.from_numpy(np.ascontiguousarray(p["kp_l"][mt["queryIdx"]])).cuda()
kr = torch.from_numpy(np.ascontiguousarray(p["kp_r"][mt["trainIdx"]])).cuda()
iters = 10000
hy = torch.zeros((iters, HYP_DTYPE.itemsize), dtype=torch.uint8, device="cuda")
CapiShardBackend(Context(0), p["W"], p["H"], kl, kr, len(mt), {}).hyps(0, iters, hy)
torch.cuda.synchronize()
sts = [torch.cuda.Stream() for _ in range(S)]
bes = [CapiShardBackend(Context(0), p["W"], p["H"], kl, kr, len(mt), {}, stream=st.cuda_stream)
       for st in sts]
outs = []
for rep in range(int(os.environ.get("REPS", "4"))):
    parts = [torch.zeros((3, 2 * iters), dtype=torch.float64, device="cuda") for _ in range(S)]
    for be, part in zip(bes, parts):
        be.shard(hy, iters, 0, 1, part)
    torch.cuda.synchronize()
    outs += [x.cpu().numpy() for x in parts]
ref = outs[0]
nd = 0
for i, o in enumerate(outs[1:], 1):
    d = np.nonzero(np.any(o.view(np.uint64) != ref.view(np.uint64), axis=0))[0]
    if len(d):
        nd += 1
        print(f"out {i}: {len(d)} rows differ, e.g. {d[:6].tolist()}")
        for r in d[:4]:
            print(f"   row {r} (ref row: {r % 16 == 0}): lb {ref[0, r]!r} vs {o[0, r]!r}; ub {ref[1, r]!r} vs "
                  f"{o[1, r]!r}; bsel {ref[2].view(np.int32)[2 * r:2 * r + 2]} vs {o[2].view(np.int32)[2 * r:2 * r + 2]}")
print(f"{len(outs)} outputs, {nd} differ from the first; K rows = {int((ref[1] != 0).sum())}")
