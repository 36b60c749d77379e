"""diagnose one bench pair in Philox mode against the oracle: sample sets, hypotheses, K,
min_idx (python scripts/dev/philox_pair_diag.py [index])"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import oracle as O  # noqa: E402
import torch  # noqa: E402
from erp_match_eightpoint_test_amd import (PairBatchRunner, hyps_to_numpy,  # noqa: E402
                                           results_to_numpy)

idx = int(sys.argv[1]) if len(sys.argv) > 1 else 8
O.build()
p = bench.make_batch(0, idx + 1, 4096, 20200423)[idx]
b = bench.to_device([p], torch.device("cuda:0"))
run = PairBatchRunner(iters=10000, sampler=1)
o = run.run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
            b["height"], b["max_nq"], b["max_nt"], want=("hyps", "samples", "rvec", "dist"))
torch.cuda.synchronize()
r = results_to_numpy(o["results"])[0]
mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=16)
M = len(mt)
ora = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
             O.make_cfg(iters=10000, sampler=1), detail=True)
s = int(M * 0.25)
smp = np.sort(o["samples"][0, :, :s].cpu().numpy(), axis=1)
bad = [it for it in range(10000) if not np.array_equal(smp[it], np.sort(ora["samples"][it]))]
print("M", r["M"], M, "status", r["status"], "K", r["K"], ora["K"], "min_idx", r["min_idx"],
      ora["min_idx"], "survivors", r["survivors"], "near_ties", r["near_ties"])
print("sample mismatches", len(bad), bad[:10])
print("R", r["R"], ora["R"], "T", r["T"], ora["T"])
K = int(r["K"])
rv = o["rvec"][0, :K].cpu().numpy()
_, mi, dref = O.consensus(rv)
print("oracle consensus on GPU rvec: min_idx", mi, "d", dref[mi], "gpu idx d", dref[r["min_idx"]])
order = np.argsort(dref)[:5]
print("5 best", order, dref[order])
