"""Matcher parity probe: the 16k fixture and random pairs vs the oracle, with details of the
first mismatching queries (dev tool; ERP_LIB_PATH selects a library variant)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle as O  # noqa: E402
from erp_match_eightpoint_test_amd import Context, capi, feature_matcher, synth  # noqa: E402


def run(p, n_show=5):
    c = Context(0)
    fm = feature_matcher(ctx=c, method=capi.MATCHER_MFMA_FILTER)
    out = fm._match_device(torch.from_numpy(p["desc_l"]).cuda(), torch.from_numpy(p["desc_r"]).cuda(), 0.3)
    got = out.cpu().numpy()
    ref, best, d0, d1 = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=16)
    gq = set(got.view(np.int32).reshape(-1, 4)[:, 0].tolist())
    rq = set(ref["queryIdx"].tolist())
    print(f"n={len(p['desc_l'])}: got {len(gq)} ref {len(rq)} extra {sorted(gq - rq)[:n_show]} missing {sorted(rq - gq)[:n_show]}")
    ok = len(gq ^ rq) == 0
    for q in sorted(gq ^ rq)[:n_show]:
        dd = ((p["desc_r"].astype(np.float64) - p["desc_l"][q].astype(np.float64)) ** 2).sum(1)
        o = np.argsort(dd)[:4]
        print(f"  q={q} oracle best={best[q]} d0={d0[q]:.6g} d1={d1[q]:.6g} |q|^2={float((p['desc_l'][q]**2).sum()):.6g}"
              f" nearest {list(zip(o.tolist(), dd[o].round(6).tolist()))}")
    if ok:
        g = got.view(np.uint32).reshape(-1, 4)
        r = ref.view(np.uint32).reshape(-1, 4)
        ok = np.array_equal(g, r)
        if not ok:
            bad = np.nonzero((g != r).any(1))[0][:n_show]
            print("  differing rows", bad, g[bad], r[bad])
    return ok


if __name__ == "__main__":
    print("lib", capi.lib_path())
    allok = True
    for n, seed in ((16384, 11), (4096, 3), (4096, 4), (2000, 5), (1000, 6)):
        allok &= run(synth.make_pair(seed, n_kpts=n))
    print("ALL OK" if allok else "MISMATCH")
