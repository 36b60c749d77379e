"""Generate the committed golden fixtures of tests/golden/ from the CPU oracle.

The reference commits no expected outputs, so the fixtures are the oracle's
outputs on seeded synthetic inputs; the inputs are stored too (numpy Generator streams are not
guaranteed stable across numpy versions).  The oracle itself is pinned by glibc_shuffle.json
(real glibc/libstdc++ outputs) and by tests/test_oracle.py.

    python tests/golden/gen_fixtures.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402
from erp_match_eightpoint_test_amd import synth  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    return path


def main():
    written = []
    # 1) matcher: 384 x 384 SURF-like descriptors (+ 5 duplicated train rows for tie cases)
    p = synth.make_pair(11, n_kpts=384)
    dl, dr = p["desc_l"], p["desc_r"].copy()
    dr[100:105] = dr[200:205]  # exact duplicates -> equal distances, lowest index must win
    mt, best, d0, d1 = O.match_two_image(dl, dr)
    written.append(save("match_384.npz", desc_l=dl, desc_r=dr, query=mt["queryIdx"],
                        train=mt["trainIdx"], dist_bits=mt["distance"].view(np.uint32),
                        best=best, d0sq_bits=d0.view(np.uint32), d1sq_bits=d1.view(np.uint32)))
    # 2) estimator: 400 correspondences, 80 iterations (reference defaults), glibc seed 1
    p = synth.make_pair(12, n_kpts=512)
    mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"])
    kl = p["kp_l"][mt["queryIdx"]][:400]
    kr = p["kp_r"][mt["trainIdx"]][:400]
    r = O.find(p["W"], p["H"], kl, kr, O.make_cfg(), detail=True)
    written.append(save("find_400_it80.npz", kl=kl, kr=kr, W=np.int32(p["W"]), H=np.int32(p["H"]),
                        R=r["R"], T=r["T"], K=np.int32(r["K"]), min_idx=np.int32(r["min_idx"]),
                        samples=np.sort(r["samples"], axis=1).astype(np.int32),
                        hyp=r["hyp"], rvec=r["rvec"], tvec=r["tvec"], dist=r["dist"],
                        euler_gt=p["euler_gt"]))
    # 3) manual-pickup regime: 100 integer-pixel correspondences, 60 % outliers, 2048x1024
    c = synth.make_correspondences(13, m=100, outlier_frac=0.6)
    r = O.find(c["W"], c["H"], c["kp_l"], c["kp_r"], O.make_cfg(iters=500), detail=True)
    written.append(save("find_manual_100_it500.npz", kl=c["kp_l"], kr=c["kp_r"],
                        W=np.int32(c["W"]), H=np.int32(c["H"]), R=r["R"], T=r["T"],
                        K=np.int32(r["K"]), min_idx=np.int32(r["min_idx"]),
                        samples=np.sort(r["samples"], axis=1).astype(np.int32), hyp=r["hyp"],
                        rvec=r["rvec"], dist=r["dist"]))
    # 4) thin-SVD edge cases: M in {4, 8, 20, 35, 36} (sample_n 1, 2, 5, 8, 9)
    edge = {}
    for m in (4, 8, 20, 35, 36):
        c = synth.make_correspondences(100 + m, m=m, outlier_frac=0.0, W=5376, H=2688,
                                       integer=False)
        r = O.find(c["W"], c["H"], c["kp_l"], c["kp_r"], O.make_cfg(), detail=True)
        edge[f"m{m}_kl"] = c["kp_l"]
        edge[f"m{m}_kr"] = c["kp_r"]
        edge[f"m{m}_R"] = r["R"]
        edge[f"m{m}_T"] = r["T"]
        edge[f"m{m}_K"] = np.int32(r["K"])
        edge[f"m{m}_status"] = np.int32(r["status"])
        edge[f"m{m}_samples"] = np.sort(r["samples"], axis=1).astype(np.int32)
        edge[f"m{m}_hyp"] = r["hyp"]
    written.append(save("find_edges.npz", **edge))
    man = {os.path.basename(w): hashlib.sha256(open(w, "rb").read()).hexdigest() for w in written}
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(json.dumps(man, indent=1))


if __name__ == "__main__":
    main()
