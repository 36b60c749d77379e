"""Generate the configs[4] oracle fixture (BASELINE.json configs[4]: a 100k-iteration
initial_guess on manual_point_pickup_test-style correspondences with 60 % outliers) from the CPU
oracle, in this container.

The input is bench.py --workload manual's: synth.make_correspondences(20200423, m=100,
outlier_frac=0.6) on 2048 x 1024 (build/config_file.ini:4-6), integer pixels; it is stored
(100 x 2 x 2 floats).  Stored results (src/eight_point.cpp:87-150 at I = 100 000):
  K, min_idx, R, T, min_dist, the 16 smallest trimmed means (rows + values);
  valid_bits: every iteration's (R1_valid, R2_valid), np.packbits over [iters, 2];
  hyp_every: every STRIDE-th iteration's record (R1, R2, T, validity, E as f32);
  chunk_hash: per CHUNK iterations, the sum of the iterations' sorted-sample-set hashes times
  P^(iteration), mod 2^64 (gen_fullsize.set_hashes per iteration) -- order and set sensitive;
  head_hash: the per-iteration set hashes of the first 2048 iterations.

    python tests/golden/gen_manual100k.py      (~2-4 min on 8 cores: K ~ 89k rows of
                                                 K-element sorts)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import oracle as O  # noqa: E402
from erp_match_eightpoint_test_amd import synth  # noqa: E402
import gen_fullsize as G  # noqa: E402

SEED = 20200423
ITERS = 100000
STRIDE = 25
CHUNK = 1000
HEAD = 2048


def chunk_hashes(h: np.ndarray, chunk: int) -> np.ndarray:
    """sum_i h_i P^i mod 2^64 per chunk of `chunk` iterations (i = iteration index)"""
    n = h.shape[0]
    pw = np.ones(n, np.uint64)
    with np.errstate(over="ignore"):
        for i in range(1, n):
            pw[i] = pw[i - 1] * G.HASH_P
        prod = h.astype(np.uint64) * pw
        return np.add.reduceat(prod, np.arange(0, n, chunk), dtype=np.uint64)


def main():
    c = synth.make_correspondences(SEED, m=100, outlier_frac=0.6)
    t0 = time.time()
    r = O.find(c["W"], c["H"], c["kp_l"], c["kp_r"], O.make_cfg(iters=ITERS), detail=True)
    print(f"oracle find: {time.time() - t0:.1f} s, K = {r['K']}, min_idx = {r['min_idx']}")
    hyp = r["hyp"]
    sel = np.arange(0, ITERS, STRIDE)
    lite = np.zeros(sel.size, G.HYP_LITE)
    for f in G.HYP_LITE.names:
        lite[f] = hyp[f][sel]
    valid = np.stack([hyp["R1_valid"], hyp["R2_valid"]], 1).astype(np.uint8)
    h = G.set_hashes(r["samples"])
    order = np.argsort(r["dist"], kind="stable")[:16]
    path = os.path.join(HERE, "find_manual_100_it100k.npz")
    np.savez_compressed(path, seed=np.int64(SEED), kl=c["kp_l"], kr=c["kp_r"],
                        W=np.int32(c["W"]), H=np.int32(c["H"]), iters=np.int32(ITERS),
                        sample_n=np.int32(r["sample_n"]), K=np.int32(r["K"]),
                        min_idx=np.int32(r["min_idx"]), R=r["R"], T=r["T"],
                        min_dist=np.float64(r["min_dist"]), best_rows=order.astype(np.int32),
                        best_dist=r["dist"][order], valid_bits=np.packbits(valid.reshape(-1)),
                        stride=np.int32(STRIDE), hyp_every=lite, chunk=np.int32(CHUNK),
                        chunk_hash=chunk_hashes(h, CHUNK), head_hash=h[:HEAD],
                        euler_gt=c.get("euler_gt", np.zeros(3)))
    man_path = os.path.join(HERE, "MANIFEST.json")
    man = json.load(open(man_path))
    man[os.path.basename(path)] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(man_path, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
