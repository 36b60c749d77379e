"""Full-size parity against committed oracle fixtures (tests/golden/gen_fullsize.py):

* configs[1]: the bench's first 4096 x 4096 pair through the fused batch path at 10 000
  iterations -- match list bit-exact, every iteration's sample set (hash) identical, every
  iteration's record within the estimator bars, K / min_idx equal, R / T within TOL_RT, the
  winner's trimmed mean within 1e-12 relative (src/eight_point.cpp:87-150);
* configs[3]: one 16384 x 16384 match on both matcher methods, bit-exact
  (src/feature_matcher.cpp:42-59);
* configs[2]: a 32-pair batch of 2048-keypoint pairs at 10 000 iterations, the 8 fixture pairs'
  records and match lists equal to the oracle's;
* configs[4]: the bench's manual workload (100 correspondences, 60 % outliers) at 100 000
  iterations (K ~ 89k valid rotations): every iteration's validity, every 25th iteration's
  record, K / min_idx / R / T / the winner's trimmed mean -- unsharded and through the
  row-sharded consensus of 2 and 8 emulated ranks (tests/golden/gen_manual100k.py).

The inputs are regenerated from their seeds and pinned by sha256 before anything is compared.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import pytest

from erp_match_eightpoint_test_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)

import gen_fullsize as G  # noqa: E402  (hash helpers; the generator itself only runs by hand)

sys.path.insert(0, os.path.dirname(__file__))
from parity_log import record  # noqa: E402


def _npz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


# R (Euler, rad) and T against the oracle (1e-6); the measured largest deviations
# are kept by parity_log (ERP_PARITY_OUT)
TOL_RT = 1e-6


@pytest.fixture(scope="module")
def ctx(gpu_lib):
    from erp_match_eightpoint_test_amd import Context
    return Context(0)


def _batch(pairs):
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ol = np.concatenate([[0], np.cumsum([len(p["desc_l"]) for p in pairs])]).astype(np.int64)
    orr = np.concatenate([[0], np.cumsum([len(p["desc_r"]) for p in pairs])]).astype(np.int64)
    return (t(np.concatenate([p["desc_l"] for p in pairs])),
            t(np.concatenate([p["desc_r"] for p in pairs])),
            t(np.concatenate([p["kp_l"] for p in pairs])),
            t(np.concatenate([p["kp_r"] for p in pairs])), t(ol), t(orr),
            t(np.array([p["W"] for p in pairs], np.int32)),
            t(np.array([p["H"] for p in pairs], np.int32)),
            int(np.diff(ol).max()), int(np.diff(orr).max()))


def _dmatch_rows(g):
    rows = np.zeros((len(g["query"]), 4), np.uint32)
    rows[:, 0] = g["query"]
    rows[:, 1] = g["train"]
    rows[:, 3] = g["dist_bits"]
    return rows


def test_find_full_size_fixture(ctx):
    """configs[1] end to end: one 4096 x 4096 pair, 10 000 iterations, against the oracle."""
    import torch
    from erp_match_eightpoint_test_amd import PairBatchRunner, hyps_to_numpy, results_to_numpy
    g = _npz("find_4096_it10k.npz")
    p = synth.make_pair(int(g["seed"]), n_kpts=4096)
    assert G.input_sha(p) == str(g["input_sha"]), "synthetic input generation changed"
    run = PairBatchRunner(ctx=ctx, iters=10000)
    outs = run.run(*_batch([p]), want=("matches", "hyps", "samples", "dist"))
    torch.cuda.synchronize()
    r = results_to_numpy(outs["results"])[0]
    M = int(g["M"])
    assert r["status"] == 0 and r["M"] == M
    got = outs["matches"][0, :M].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, _dmatch_rows(g))
    # every iteration's sample set (glibc replay over 10 000 x (M-1) draws)
    s = int(g["sample_n"])
    assert int(r["sample_n"]) == s
    samples = outs["samples"][0, :, :s].cpu().numpy()
    bad = np.nonzero(G.set_hashes(samples) != g["sample_hash"])[0]
    assert bad.size == 0, f"{bad.size} iterations sample a different set, first {bad[:8]}"
    # every iteration's record
    gh = hyps_to_numpy(outs["hyps"])[0]
    oh = g["hyp"]
    assert np.array_equal(gh["R1_valid"] + gh["R2_valid"],
                          oh["R1_valid"].astype(np.int32) + oh["R2_valid"].astype(np.int32))
    same = np.maximum(np.abs(gh["R1"] - oh["R1"]).max(1), np.abs(gh["R2"] - oh["R2"]).max(1))
    swap = np.maximum(np.abs(gh["R1"] - oh["R2"]).max(1), np.abs(gh["R2"] - oh["R1"]).max(1))
    e = np.minimum(np.abs(gh["E"] - oh["E"]).max(1), np.abs(gh["E"] + oh["E"]).max(1))
    record("configs[1] find_4096_it10k: every iteration", R=np.minimum(same, swap).max(),
           T=np.abs(gh["T"] - oh["T"]).max(), E=e.max())
    record("configs[1] find_4096_it10k: result", R=np.abs(r["R"] - g["R"]).max(),
           T=np.abs(r["T"] - g["T"]).max())
    assert np.minimum(same, swap).max() <= TOL_RT
    assert np.abs(gh["T"] - oh["T"]).max() <= TOL_RT
    assert e.max() <= 1e-6  # (E stored as f32 in the fixture: <= 6e-8 of that is storage)
    # consensus: the same number of valid rotations, the same first minimum, its R and T
    assert int(r["K"]) == int(g["K"])
    assert int(r["min_idx"]) == int(g["min_idx"])
    assert np.abs(r["R"] - g["R"]).max() <= TOL_RT and np.abs(r["T"] - g["T"]).max() <= TOL_RT
    assert abs(float(r["min_dist"]) - float(g["min_dist"])) <= 1e-12 * abs(float(g["min_dist"]))
    # the 16 smallest trimmed means the oracle saw: the GPU computes them exactly too
    d = outs["dist"][0].cpu().numpy()
    for row, val in zip(g["best_rows"], g["best_dist"]):
        if np.isfinite(d[row]):
            assert abs(d[row] - val) <= 1e-12 * abs(val), (row, d[row], val)
    assert np.isfinite(d[int(g["min_idx"])])


@pytest.mark.parametrize("method", ["mfma_filter", "valu_exact"])
def test_dense_16384_fixture(gpu_lib, method):
    """configs[3]: one 16384 x 16384 exact k=2 + ratio match on each method vs the oracle."""
    import torch
    from erp_match_eightpoint_test_amd import Context, capi, feature_matcher
    g = _npz("match_16384.npz")
    n = int(g["n"])
    p = synth.make_pair(int(g["seed"]), n_kpts=n)
    assert G.input_sha(p) == str(g["input_sha"]), "synthetic input generation changed"
    c = Context(0)
    m = capi.MATCHER_MFMA_FILTER if method == "mfma_filter" else capi.MATCHER_VALU_EXACT
    fm = feature_matcher(ctx=c, method=m)
    out = fm._match_device(torch.from_numpy(p["desc_l"]).cuda(),
                           torch.from_numpy(p["desc_r"]).cuda(), 0.3)
    got = out.cpu().numpy().view(np.uint32)
    assert got.shape[0] == len(g["query"])
    assert np.array_equal(got, _dmatch_rows(g))


def test_batch_2048_configs2_fixture(ctx):
    """configs[2] per rank: 32 pairs of 2048 x 2048 keypoints at 10 000 iterations in one
    batch; the 8 fixture pairs (interleaved with 24 others) equal the oracle's records."""
    import torch
    from erp_match_eightpoint_test_amd import PairBatchRunner, results_to_numpy
    g = _npz("batch_2048_it10k.npz")
    n = int(g["n"])
    seeds = [int(s) for s in g["seed"]]
    pairs, where = [], {}
    for i in range(32):
        if i % 4 == 0:
            k = i // 4
            where[k] = i
            pairs.append(synth.make_pair(seeds[k], n_kpts=n))
            assert G.input_sha(pairs[-1]) == str(g["input_sha"][k])
        else:
            pairs.append(synth.make_pair(55000 + i, n_kpts=n))
    run = PairBatchRunner(ctx=ctx, iters=int(g["iters"]))
    outs = run.run(*_batch(pairs), want=("matches",))
    torch.cuda.synchronize()
    res = results_to_numpy(outs["results"])
    assert np.all(res["status"] == 0)
    for k, i in where.items():
        r = res[i]
        M = int(g["M"][k])
        assert int(r["M"]) == M and int(r["K"]) == int(g["K"][k]), (k, r["M"], r["K"])
        assert int(r["min_idx"]) == int(g["min_idx"][k])
        record("configs[2] batch_2048_it10k: results", R=np.abs(r["R"] - g["R"][k]).max(),
               T=np.abs(r["T"] - g["T"][k]).max())
        assert np.abs(r["R"] - g["R"][k]).max() <= TOL_RT
        assert np.abs(r["T"] - g["T"][k]).max() <= TOL_RT
        mt = outs["matches"][i, :M].cpu().numpy()
        assert hashlib.sha256(mt.view(np.uint8).tobytes()).hexdigest() == str(g["match_sha"][k])


@pytest.mark.parametrize("shards", [1, 2, 8])
def test_manual_100k_fixture(ctx, shards):
    """configs[4] at full size against the oracle (src/eight_point.cpp:87-150, I = 100 000)."""
    import ctypes as C
    import torch
    from erp_match_eightpoint_test_amd import capi, dist as D, hyps_to_numpy, results_to_numpy
    g = _npz("find_manual_100_it100k.npz")
    W, H, iters, m = int(g["W"]), int(g["H"]), int(g["iters"]), len(g["kl"])
    dkl = torch.from_numpy(np.ascontiguousarray(g["kl"], np.float32)).cuda()
    dkr = torch.from_numpy(np.ascontiguousarray(g["kr"], np.float32)).cuda()
    if shards == 1:
        cfg = capi.default_cfg(iters=iters)
        res = torch.zeros(capi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        hyp = torch.zeros((iters, capi.HYP_DTYPE.itemsize), dtype=torch.uint8, device="cuda")
        assert ctx.L.erp_eight_point_find_dev(ctx.h, W, H, dkl.data_ptr(), dkr.data_ptr(), m,
                                              C.byref(cfg), res.data_ptr(), hyp.data_ptr(),
                                              torch.cuda.current_stream().cuda_stream) == 0
    else:
        res, hyp = D.find_hypothesis_sharded_dev(ctx, W, H, dkl, dkr, m, iters,
                                                 emulate_world=shards)
        hyp = hyp[:iters]
    torch.cuda.synchronize()
    r = results_to_numpy(res.view(1, -1))[0]
    gh = hyps_to_numpy(hyp.unsqueeze(0))[0]
    bits = np.unpackbits(g["valid_bits"])[: 2 * iters].reshape(iters, 2)
    got = np.stack([gh["R1_valid"], gh["R2_valid"]], 1) != 0
    # R1 / R2 order inside an iteration follows a noise-level sign: validity as
    # a count per iteration, the records as sets
    bad = np.nonzero(got.sum(1) != bits.sum(1))[0]
    assert bad.size == 0, f"{bad.size} iterations differ in validity, first {bad[:8]}"
    sel = np.arange(0, iters, int(g["stride"]))
    oh, hh = g["hyp_every"], gh[sel]
    same = np.maximum(np.abs(hh["R1"] - oh["R1"]).max(1), np.abs(hh["R2"] - oh["R2"]).max(1))
    swap = np.maximum(np.abs(hh["R1"] - oh["R2"]).max(1), np.abs(hh["R2"] - oh["R1"]).max(1))
    e = np.minimum(np.abs(hh["E"] - oh["E"]).max(1), np.abs(hh["E"] + oh["E"]).max(1))
    record(f"configs[4] manual_100_it100k x{shards} shards: every 25th iteration",
           R=np.minimum(same, swap).max(), T=np.abs(hh["T"] - oh["T"]).max(), E=e.max())
    record(f"configs[4] manual_100_it100k x{shards} shards: result",
           R=np.abs(r["R"] - g["R"]).max(), T=np.abs(r["T"] - g["T"]).max())
    assert np.minimum(same, swap).max() <= TOL_RT
    assert np.abs(hh["T"] - oh["T"]).max() <= TOL_RT
    assert e.max() <= 1e-6
    assert int(r["status"]) == 0 and int(r["K"]) == int(g["K"])
    assert int(r["min_idx"]) == int(g["min_idx"]), (int(r["min_idx"]), int(g["min_idx"]))
    assert np.abs(r["R"] - g["R"]).max() <= TOL_RT and np.abs(r["T"] - g["T"]).max() <= TOL_RT
    assert abs(float(r["min_dist"]) - float(g["min_dist"])) <= 1e-12 * abs(float(g["min_dist"]))
