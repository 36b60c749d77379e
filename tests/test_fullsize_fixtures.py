"""CPU checks of the full-size fixtures (tests/golden/gen_fullsize.py): the seeded inputs still
regenerate to the pinned bytes, and the oracle reproduces a configs[2] record."""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

from erp_match_eightpoint_test_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)

import gen_fullsize as G  # noqa: E402


def _npz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def test_manifest_hashes():
    man = json.load(open(os.path.join(GOLD, "MANIFEST.json")))
    for name in ("find_4096_it10k.npz", "match_16384.npz", "batch_2048_it10k.npz"):
        with open(os.path.join(GOLD, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == man[name], name


def test_fullsize_inputs_regenerate():
    g = _npz("find_4096_it10k.npz")
    assert G.input_sha(synth.make_pair(int(g["seed"]), n_kpts=4096)) == str(g["input_sha"])
    g = _npz("match_16384.npz")
    assert G.input_sha(synth.make_pair(int(g["seed"]), n_kpts=int(g["n"]))) == str(g["input_sha"])
    g = _npz("batch_2048_it10k.npz")
    for s, h in zip(g["seed"], g["input_sha"]):
        assert G.input_sha(synth.make_pair(int(s), n_kpts=int(g["n"]))) == str(h)


def test_fullsize_find_fixture_consistent():
    """internal consistency: the winner is among the smallest means, sample hashes per iteration."""
    g = _npz("find_4096_it10k.npz")
    assert g["sample_hash"].shape == (10000,) and g["hyp"].shape == (10000,)
    valid = int(g["hyp"]["R1_valid"].sum() + g["hyp"]["R2_valid"].sum())
    assert valid == int(g["K"])
    assert int(g["best_rows"][0]) == int(g["min_idx"])
    assert int(g["sample_n"]) == int(int(g["M"]) * 0.25)


def test_oracle_reproduces_batch_pair0(oracle):
    g = _npz("batch_2048_it10k.npz")
    p = synth.make_pair(int(g["seed"][0]), n_kpts=int(g["n"]))
    mt, _, _, _ = oracle.match_two_image(p["desc_l"], p["desc_r"])
    assert hashlib.sha256(mt.view(np.uint8).tobytes()).hexdigest() == str(g["match_sha"][0])
    r = oracle.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                    oracle.make_cfg(iters=int(g["iters"])))
    assert r["K"] == g["K"][0] and r["min_idx"] == g["min_idx"][0]
    assert np.array_equal(r["R"], g["R"][0]) and np.array_equal(r["T"], g["T"][0])


def test_manual100k_fixture_consistent(oracle):
    """configs[4] fixture (tests/golden/gen_manual100k.py): the pinned input is the bench's
    manual workload, K equals the stored validity bits, and the oracle reproduces the first
    2048 iterations' sample sets and records (the same glibc stream prefix)."""
    import gen_manual100k as GM
    g = _npz("find_manual_100_it100k.npz")
    man = json.load(open(os.path.join(GOLD, "MANIFEST.json")))
    with open(os.path.join(GOLD, "find_manual_100_it100k.npz"), "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == man["find_manual_100_it100k.npz"]
    c = synth.make_correspondences(int(g["seed"]), m=100, outlier_frac=0.6)
    assert np.array_equal(c["kp_l"], g["kl"]) and np.array_equal(c["kp_r"], g["kr"])
    iters = int(g["iters"])
    bits = np.unpackbits(g["valid_bits"])[: 2 * iters]
    assert int(bits.sum()) == int(g["K"])
    assert int(g["best_rows"][0]) == int(g["min_idx"])
    head = GM.HEAD
    r = oracle.find(int(g["W"]), int(g["H"]), g["kl"], g["kr"], oracle.make_cfg(iters=head),
                    detail=True)
    assert np.array_equal(G.set_hashes(r["samples"]), g["head_hash"])
    assert np.array_equal(GM.chunk_hashes(G.set_hashes(r["samples"]), int(g["chunk"]))[:2],
                          g["chunk_hash"][:2])
    v = np.stack([r["hyp"]["R1_valid"], r["hyp"]["R2_valid"]], 1).astype(np.uint8).reshape(-1)
    assert np.array_equal(v, bits[: 2 * head])
    sel = np.arange(0, head, int(g["stride"]))
    he = g["hyp_every"][: sel.size]
    assert np.abs(r["hyp"]["R1"][sel] - he["R1"]).max() == 0
    assert np.abs(r["hyp"]["T"][sel] - he["T"]).max() == 0
