"""Visual outputs on the CPU: the oracle's literal restatements
(oracle/erp_viz.c) against known answers and against the closed-form final state the device
kernel computes (erp_match_eightpoint_test_amd/csrc/viz.hip: epipolar_kernel).

* hsv2bgr: cv::cvtColor(COLOR_HSV2BGR) known answers (hue range 180: 0 red, 30 yellow, 60 green,
  90 cyan, 120 blue, 150 magenta at full saturation and value) and the draw_match palette.
* RGB2GRAY fixed point (the reference calls CV_RGB2GRAY on BGR images: channel 0 weighted as R).
* epipolar: the literal sequential loop (rows, cols, keys; curve write, then 11 x 11 dot write at
  its unchecked linear address) == "dot of the last covering key, else curve of the last key,
  corner pixel interleaved" -- the rule the device kernel evaluates per pixel -- on canvases
  with dots wrapping across the left/right edges and leaving the buffer at the top/bottom.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

COLORS = np.array([[0, 0, 255], [0, 127, 255], [0, 255, 255], [0, 255, 0], [255, 0, 0],
                   [135, 0, 75], [211, 0, 148]], np.uint8)  # src/epipolar_tool.cpp:18-24


@pytest.mark.parametrize("h,bgr", [(0, (0, 0, 255)), (30, (0, 255, 255)), (60, (0, 255, 0)),
                                   (90, (255, 255, 0)), (120, (255, 0, 0)),
                                   (150, (255, 0, 255)), (180, (0, 0, 255))])
def test_hsv2bgr_primaries(oracle, h, bgr):
    assert tuple(oracle.hsv2bgr(h, 255, 255)) == bgr


def test_hsv2bgr_grey_and_palette(oracle):
    assert tuple(oracle.hsv2bgr(77, 0, 150)) == (150, 150, 150)
    # draw_match's S = 180, V = 150: the darkest channel is V (1 - S) = 150 * 75 / 255 = 44.1
    assert tuple(oracle.hsv2bgr(0, 180, 150)) == (44, 44, 150)
    assert tuple(oracle.hsv2bgr(90, 180, 150)) == (150, 150, 44)
    for h in range(0, 181):
        c = oracle.hsv2bgr(h, 180, 150)
        assert c.max() == 150 and c.min() == 44


def test_draw_match_grey_channels(oracle):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    out = oracle.draw_match(a, b, np.zeros((0, 2)), np.zeros((0, 2)))
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    ga = (a64[..., 0] * 4899 + a64[..., 1] * 9617 + a64[..., 2] * 1868 + 8192) >> 14
    gb = (b64[..., 0] * 4899 + b64[..., 1] * 9617 + b64[..., 2] * 1868 + 8192) >> 14
    assert (out[..., 0] == ga).all() and (out[..., 1] == gb).all() and (out[..., 2] == 0).all()
    white = np.full((2, 2, 3), 255, np.uint8)
    assert (oracle.draw_match(white, white, [], [])[..., :2] == 255).all()


def test_draw_match_line_geometry(oracle):
    """a horizontal segment (10, 10) -> (30, 10): the capsule of radius 2.5 covers rows 8..12
    over columns 10..30 and rounds off at the ends; later matches paint over earlier ones"""
    z = np.zeros((24, 40, 3), np.uint8)
    out = oracle.draw_match(z, z, [[10.2, 9.8]], [[29.6, 10.4]])
    m = out[..., 2] > 0
    assert m[8:13, 10:31].all() and not m[7].any() and not m[13].any()
    assert m[10, 8] and m[10, 32] and not m[10, 7] and not m[10, 33]
    assert not m[8, 8] and not m[12, 32]  # corners of the bounding box lie outside the cap
    c0 = oracle.hsv2bgr(0, 180, 150)
    assert (out[m] == c0).all()
    two = oracle.draw_match(z, z, [[10, 10], [20, 2]], [[30, 10], [20, 20]])
    c1 = oracle.hsv2bgr(90, 180, 150)
    assert (two[10, 20] == c1).all() and (two[10, 12] == c0).all()


def _keys_l(kl, idx, W, H):
    out = []
    for t in idx:
        lon = 2 * math.pi * float(np.float32(kl[t, 0]) / np.float32(W))
        lat = math.pi * float(np.float32(kl[t, 1]) / np.float32(H))
        out.append([-math.sin(lat) * math.cos(lon), math.sin(lat) * math.sin(lon), math.cos(lat)])
    return np.array(out)


def _closed_form(oracle, kl, kr, W, H, ow, oh, n_key, E, idx):
    """the device kernel's per-pixel rule (viz.hip epipolar_kernel), in Python"""
    ls = _keys_l(kl, idx, W, H)
    rw, rh = ow / W, oh / H
    di = [int(float(np.float32(kr[t, 1])) * rh) for t in idx]
    dj = [int(float(np.float32(kr[t, 0])) * rw) for t in idx]
    out = np.zeros((oh, ow, 3), np.uint8)
    for i in range(oh):
        for j in range(ow):
            q = i * ow + j
            curve = dot = last = -1
            for t in range(n_key):
                if abs(oracle.epipolar_value(ls[t], E, i, j, ow, oh)) < 0.002:
                    curve = last = t
                r = q - (di[t] * ow + dj[t])
                if any(-5 <= r - dy * ow <= 5 for dy in range(-5, 6)):
                    dot = last = t
            c = dot if dot >= 0 else curve
            if i == oh - 1 and j == ow - 1:
                c = last
            if c >= 0:
                out[i, j] = COLORS[c]
    return out


@pytest.mark.parametrize("case", ["interior", "edges"])
def test_epipolar_sequential_rule(oracle, case):
    rng = np.random.default_rng(11 if case == "interior" else 12)
    W, H, ow, oh, m, n_key = 640, 320, 72, 36, 30, 7
    kl = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
    kr = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
    if case == "edges":  # dots across every edge and onto the last pixel
        kr[:] = np.array([[2, 150], [W - 3, 200], [300, 3], [320, H - 2], [W - 1, H - 1], [0, 0],
                          [5, H - 4]] * 5, np.float32)[:m]
    ang = rng.normal(size=3) * 0.2
    Rm = _rodrigues(ang)
    t = rng.normal(size=3)
    t /= np.linalg.norm(t)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    E = tx @ Rm * 0.03  # |l^T E p| < 0.002: a band ~0.07 rad wide, about one pixel here
    lit, idx, margin = oracle.epipolar_draw(kl, kr, W, H, ow, oh, n_key, E)
    assert len(set(idx.tolist())) == n_key
    assert (oracle.GlibcRand(1).random_array(m)[:n_key] == idx).all()
    ref = _closed_form(oracle, kl, kr, W, H, ow, oh, n_key, E, idx)
    assert (lit == ref).all(), np.argwhere((lit != ref).any(-1))[:10]
    assert lit.any(-1).sum() > 7 * 121 + 50  # curves drawn besides the dots


def _rodrigues(v):
    th = np.linalg.norm(v)
    k = v / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def test_epipolar_seed_offset(oracle):
    rng = np.random.default_rng(5)
    kl = rng.uniform(0, 100, (50, 2))
    E = np.eye(3)
    _, a, _ = oracle.epipolar_draw(kl, kl, 100, 50, 20, 10, 5, E, seed=1, offset=0)
    _, b, _ = oracle.epipolar_draw(kl, kl, 100, 50, 20, 10, 5, E, seed=1, offset=3)
    g = oracle.GlibcRand(1, 3)
    assert (g.random_array(50)[:5] == b).all() and not (a == b).all()
    with pytest.raises(ValueError):
        oracle.epipolar_draw(kl, kl, 100, 50, 20, 10, 8, E)
