"""Visual outputs on the GPU through the C ABI
(erp_epipolar_draw_dev, erp_draw_match_dev) against the oracle's literal restatements
(oracle/erp_viz.c).

* epipolar_tool.draw_epipole: bit-exact canvases; the only pixels allowed to differ are those
  whose |l^T E p| is within 1e-12 of the 0.002 threshold (the device's sin/cos may differ from
  glibc's by an ulp: ~1e-16 on the value) -- the oracle reports how close the canvas came, and a
  differing pixel is checked against that certificate.  random_idx equals the glibc shuffle.
* feature_matcher.draw_match: bit-exact (integer grey, the HSV palette, the capsule test in
  double on integer endpoints); lines running off the image, zero-length lines, many
  overlapping lines (the later match wins), zero matches.
* spherical_surf.do_all(draw=True): match_output == draw_match of the returned keypoints.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gpu_lib):
    from erp_match_eightpoint_test_amd import Context
    return Context(0)


def _essential(rng, scale):
    v = rng.normal(size=3) * 0.3
    th = np.linalg.norm(v)
    k = v / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K
    t = rng.normal(size=3)
    t /= np.linalg.norm(t)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    return tx @ R * scale


def _certify(oracle, got, want, kl, idx, W, H, E):
    """pixels where the canvases differ must sit within 1e-12 of the threshold for some key"""
    bad = np.argwhere((got != want).any(-1))
    oh, ow = got.shape[:2]
    ls = []
    for t in idx:
        lon = 2 * math.pi * float(np.float32(kl[t, 0]) / np.float32(W))
        lat = math.pi * float(np.float32(kl[t, 1]) / np.float32(H))
        ls.append([-math.sin(lat) * math.cos(lon), math.sin(lat) * math.sin(lon), math.cos(lat)])
    for i, j in bad:
        d = min(abs(abs(oracle.epipolar_value(l, E, int(i), int(j), ow, oh)) - 0.002) for l in ls)
        assert d < 1e-12, (i, j, d)
    return len(bad)


@pytest.mark.parametrize("W,H,ow,oh,m,n_key,scale,seed,offset", [
    (2048, 1024, 960, 480, 300, 7, 1.0, 1, 0),      # the reference's test sizes, scaled
    (5376, 2688, 1344, 672, 4000, 7, 0.5, 1, 80),   # full-res keys, offset past one RANSAC run
    (640, 320, 641, 333, 9, 5, 0.1, 7, 3),          # odd canvas, fat curves, fewer keys
    (1000, 500, 64, 32, 1, 1, 1.0, 1, 0),           # one match
    (1000, 500, 64, 32, 20, 0, 1.0, 1, 0),          # no key: a black canvas
])
def test_epipolar_draw_matches_oracle(ctx, oracle, W, H, ow, oh, m, n_key, scale, seed, offset):
    from erp_match_eightpoint_test_amd import epipolar_tool
    rng = np.random.default_rng(W + m + n_key)
    kl = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
    kr = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
    kr[: min(m, 3)] = np.array([[0.5, 0.5], [W - 0.5, H - 0.5], [W - 1, 3]], np.float32)[: min(m, 3)]
    E = _essential(rng, scale)
    tool = epipolar_tool(kl, kr, W, H, ow, oh, n_key, seed=seed, offset=offset, ctx=ctx)
    before = tool.random_idx.copy()  # filled by the constructor, as the reference's
    got = tool.draw_epipole(E).cpu().numpy()
    want, idx, margin = oracle.epipolar_draw(kl, kr, W, H, ow, oh, n_key, E, seed=seed,
                                             offset=offset)
    assert (tool.random_idx == idx).all() and (before == idx).all()
    n_bad = _certify(oracle, got, want, kl, idx, W, H, E)
    print(f"\nepipolar {ow}x{oh}: {int(want.any(-1).sum())} drawn pixels, threshold margin "
          f"{margin:.3g}, {n_bad} certified near-threshold differences")
    if n_key:
        assert want.any(-1).sum() > 0


def test_epipolar_invalid_args(ctx):
    from erp_match_eightpoint_test_amd import ErpError, epipolar_tool
    k = np.zeros((5, 2), np.float32)
    with pytest.raises(ErpError):
        epipolar_tool(k, k, 100, 50, 10, 10, 8, ctx=ctx)
    with pytest.raises(ErpError):
        epipolar_tool(k, k, 100, 50, 10, 10, 6, ctx=ctx)  # more keys than matches


def _images(rng, H, W):
    import torch
    a = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    return a, b, torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()


@pytest.mark.parametrize("H,W,m,kind", [
    (480, 960, 300, "random"),
    (1024, 2048, 2000, "random"),
    (257, 513, 150, "offimage"),
    (64, 96, 40, "degenerate"),
    (64, 96, 0, "none"),
])
def test_draw_match_matches_oracle(ctx, oracle, H, W, m, kind):
    import torch
    from erp_match_eightpoint_test_amd import feature_matcher
    rng = np.random.default_rng(H + m)
    a, b, ta, tb = _images(rng, H, W)
    if kind == "offimage":  # endpoints up to 20 px outside the image (lines clipped)
        kl = rng.uniform([-20, -20], [W + 20, H + 20], (m, 2))
        kr = rng.uniform([-20, -20], [W + 20, H + 20], (m, 2))
    elif kind == "degenerate":  # points, half-integer rounding, vertical / horizontal runs
        kl = rng.integers(0, [W, H], (m, 2)).astype(np.float64) + 0.5
        kr = kl.copy()
        kr[m // 2:, 0] = kl[m // 2:, 0] + rng.integers(-30, 30, m - m // 2)
        kr[: m // 4, 1] += 40
    else:
        kl = rng.uniform(0, [W, H], (m, 2))
        kr = rng.uniform(0, [W, H], (m, 2))
    kl, kr = kl.astype(np.float32), kr.astype(np.float32)
    fm = feature_matcher(ctx=ctx)
    got = fm.draw_match(ta, tb, torch.from_numpy(kl).cuda(), torch.from_numpy(kr).cuda())
    want = oracle.draw_match(a, b, kl, kr)
    diff = np.argwhere((got.cpu().numpy() != want).any(-1))
    assert len(diff) == 0, (len(diff), diff[:10])


def test_draw_match_stamps_do_not_leak(ctx, oracle):
    """the line buffer is reused across calls (epoch stamps): a call without matches after one
    with many shows no line"""
    import torch
    from erp_match_eightpoint_test_amd import feature_matcher
    rng = np.random.default_rng(9)
    a, b, ta, tb = _images(rng, 100, 200)
    fm = feature_matcher(ctx=ctx)
    k = torch.from_numpy(rng.uniform(0, [200, 100], (50, 2)).astype(np.float32)).cuda()
    assert (fm.draw_match(ta, tb, k, k.flip(0))[..., 2] != 0).any()
    none = torch.zeros((0, 2), dtype=torch.float32, device="cuda")
    assert (fm.draw_match(ta, tb, none, none).cpu().numpy() == oracle.draw_match(a, b, [], [])).all()


def test_draw_match_canvas_grows_between_calls(oracle):
    """one context, a small canvas then larger ones: the grown stamp buffer (possibly at the
    freed address) must be cleared -- stale stamps of the small call must not show as lines"""
    import torch
    from erp_match_eightpoint_test_amd import Context, feature_matcher
    fm = feature_matcher(ctx=Context(0))
    rng = np.random.default_rng(21)
    for H, W, m in ((60, 100, 80), (200, 300, 0), (240, 400, 5), (500, 900, 0)):
        a, b, ta, tb = _images(rng, H, W)
        kl = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
        kr = rng.uniform(0, [W, H], (m, 2)).astype(np.float32)
        got = fm.draw_match(ta, tb, torch.from_numpy(kl).cuda(), torch.from_numpy(kr).cuda())
        want = oracle.draw_match(a, b, kl, kr)
        assert (got.cpu().numpy() == want).all(), (H, W, m)


def test_draw_match_nonfinite_and_far_keypoints(ctx, oracle):
    """a NaN keypoint draws nothing (as a zero-length line far off the canvas); an endpoint
    1e30 px away draws like one at the 2^20 clamp (the walk is clipped to the canvas, bounded)"""
    import torch
    from erp_match_eightpoint_test_amd import feature_matcher
    rng = np.random.default_rng(22)
    a, b, ta, tb = _images(rng, 64, 128)
    kl = np.array([[10, 10], [np.nan, 5], [20, 30], [5, 5]], np.float32)
    kr = np.array([[100, 50], [30, 30], [1e30, 30], [60, 40]], np.float32)
    got = feature_matcher(ctx=ctx).draw_match(ta, tb, torch.from_numpy(kl).cuda(),
                                              torch.from_numpy(kr).cuda()).cpu().numpy()
    kl2, kr2 = kl.copy(), kr.copy()
    kl2[1] = kr2[1] = (-5000, -5000)
    kr2[2] = (1048576, 30)
    assert (got == oracle.draw_match(a, b, kl2, kr2)).all()


def test_device_mismatch_rejected(ctx):
    import torch
    from erp_match_eightpoint_test_amd import feature_matcher
    a = torch.zeros((8, 8, 3), dtype=torch.uint8)
    fm = feature_matcher(ctx=ctx)
    with pytest.raises((ValueError, TypeError)):
        fm.draw_match(a, a, np.zeros((0, 2), np.float32), np.zeros((0, 2), np.float32))


def test_do_all_match_output(ctx):
    import torch
    from erp_match_eightpoint_test_amd import feature_matcher, spherical_surf, synth
    left = synth.sphere_texture(3, 512, 1024)
    right = np.ascontiguousarray(np.roll(left, 24, axis=1))  # a yaw of 8.4 degrees
    ss = spherical_surf(ctx=ctx)
    tl, tr = torch.from_numpy(np.ascontiguousarray(left)).cuda(), torch.from_numpy(
        np.ascontiguousarray(right)).cuda()
    kl, kr, M, total, out = ss.do_all(tl, tr, draw=True)
    assert out.shape == tl.shape and M == kl.shape[0]
    again = feature_matcher(ctx=ctx).draw_match(tl, tr, kl, kr)
    assert torch.equal(out, again)
