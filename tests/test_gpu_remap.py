"""GPU parity of the ERP remaps against the oracle: band remap
(crop_rotated_image x3 + the unrotated band), keypoint un-rotation, rotate_image, rectify and
the vertical view.  Outputs are pre-filled with the same sentinel on both sides, so pixels the
reference leaves unwritten compare too.

Bar: byte-exact, except output pixels whose reference value before the truncating int
conversion (rotate_pixel's H*acos(.)/M_PI or W*atan2(.)/(2*M_PI)) lies within 1e-9 of an
integer: there the index is decided by the last ulp of libm's sin/cos/acos/atan2.  The kernels
recompute such pixels with correctly rounded transcendentals; glibc (the reference's libm,
whose algorithms are not available to restate) misrounds ~0.1 % of near-midpoint cases, and
only those pixels may differ.  Each is certified by the oracle's pre-truncation values; any
other difference fails.  Generic rotations have none; exact multiples of 90 degrees and the
identity put whole pixel rows on those boundaries."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rctx(gpu_lib):
    from erp_match_eightpoint_test_amd import Context
    return Context(0)


def _image(seed, H, W):
    """a textured synthetic ERP image (smooth gradients + noise, so remap errors show)"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    base = np.stack([(x * 7 + y * 3) % 256, (x * 2 + y * 11) % 256, (x ^ y) % 256], -1)
    return ((base + rng.integers(0, 16, (H, W, 3))) % 256).astype(np.uint8)


def _certify(got, ref, src_of, m, W, H, tol=1e-9):
    """differences between got and ref must all be truncation-boundary pixels: src_of(idx) maps
    the differing output pixel indices [n, 2] to rotate_pixel's (row, col) inputs.  Returns the
    number of certified boundary differences."""
    import oracle as O
    bad = np.argwhere(np.any(got != ref, axis=-1))
    if len(bad) == 0:
        return 0
    rows, cols = src_of(bad)
    v = O.rotate_pixel_prefix(rows, cols, m, W, H)
    dist = np.abs(v - np.round(v)).min(axis=1)
    worst = np.argmax(dist)
    assert dist.max() < tol, (len(bad), bad[worst], v[worst], dist.max())
    print(f"certified boundary pixels: {len(bad)} of {got.shape[0] * got.shape[1]}")
    return len(bad)


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("H,W", [(64, 128), (336, 672), (1344, 2688), (2688, 5376)])
def test_spherical_bands(rctx, oracle, H, W):
    from erp_match_eightpoint_test_amd import spherical_surf
    ims = np.stack([_image(H + k, H, W) for k in range(3)])
    got = spherical_surf(ctx=rctx).bands(_dev(ims), fill=7).cpu().numpy()
    r0 = H * 3 // 8
    for k in range(3):
        ref = oracle.spherical_bands(ims[k], fill=7)
        assert np.array_equal(got[k, 1], ref[1])
        for b, pitch in ((0, 45.0), (2, -45.0), (3, -90.0)):
            n = _certify(got[k, b], ref[b], lambda ix: (ix[:, 0] + r0, ix[:, 1]),
                         oracle.pitch_matrix(pitch), W, H)
            if pitch != -90.0:
                assert n == 0, (k, b, n)


@pytest.mark.parametrize("pitch", [45.0, -45.0, -90.0, 30.0, 0.0])
def test_crop_rotated_image(rctx, oracle, pitch):
    from erp_match_eightpoint_test_amd import spherical_surf
    im = _image(5, 672, 1344)
    got = spherical_surf(ctx=rctx).crop_rotated_image(pitch, _dev(im), fill=3).cpu().numpy()
    n = _certify(got, oracle.crop_rotated_image(im, pitch, fill=3),
                 lambda ix: (ix[:, 0] + 672 * 3 // 8, ix[:, 1]), oracle.pitch_matrix(pitch),
                 1344, 672)
    if pitch in (45.0, -45.0, 30.0):
        assert n == 0


def test_unrotate_band_keypoints(rctx, oracle):
    import torch
    from erp_match_eightpoint_test_amd import spherical_surf
    rng = np.random.default_rng(2)
    W, H = 5376, 2688
    counts = [3000, 2500, 2800, 0]
    n = sum(counts)
    kp = np.stack([rng.uniform(0, W, n), rng.uniform(0, H // 4, n)], 1).astype(np.float32)
    kp[:20] = np.floor(kp[:20])                      # integer keypoints
    kp[20] = [W - 1e-3, H / 4 - 1e-3]                 # edge of the band
    kp[21] = [np.nan, 5.0]                            # x86 INT_MIN conversion path
    for cnt in (counts, [1000, 1000, 1000, 5300]):
        t = _dev(kp)
        spherical_surf(ctx=rctx).unrotate_band_keypoints(t, cnt, W, H)
        torch.cuda.synchronize()
        ref = oracle.unrotate_band_keypoints(kp, cnt, W, H)
        assert np.array_equal(t.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_rotate_keypoint(rctx, oracle):
    from erp_match_eightpoint_test_amd import spherical_surf
    rng = np.random.default_rng(4)
    W, H = 2048, 1024
    kp = np.stack([rng.uniform(0, W, 5000), rng.uniform(0, H // 4, 5000)], 1).astype(np.float32)
    for pitch in (45.0, -45.0, -90.0, 12.5):
        t = spherical_surf(ctx=rctx).rotate_keypoint(pitch, _dev(kp), W, H)
        ref = oracle.rotate_keypoint(kp, pitch, W, H)
        assert np.array_equal(t.cpu().numpy().view(np.uint32), ref.view(np.uint32)), pitch


@pytest.mark.parametrize("H,W", [(100, 200), (672, 1344), (2688, 5376)])
def test_rotate_image(rctx, oracle, H, W):
    from erp_match_eightpoint_test_amd import erp_rotation
    er = erp_rotation(ctx=rctx)
    im = _image(W, H, W)
    for th in ([0.1, -0.2, 0.3], [0.0, 0.0, 0.0], [np.pi / 2, 0, 0]):
        R = oracle.eular2rot(th)
        got = er.rotate_image(_dev(im), R, fill=9).cpu().numpy()
        n = _certify(got, oracle.rotate_image(im, R, fill=9), lambda ix: (ix[:, 0], ix[:, 1]),
                     oracle.inv3(R), W, H)
        if th[0] == 0.1:
            assert n == 0


def test_rectify_and_vertical(rctx, oracle):
    from erp_match_eightpoint_test_amd import erp_rotation
    er = erp_rotation(ctx=rctx)
    H, W = 1344, 2688
    L_, R_ = _image(1, H, W), _image(2, H, W)
    rv = np.array([0.05, -0.12, 0.03], np.float32).astype(np.float64)  # Vec3f -> Vec3d
    tv = np.array([0.6, 0.1, -0.79], np.float32).astype(np.float64)
    lo, ro = er.rectify(_dev(L_), _dev(R_), rv, tv, fill=1)
    rl, rr = oracle.rectify(L_, R_, rv, tv, fill=1)
    assert np.array_equal(lo.cpu().numpy(), rl) and np.array_equal(ro.cpu().numpy(), rr)
    # the vertical view of the SAME rectified image on both sides
    v = er.vertical_rotate(_dev(rl), fill=2).cpu().numpy()
    assert v.shape == (W, H, 3)
    th = np.pi * 89.999 / 180.0
    m = oracle.inv3(oracle.inv3(oracle.eular2rot([th, 0, 0])))
    _certify(v, oracle.vertical_rotate(rl, fill=2), lambda ix: (H - 1 - ix[:, 1], ix[:, 0]),
             m, W, H)


def test_rotate_image_random_rotations(rctx, oracle):
    """rotate_image under 10 random rotations (the seams, the poles and arbitrary boundary
    crossings inside the view) against the oracle's literal double formula: byte-exact up to the
    certified truncation-boundary pixels (the fp64 fast path and its correctly rounded deferral
    band, remap.hip)"""
    from erp_match_eightpoint_test_amd import erp_rotation
    er = erp_rotation(ctx=rctx)
    H, W = 672, 1344
    im = _image(77, H, W)
    rng = np.random.default_rng(2024)
    for _ in range(10):
        th = rng.uniform(-np.pi, np.pi, 3)
        R = oracle.eular2rot(th)
        got = er.rotate_image(_dev(im), R, fill=4).cpu().numpy()
        _certify(got, oracle.rotate_image(im, R, fill=4), lambda ix: (ix[:, 0], ix[:, 1]),
                 oracle.inv3(R), W, H)
