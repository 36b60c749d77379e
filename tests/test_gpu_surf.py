"""GPU SURF against the oracle's restatement (oracle/erp_surf.c).

Bars: keypoints (x, y, size, response, octave, class_id, angle) bit-exact and in the same
KeypointGreater order -- the detector and the orientation are integer / float / double work
repeated operation for operation; descriptors bit-exact except for keypoints whose rotated
window sin / cos differ between glibc's sinf / cosf (the oracle) and the device's double sin /
cos rounded to float -- certified per keypoint with libm on the host (measured: no such
keypoint in any test so far, every descriptor bit-exact).  Parity with OpenCV itself is
unpinned (OpenCV is absent)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scene(seed, H, W, color=False):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    img = np.zeros((H, W))
    for _ in range(H * W // 2500):
        cx, cy, r = rng.uniform(0, W), rng.uniform(0, H), rng.uniform(2, 25)
        img += rng.uniform(-90, 90) * np.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * r * r))
    img = np.clip(img + 128 + rng.normal(0, 4, (H, W)), 0, 255).astype(np.uint8)
    if color:
        img = np.stack([img, np.roll(img, 3, 1), np.roll(img, 5, 0)], -1)
    return img


@pytest.fixture(scope="module")
def fm(gpu_lib):
    from erp_match_eightpoint_test_amd import Context, feature_matcher
    return feature_matcher(ctx=Context(0))


def _sincos_differ(angle_deg: np.ndarray) -> np.ndarray:
    """keypoints whose rotated-window sin/cos may differ between the oracle (glibc sinf / cosf
    of the float angle in radians) and the device (the double sin / cos rounded to float)"""
    import ctypes
    import math
    libm = ctypes.CDLL("libm.so.6")
    libm.sinf.restype = libm.cosf.restype = ctypes.c_float
    libm.sinf.argtypes = libm.cosf.argtypes = [ctypes.c_float]
    out = np.zeros(len(angle_deg), bool)
    for k, a in enumerate(angle_deg):
        d = float(np.float32(a) * np.float32(math.pi / 180))
        out[k] = (np.float32(libm.sinf(d)) != np.float32(math.sin(d))
                  or np.float32(libm.cosf(d)) != np.float32(math.cos(d)))
    return out


def _compare(kg, dg, ko, do):
    """keypoints and angles bit-exact; descriptors bit-exact except where the window's sin / cos
    provably differ between glibc's sinf / cosf and the device's rounded double (certified per
    keypoint; none so far)"""
    assert len(kg) == len(ko), (len(kg), len(ko))
    for f in ("x", "y", "size", "response", "octave", "class_id", "angle"):
        assert np.array_equal(kg[f], ko[f]), f
    dd = np.abs(dg - do).max(axis=1) if len(dg) else np.zeros(0)
    differ = dd != 0
    certified = _sincos_differ(ko["angle"][differ]) if differ.any() else np.zeros(0, bool)
    print(f"\n{len(kg)} keypoints: angles exact, {int(differ.sum())} descriptors not bit-exact "
          f"(max {dd.max() if len(dd) else 0:.3g}), {int(certified.sum())} of them certified")
    assert certified.all(), np.flatnonzero(differ)[~certified][:10]
    assert (dd[differ] <= 2e-3).all()
    assert np.allclose(np.linalg.norm(dg, axis=1), 1.0, atol=1e-5)


@pytest.mark.parametrize("H,W", [(96, 160), (336, 672), (672, 1344)])
def test_surf_gray_vs_oracle(fm, oracle, H, W):
    import torch
    img = _scene(H + W, H, W)
    kg, dg = fm.surf(torch.from_numpy(img).cuda())
    ko, do = oracle.surf(img)
    assert len(ko) > (0 if H < 200 else 10)
    _compare(kg[0], dg[0], ko, do)


def test_surf_bgr_batch_vs_oracle(fm, oracle):
    import torch
    ims = np.stack([_scene(40 + k, 336, 1344, color=True) for k in range(3)])
    kg, dg = fm.surf(torch.from_numpy(ims).cuda())
    for k in range(3):
        ko, do = oracle.surf(ims[k])
        _compare(kg[k], dg[k], ko, do)


def test_surf_band_size_and_small_max_kp(fm, oracle):
    """a full 5376 x 2688 band (672 x 5376) and a max_kp smaller than the count (the binding
    reruns with the size the device reported)"""
    import torch
    img = _scene(7, 672, 5376)
    kg, dg = fm.surf(torch.from_numpy(img).cuda(), max_kp=64)
    ko, do = oracle.surf(img)
    assert len(ko) > 64
    _compare(kg[0], dg[0], ko, do)


def test_surf_flat_image(fm):
    import torch
    kg, dg = fm.surf(torch.full((200, 300), 77, dtype=torch.uint8, device="cuda"))
    assert len(kg[0]) == 0 and dg[0].shape == (0, 64)


def _sphere_texture(seed, H, W, n_blobs=500):
    """an ERP image of random Gaussian blobs on the unit sphere (OMAF axes), BGR"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    lat, lon = np.pi * (y + 0.5) / H, 2 * np.pi * (x + 0.5) / W
    b = np.stack([-np.sin(lat) * np.cos(lon), np.sin(lat) * np.sin(lon), np.cos(lat)], -1)
    c = rng.standard_normal((n_blobs, 3))
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    sig = rng.uniform(0.01, 0.06, n_blobs)
    amp = rng.uniform(-120, 120, (n_blobs, 3))
    img = np.full((H, W, 3), 128.0)
    for k in range(n_blobs):
        d2 = ((b - c[k]) ** 2).sum(-1)
        m = d2 < (4 * sig[k]) ** 2
        img[m] += amp[k] * np.exp(-d2[m] / (2 * sig[k] ** 2))[:, None]
    return np.clip(img, 0, 255).astype(np.uint8)


def test_do_all_end_to_end_kat(gpu_lib, oracle):
    """spherical_surf::do_all end to end on the GPU (bands -> SURF x 8 -> un-rotation -> match
    -> gather) on a synthetic ERP pair related by a known camera rotation, the reference's own
    one_image_test/main.cpp:73-145 experiment: im2 = rotate_image(im, R^-1), i.e.
    im2(p) = im(rotate_pixel(p, R)), so a left keypoint q must reappear at rotate_pixel(q, R^-1)
    (median angular error below 0.5 degree, the test's 'Surf match error'); and the match list
    agrees with the same pipeline on the oracle for >= 95 % of the pairs."""
    import torch
    from erp_match_eightpoint_test_amd import Context, erp_rotation, spherical_surf
    H, W = 672, 1344
    im = _sphere_texture(3, H, W)
    R = oracle.eular2rot(np.radians([10.0, 5.0, 15.0]))
    ctx = Context(0)
    er = erp_rotation(ctx=ctx)
    im2 = er.rotate_image(torch.from_numpy(im).cuda(), oracle.inv3(R))
    kl, kr, M, total = spherical_surf(ctx=ctx).do_all(torch.from_numpy(im).cuda(), im2)
    assert M > 50 and total > M
    kl, kr = kl.cpu().numpy(), kr.cpu().numpy()
    Ri = oracle.inv3(R)
    pr = np.array([oracle.rotate_pixel(int(p[1]), int(p[0]), Ri, W, H) for p in kl], float)

    def bear(px, py):
        lat, lon = np.pi * py / H, 2 * np.pi * px / W
        return np.stack([np.sin(lat) * np.cos(lon), np.sin(lat) * np.sin(lon), np.cos(lat)], -1)
    err = np.degrees(np.arccos(np.clip((bear(pr[:, 1], pr[:, 0]) * bear(kr[:, 0], kr[:, 1])).sum(-1), -1, 1)))
    assert np.median(err) < 0.5, np.median(err)
    # the same pipeline on the oracle
    im2h = im2.cpu().numpy()
    keys, descs = [], []
    for img in (im, im2h):
        b = oracle.spherical_bands(img)
        kd = [oracle.surf(b[k]) for k in range(4)]
        pts = np.concatenate([np.stack([k["x"], k["y"]], 1) for k, _ in kd]).astype(np.float32)
        keys.append(oracle.unrotate_band_keypoints(pts, [len(k) for k, _ in kd], W, H))
        descs.append(np.concatenate([d for _, d in kd]))
    mt, _, _, _ = oracle.match_two_image(descs[0], descs[1])
    ref = {(tuple(keys[0][q]), tuple(keys[1][t])) for q, t in zip(mt["queryIdx"], mt["trainIdx"])}
    got = {(tuple(a), tuple(b)) for a, b in zip(kl, kr)}
    assert len(ref & got) >= 0.95 * max(len(ref), len(got)), (len(ref), len(got), len(ref & got))
