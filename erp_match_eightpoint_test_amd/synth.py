"""Seeded synthetic ERP pairs (there is no image data: the reference's config-1 images are
missing blobs and SURF needs OpenCV contrib).  Shapes follow BASELINE.md / SURVEY.md §8d:

* geometry: W x H = 5376 x 2688 (the reference's real ERP size), GT Euler angles uniform in
  [0, 15] deg per axis (two_synthesis_image_test/main.cpp:80-92), unit translation, depths
  U[2, 10]; left bearings uniform on the sphere; right bearing r ~ R^T (depth * l) + t so that
  the reference estimator returns Euler(R) (the right image is rotated by R^-1 in
  two_synthesis_image_test/main.cpp:105);
* pixels from bearings with the OMAF axes of src/eight_point.cpp:179-185; 3/4 of the keypoints
  truncated to integer pixels like the rotated SURF bands (src/spherical_surf.cpp:57-61), 1/4
  fractional like band n1 (:123-124);
* descriptors: SURF 64-D layout (|.| on the sum-|dx|/|dy| slots), L2-normalised; right inliers
  normalise(left + N(0, sigma)) in permuted order; outliers fresh.
"""
from __future__ import annotations

import math

import numpy as np

W_REF, H_REF = 5376, 2688
ABS_SLOTS = np.array([4 * k + 2 for k in range(16)] + [4 * k + 3 for k in range(16)])


def eular2rot(e) -> np.ndarray:
    """R = Rx * Ry * Rz (src/erp_rotation.cpp:14-40)."""
    x, y, z = e
    Rx = np.array([[1, 0, 0], [0, math.cos(x), -math.sin(x)], [0, math.sin(x), math.cos(x)]])
    Ry = np.array([[math.cos(y), 0, math.sin(y)], [0, 1, 0], [-math.sin(y), 0, math.cos(y)]])
    Rz = np.array([[math.cos(z), -math.sin(z), 0], [math.sin(z), math.cos(z), 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def bearing_to_pixel(b: np.ndarray, W: int, H: int) -> np.ndarray:
    b = b / np.linalg.norm(b, axis=1, keepdims=True)
    lat = np.arccos(np.clip(b[:, 2], -1.0, 1.0))
    lon = np.mod(np.arctan2(b[:, 1], -b[:, 0]), 2 * np.pi)
    px = W * lon / (2 * np.pi)
    py = H * lat / np.pi
    px = np.clip(px, 0.0, np.nextafter(W, 0))
    py = np.clip(py, 0.0, np.nextafter(H, 0))
    return np.stack([px, py], 1)


def random_descriptors(rng: np.random.Generator, n: int, dim: int = 64) -> np.ndarray:
    d = rng.standard_normal((n, dim))
    if dim == 64:
        d[:, ABS_SLOTS] = np.abs(d[:, ABS_SLOTS])
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d.astype(np.float32)


def _quantise(rng: np.random.Generator, px: np.ndarray, integer_frac: float) -> np.ndarray:
    px = px.copy()
    trunc = rng.random(px.shape[0]) < integer_frac
    px[trunc] = np.floor(px[trunc])
    return px.astype(np.float32)


def make_pair(seed: int, n_kpts: int = 4096, n_train: int | None = None, W: int = W_REF,
              H: int = H_REF, inlier_frac: float = 0.8, sigma: float = 0.03,
              euler_max_deg: float = 15.0, integer_frac: float = 0.75, dim: int = 64,
              mismatch_frac: float = 0.0) -> dict:
    """One synthetic ERP pair: descriptors + keypoints for left (queries) and right (train).
    mismatch_frac: that fraction of the true partners keep their descriptor but get a random
    right keypoint (wrong matches that pass the ratio test: geometric outliers for the
    consensus); drawn from a second generator, so the other outputs do not change."""
    rng = np.random.default_rng(seed)
    N = n_kpts
    T = n_kpts if n_train is None else n_train
    n_in = min(int(round(inlier_frac * N)), T)
    euler = np.radians(rng.uniform(0.0, euler_max_deg, 3))
    R = eular2rot(euler)
    t = rng.standard_normal(3)
    t /= np.linalg.norm(t)
    # left keypoints / bearings (uniform on the sphere)
    l = rng.standard_normal((N, 3))
    l /= np.linalg.norm(l, axis=1, keepdims=True)
    depth = rng.uniform(2.0, 10.0, N)
    X = l * depth[:, None]
    Xr = X[:n_in] @ R + t  # (R^T X + t) row-wise
    kp_l = _quantise(rng, bearing_to_pixel(l, W, H), integer_frac)
    kp_r_in = _quantise(rng, bearing_to_pixel(Xr, W, H), integer_frac)
    # descriptors
    desc_l = random_descriptors(rng, N, dim)
    noisy = desc_l[:n_in].astype(np.float64) + rng.normal(0.0, sigma, (n_in, dim))
    noisy /= np.linalg.norm(noisy, axis=1, keepdims=True)
    desc_r = np.empty((T, dim), np.float32)
    kp_r = np.empty((T, 2), np.float32)
    perm = rng.permutation(T)  # right slot of each right keypoint
    desc_r[perm[:n_in]] = noisy.astype(np.float32)
    kp_r[perm[:n_in]] = kp_r_in
    n_out = T - n_in
    if n_out:
        desc_r[perm[n_in:]] = random_descriptors(rng, n_out, dim)
        ro = rng.standard_normal((n_out, 3))
        kp_r[perm[n_in:]] = _quantise(rng, bearing_to_pixel(ro, W, H), integer_frac)
    if mismatch_frac > 0 and n_in:
        rng2 = np.random.default_rng(seed + 1_000_003)
        bad = rng2.random(n_in) < mismatch_frac
        rb = rng2.standard_normal((int(bad.sum()), 3))
        kp_r[perm[:n_in][bad]] = _quantise(rng2, bearing_to_pixel(rb, W, H), integer_frac)
    gt_partner = np.full(N, -1, np.int64)
    gt_partner[:n_in] = perm[:n_in]
    return {"desc_l": desc_l, "desc_r": desc_r, "kp_l": kp_l, "kp_r": kp_r, "W": W, "H": H,
            "euler_gt": euler, "t_gt": t, "gt_partner": gt_partner}


def make_correspondences(seed: int, m: int = 100, outlier_frac: float = 0.6, W: int = 2048,
                         H: int = 1024, euler_max_deg: float = 15.0, integer: bool = True) -> dict:
    """Manual-pickup regime (manual_point_pickup_test, build/config_file.ini:4-6): m matched
    keypoint pairs at integer pixels of a 2048x1024 ERP, a fraction of them outliers."""
    rng = np.random.default_rng(seed)
    euler = np.radians(rng.uniform(0.0, euler_max_deg, 3))
    R = eular2rot(euler)
    t = rng.standard_normal(3)
    t /= np.linalg.norm(t)
    l = rng.standard_normal((m, 3))
    l /= np.linalg.norm(l, axis=1, keepdims=True)
    X = l * rng.uniform(2.0, 10.0, m)[:, None]
    r = X @ R + t
    n_out = int(round(outlier_frac * m))
    if n_out:
        idx = rng.choice(m, n_out, replace=False)
        r[idx] = rng.standard_normal((n_out, 3))
    kl = bearing_to_pixel(l, W, H)
    kr = bearing_to_pixel(r, W, H)
    if integer:
        kl, kr = np.floor(kl), np.floor(kr)
    return {"kp_l": kl.astype(np.float32), "kp_r": kr.astype(np.float32), "W": W, "H": H,
            "euler_gt": euler, "t_gt": t}


def sphere_texture(seed: int, H: int, W: int, n_blobs: int = 500) -> np.ndarray:
    """an H x W x 3 (BGR) ERP image of random Gaussian blobs on the unit sphere (OMAF axes):
    synthetic input for the band remap / SURF / end-to-end pipeline (the reference's images
    are missing blobs)"""
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
