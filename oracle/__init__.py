"""ctypes wrapper of the CPU oracle (oracle/erp_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; it
is the parity checker, never the thing measured or shipped.  Every function cites the
reference file:line it restates in oracle/erp_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liberp_oracle.so")


class DMatch(C.Structure):
    _fields_ = [("queryIdx", C.c_int32), ("trainIdx", C.c_int32), ("imgIdx", C.c_int32),
                ("distance", C.c_float)]


DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"),
                         ("distance", "<f4")])


class Glibc(C.Structure):
    _fields_ = [("r", C.c_uint32 * 34), ("pos", C.c_uint32)]


class Hyp(C.Structure):
    _fields_ = [("R1", C.c_float * 3), ("R2", C.c_float * 3), ("T", C.c_float * 3),
                ("R1_valid", C.c_int32), ("R2_valid", C.c_int32), ("inliers", C.c_int32),
                ("E", C.c_double * 9), ("E_corr", C.c_double * 9)]


HYP_DTYPE = np.dtype([("R1", "<f4", 3), ("R2", "<f4", 3), ("T", "<f4", 3), ("R1_valid", "<i4"),
                      ("R2_valid", "<i4"), ("inliers", "<i4"), ("E", "<f8", 9),
                      ("E_corr", "<f8", 9)], align=True)
assert HYP_DTYPE.itemsize == C.sizeof(Hyp)


class Cfg(C.Structure):
    _fields_ = [("iters", C.c_int32), ("sample_frac", C.c_double), ("trim_lo", C.c_double),
                ("trim_hi", C.c_double), ("valid_abs", C.c_double), ("seed", C.c_uint32),
                ("offset", C.c_uint64), ("sampler", C.c_int32), ("inlier_thr", C.c_double)]


class Diag(C.Structure):
    _fields_ = [("K", C.c_int32), ("min_idx", C.c_int32), ("sample_n", C.c_int32),
                ("status", C.c_int32), ("min_dist", C.c_double)]


class SurfParams(C.Structure):
    _fields_ = [("hessian_threshold", C.c_double), ("n_octaves", C.c_int32),
                ("n_octave_layers", C.c_int32)]


KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc only; no reference sources involved)."""
    if force or not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(os.path.join(HERE, f))
                                             for f in ("erp_oracle.c", "erp_surf.c", "erp_viz.c",
                                                       "erp_oracle.h"))):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.erpo_glibc_seed.argtypes = [C.POINTER(Glibc), C.c_uint32]
        L.erpo_glibc_rand.argtypes = [C.POINTER(Glibc)]
        L.erpo_glibc_rand.restype = C.c_int32
        L.erpo_glibc_discard.argtypes = [C.POINTER(Glibc), C.c_uint64]
        L.erpo_glibc_window.argtypes = [C.POINTER(Glibc), P]
        L.erpo_random_array.argtypes = [P, C.c_int32, C.POINTER(Glibc)]
        L.erpo_philox4x32.argtypes = [P, P, P]
        L.erpo_philox_sample.argtypes = [C.c_int32, C.c_int32, C.c_uint64, C.c_uint32, P]
        L.erpo_l2sq.argtypes = [P, P, C.c_int32]
        L.erpo_l2sq.restype = C.c_float
        L.erpo_match_two_image.argtypes = [P, C.c_int32, P, C.c_int32, C.c_int32, C.c_float, P, P,
                                           P, P, C.c_int32]
        L.erpo_match_two_image.restype = C.c_int32
        L.erpo_eular2rot.argtypes = [P, P]
        L.erpo_rot2eular.argtypes = [P, P]
        L.erpo_pixel_to_bearing.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, P]
        L.erpo_svdecomp.argtypes = [P, C.c_int32, C.c_int32, P, P, P]
        L.erpo_svdecomp.restype = C.c_int
        L.erpo_rank2.argtypes = [P, P]
        L.erpo_rank2.restype = None
        L.erpo_inlier_count.argtypes = [P, P, C.c_int32, P, C.c_double, C.c_double,
                                        C.POINTER(C.c_int32)]
        L.erpo_inlier_count.restype = C.c_int32
        L.erpo_eight_point_estimation.argtypes = [P, P, C.c_int32, C.POINTER(Hyp)]
        L.erpo_eight_point_estimation.restype = C.c_int
        L.erpo_consensus.argtypes = [P, C.c_int32, C.c_double, C.c_double, C.POINTER(C.c_int32), P]
        L.erpo_consensus.restype = C.c_int
        L.erpo_initial_guess.argtypes = [P, P, C.c_int32, C.POINTER(Cfg), P, P, C.POINTER(Diag), P,
                                         P, P, P, P]
        L.erpo_initial_guess.restype = C.c_int
        L.erpo_find.argtypes = [C.c_int32, C.c_int32, P, P, C.c_int32, C.POINTER(Cfg), P, P,
                                C.POINTER(Diag), P, P, P, P, P]
        L.erpo_find.restype = C.c_int
        L.erpo_rotate_pixel.argtypes = [C.c_int32, C.c_int32, P, C.c_int32, C.c_int32, P]
        L.erpo_rotate_pixel_prefix.argtypes = [P, P, C.c_int32, P, C.c_int32, C.c_int32, P]
        L.erpo_surf.argtypes = [P, C.c_int32, C.c_int32, C.c_int32, C.POINTER(SurfParams), P, P,
                                C.c_int32]
        L.erpo_surf.restype = C.c_int32
        L.erpo_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.erpo_fast_atan2.restype = C.c_float
        L.erpo_gray_bgr.argtypes = [P, C.c_int32, C.c_int32, P]
        L.erpo_integral.argtypes = [P, C.c_int32, C.c_int32, P]
        L.erpo_resize_area.argtypes = [P, C.c_int, P, C.c_int]
        L.erpo_inv3.argtypes = [P, P]
        L.erpo_inv3.restype = C.c_int32
        L.erpo_rot_from_vec.argtypes = [P, P, P]
        L.erpo_crop_rotated_image.argtypes = [P, C.c_int32, C.c_int32, C.c_float, P]
        L.erpo_rotate_keypoint.argtypes = [P, C.c_int32, C.c_float, C.c_int32, C.c_int32]
        L.erpo_unrotate_band_keypoints.argtypes = [P, P, C.c_int32, C.c_int32]
        L.erpo_rotate_image.argtypes = [P, C.c_int32, C.c_int32, P, P]
        L.erpo_rotate_image.restype = C.c_int32
        L.erpo_rectify.argtypes = [P, P, C.c_int32, C.c_int32, P, P, P, P]
        L.erpo_rectify.restype = C.c_int32
        L.erpo_vertical_rotate.argtypes = [P, C.c_int32, C.c_int32, P]
        L.erpo_vertical_rotate.restype = C.c_int32
        L.erpo_epipolar_draw.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_int32, C.c_uint32, C.c_uint64, P, P, P, P]
        L.erpo_epipolar_draw.restype = C.c_int32
        L.erpo_epipolar_value.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32]
        L.erpo_epipolar_value.restype = C.c_double
        L.erpo_hsv2bgr.argtypes = [C.c_int, C.c_int, C.c_int, P]
        L.erpo_draw_match.argtypes = [P, P, C.c_int32, C.c_int32, P, P, C.c_int32, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def make_cfg(iters=80, sample_frac=0.25, trim_lo=0.2, trim_hi=0.8, valid_abs=1.57, seed=1,
             offset=0, sampler=0, inlier_thr=0.0) -> Cfg:
    """Reference defaults: src/eight_point.cpp:99 (80), :102 (0.25), :143 (0.2/0.8), :76 (1.57).
    sampler 1: the counter-based Philox sampler (no reference counterpart; erp_oracle.c);
    inlier_thr > 0: every iteration's inlier count into hyp["inliers"] (no counterpart)."""
    return Cfg(iters, sample_frac, trim_lo, trim_hi, valid_abs, seed, offset, sampler,
               float(inlier_thr))


def rank2(e) -> np.ndarray:
    """E_mat_correct of a solved 9-vector (src/eight_point.cpp:45-50) -> 9 doubles"""
    e = np.ascontiguousarray(e, np.float64).reshape(9)
    Ec = np.zeros(9, np.float64)
    lib().erpo_rank2(_p(e), _p(Ec))
    return Ec


def inlier_count(bl, br, Ec, thr: float, band: float = 0.0):
    """(count of |l^T Ec r| < thr in erp_match.h's fixed fp64 order, matches within `band` of
    the threshold)"""
    bl = np.ascontiguousarray(bl, np.float64).reshape(-1, 3)
    br = np.ascontiguousarray(br, np.float64).reshape(-1, 3)
    Ec = np.ascontiguousarray(Ec, np.float64).reshape(9)
    nb = C.c_int32(0)
    n = lib().erpo_inlier_count(_p(bl), _p(br), bl.shape[0], _p(Ec), float(thr), float(band),
                                C.byref(nb))
    return int(n), int(nb.value)


def philox4x32(ctr, key) -> np.ndarray:
    """One Philox4x32-10 block (Random123 constants)."""
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().erpo_philox4x32(_p(c), _p(k), _p(o))
    return o


def philox_sample(m: int, s: int, h: int, seed: int = 1) -> np.ndarray:
    """The Philox sampler's s-subset of [0, m) for iteration counter h (ascending)."""
    out = np.zeros(max(s, 1), np.int32)
    lib().erpo_philox_sample(m, s, C.c_uint64(h), C.c_uint32(seed), _p(out))
    return out[:s]


class GlibcRand:
    """glibc rand() restatement (seed 1 = never seeded, as in the reference)."""

    def __init__(self, seed: int = 1, offset: int = 0):
        self.g = Glibc()
        lib().erpo_glibc_seed(C.byref(self.g), seed)
        if offset:
            lib().erpo_glibc_discard(C.byref(self.g), offset)

    def rand(self) -> int:
        return lib().erpo_glibc_rand(C.byref(self.g))

    def window(self) -> np.ndarray:
        w = np.zeros(31, np.uint32)
        lib().erpo_glibc_window(C.byref(self.g), _p(w))
        return w

    def random_array(self, n: int) -> np.ndarray:
        a = np.zeros(max(n, 1), np.int32)
        lib().erpo_random_array(_p(a), n, C.byref(self.g))
        return a[:n]


def match_two_image(q: np.ndarray, t: np.ndarray, ratio: float = 0.3, nthreads: int = 0):
    """Exact k=2 + Lowe ratio (src/feature_matcher.cpp:42-59).

    Returns (matches structured array, best (nq,), d0sq (nq,), d1sq (nq,))."""
    q = np.ascontiguousarray(q, np.float32)
    t = np.ascontiguousarray(t, np.float32)
    nq, dim = q.shape
    nt = t.shape[0]
    out = np.zeros(max(nq, 1), DMATCH_DTYPE)
    best = np.zeros(max(nq, 1), np.int32)
    d0 = np.zeros(max(nq, 1), np.float32)
    d1 = np.zeros(max(nq, 1), np.float32)
    m = lib().erpo_match_two_image(_p(q), nq, _p(t), nt, dim, ratio, _p(out), _p(best), _p(d0),
                                   _p(d1), nthreads)
    if m < 0:
        raise ValueError(f"erpo_match_two_image failed ({m})")
    return out[:m].copy(), best[:nq], d0[:nq], d1[:nq]


def l2sq(a: np.ndarray, b: np.ndarray) -> float:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return lib().erpo_l2sq(_p(a), _p(b), a.shape[0])


def eular2rot(e) -> np.ndarray:
    e = np.ascontiguousarray(e, np.float64)
    R = np.zeros(9, np.float64)
    lib().erpo_eular2rot(_p(e), _p(R))
    return R.reshape(3, 3)


def rot2eular(R) -> np.ndarray:
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    e = np.zeros(3, np.float64)
    lib().erpo_rot2eular(_p(R), _p(e))
    return e


def pixel_to_bearing(W: int, H: int, kp: np.ndarray) -> np.ndarray:
    kp = np.asarray(kp, np.float32).reshape(-1, 2)
    out = np.zeros((kp.shape[0], 3), np.float64)
    b = np.zeros(3, np.float64)
    for i in range(kp.shape[0]):
        lib().erpo_pixel_to_bearing(W, H, float(kp[i, 0]), float(kp[i, 1]), _p(b))
        out[i] = b
    return out


def svdecomp(a: np.ndarray):
    a = np.ascontiguousarray(a, np.float64)
    m, n = a.shape
    k = min(m, n)
    w = np.zeros(k, np.float64)
    u = np.zeros((m, k), np.float64)
    vt = np.zeros((k, n), np.float64)
    if lib().erpo_svdecomp(_p(a), m, n, _p(w), _p(u), _p(vt)) != 0:
        raise ValueError("svdecomp failed")
    return w, u, vt


def eight_point_estimation(bl: np.ndarray, br: np.ndarray) -> np.ndarray:
    bl = np.ascontiguousarray(bl, np.float64)
    br = np.ascontiguousarray(br, np.float64)
    h = Hyp()
    rc = lib().erpo_eight_point_estimation(_p(bl), _p(br), bl.shape[0], C.byref(h))
    if rc != 0:
        raise ValueError(f"eight_point_estimation failed ({rc})")
    return np.frombuffer(bytes(h), HYP_DTYPE)[0]


def consensus(rvec: np.ndarray, trim_lo=0.2, trim_hi=0.8):
    rvec = np.ascontiguousarray(rvec, np.float32).reshape(-1, 3)
    K = rvec.shape[0]
    mi = C.c_int32(0)
    dist = np.zeros(max(K, 1), np.float64)
    rc = lib().erpo_consensus(_p(rvec), K, trim_lo, trim_hi, C.byref(mi), _p(dist))
    return rc, mi.value, dist[:K]


def _run_guess(fn, args, m, cfg: Cfg, want_detail: bool):
    iters = cfg.iters
    sample_n = int(m * cfg.sample_frac) if m > 0 else 0
    R = np.zeros(3, np.float32)
    T = np.zeros(3, np.float32)
    diag = Diag()
    hyp = np.zeros(max(iters, 1), HYP_DTYPE) if want_detail else None
    samples = np.zeros(max(iters * sample_n, 1), np.int32) if want_detail else None
    rvec = np.zeros((max(2 * iters, 1), 3), np.float32) if want_detail else None
    tvec = np.zeros((max(2 * iters, 1), 3), np.float32) if want_detail else None
    dist = np.zeros(max(2 * iters, 1), np.float64) if want_detail else None
    rc = fn(*args, C.byref(cfg), _p(R), _p(T), C.byref(diag), _p(hyp), _p(samples), _p(rvec),
            _p(tvec), _p(dist))
    res = {"rc": rc, "R": R, "T": T, "K": diag.K, "min_idx": diag.min_idx,
           "sample_n": diag.sample_n, "status": diag.status, "min_dist": diag.min_dist}
    if want_detail:
        K = max(diag.K, 0)
        res.update(hyp=hyp[:iters], samples=samples[:iters * sample_n].reshape(iters, sample_n),
                   rvec=rvec[:K], tvec=tvec[:K], dist=dist[:K])
    return res


def initial_guess(bl, br, cfg: Cfg | None = None, detail: bool = False):
    cfg = cfg or make_cfg()
    bl = np.ascontiguousarray(bl, np.float64)
    br = np.ascontiguousarray(br, np.float64)
    m = bl.shape[0]
    return _run_guess(lib().erpo_initial_guess, (_p(bl), _p(br), m), m, cfg, detail)


def find(W: int, H: int, kl, kr, cfg: Cfg | None = None, detail: bool = False):
    """eight_point::find (src/eight_point.cpp:152-192) on pixel keypoints (m x 2 float)."""
    cfg = cfg or make_cfg()
    kl = np.ascontiguousarray(kl, np.float32).reshape(-1, 2)
    kr = np.ascontiguousarray(kr, np.float32).reshape(-1, 2)
    m = kl.shape[0]
    return _run_guess(lib().erpo_find, (W, H, _p(kl), _p(kr), m), m, cfg, detail)


# ------------------------------------------------------------------ ERP remaps (section 8f)
def _img(im):
    im = np.ascontiguousarray(im, np.uint8)
    assert im.ndim == 3 and im.shape[2] == 3
    return im


def rotate_pixel(row: int, col: int, m, W: int, H: int) -> tuple[int, int]:
    m = np.ascontiguousarray(m, np.float64).reshape(9)
    o = np.zeros(2, np.int32)
    lib().erpo_rotate_pixel(int(row), int(col), _p(m), W, H, _p(o))
    return int(o[0]), int(o[1])


def inv3(m) -> np.ndarray:
    m = np.ascontiguousarray(m, np.float64).reshape(9)
    o = np.zeros(9, np.float64)
    if not lib().erpo_inv3(_p(m), _p(o)):
        raise ValueError("singular")
    return o.reshape(3, 3)


def rot_from_vec(v1, v2) -> np.ndarray:
    a = np.ascontiguousarray(v1, np.float64)
    b = np.ascontiguousarray(v2, np.float64)
    R = np.zeros(9, np.float64)
    lib().erpo_rot_from_vec(_p(a), _p(b), _p(R))
    return R.reshape(3, 3)


def crop_rotated_image(im, pitch_deg: float, fill: int = 0) -> np.ndarray:
    im = _img(im)
    H, W = im.shape[:2]
    out = np.full((H // 4, W, 3), fill, np.uint8)
    lib().erpo_crop_rotated_image(_p(im), W, H, pitch_deg, _p(out))
    return out


def spherical_bands(im, fill: int = 0) -> np.ndarray:
    """do_all's four bands (src/spherical_surf.cpp:77-83): [4, H/4, W, 3]"""
    im = _img(im)
    H = im.shape[0]
    n1 = im[H * 3 // 8: H * 3 // 8 + H // 4]
    return np.stack([crop_rotated_image(im, 45.0, fill), n1, crop_rotated_image(im, -45.0, fill),
                     crop_rotated_image(im, -90.0, fill)])


def rotate_keypoint(kp, pitch_deg: float, W: int, H: int) -> np.ndarray:
    kp = np.array(kp, np.float32).reshape(-1, 2)
    lib().erpo_rotate_keypoint(_p(kp), kp.shape[0], pitch_deg, W, H)
    return kp


def unrotate_band_keypoints(kp, counts, W: int, H: int) -> np.ndarray:
    kp = np.array(kp, np.float32).reshape(-1, 2)
    c = np.ascontiguousarray(counts, np.int32)
    assert c.sum() == kp.shape[0]
    lib().erpo_unrotate_band_keypoints(_p(kp), _p(c), W, H)
    return kp


def rotate_image(im, rot_mat, fill: int = 0) -> np.ndarray:
    im = _img(im)
    H, W = im.shape[:2]
    m = np.ascontiguousarray(rot_mat, np.float64).reshape(9)
    out = np.full_like(im, fill)
    if not lib().erpo_rotate_image(_p(im), W, H, _p(m), _p(out)):
        raise ValueError("singular rot_mat")
    return out


def rectify(left, right, rot_vec, t_vec, fill: int = 0):
    left, right = _img(left), _img(right)
    H, W = left.shape[:2]
    rv = np.ascontiguousarray(rot_vec, np.float64)
    tv = np.ascontiguousarray(t_vec, np.float64)
    lo, ro = np.full_like(left, fill), np.full_like(right, fill)
    if not lib().erpo_rectify(_p(left), _p(right), W, H, _p(rv), _p(tv), _p(lo), _p(ro)):
        raise ValueError("singular rectification matrix")
    return lo, ro


def vertical_rotate(im, fill: int = 0) -> np.ndarray:
    im = _img(im)
    H, W = im.shape[:2]
    out = np.full((W, H, 3), fill, np.uint8)
    if not lib().erpo_vertical_rotate(_p(im), W, H, _p(out)):
        raise ValueError("singular")
    return out


def pitch_matrix(deg: float) -> np.ndarray:
    """eular2rot(Vec3f(0, RAD(deg), 0)) (src/spherical_surf.cpp:26)"""
    return eular2rot([0.0, float(np.float32(np.pi * np.float64(np.float32(deg)) / 180.0)), 0.0])


def rotate_pixel_prefix(rows, cols, m, W: int, H: int) -> np.ndarray:
    """[n, 2] values rotate_pixel truncates (row value, column value)"""
    r = np.ascontiguousarray(rows, np.int32)
    c = np.ascontiguousarray(cols, np.int32)
    m = np.ascontiguousarray(m, np.float64).reshape(9)
    out = np.zeros((len(r), 2), np.float64)
    lib().erpo_rotate_pixel_prefix(_p(r), _p(c), len(r), _p(m), W, H, _p(out))
    return out


# ------------------------------------------------------------------ SURF (section 8f-2)
def surf(img, hessian_threshold=100.0, n_octaves=4, n_octave_layers=3, max_kp=1 << 16):
    """SURF::detect + compute (OpenCV defaults restated; parity with OpenCV unpinned):
    img uint8 [H, W] or [H, W, 3] (BGR) -> (keypoints KEYPOINT_DTYPE, descriptors [n, 64])"""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    prm = SurfParams(hessian_threshold, n_octaves, n_octave_layers)
    while True:
        kps = np.zeros(max_kp, KEYPOINT_DTYPE)
        desc = np.zeros((max_kp, 64), np.float32)
        n = lib().erpo_surf(_p(img), W, H, ch, C.byref(prm), _p(kps), _p(desc), max_kp)
        if n >= 0:
            return kps[:n].copy(), desc[:n].copy()
        max_kp = -n


def gray_bgr(img):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    out = np.zeros((H, W), np.uint8)
    lib().erpo_gray_bgr(_p(img), W, H, _p(out))
    return out


# ---------------- visual outputs (erp_viz.c) ----------------
def epipolar_draw(key_left, key_right, im_width: int, im_height: int, out_w: int, out_h: int,
                  n_key: int, E, seed: int = 1, offset: int = 0):
    """epipolar_tool(...).draw_epipole(E) run sequentially (src/epipolar_tool.cpp:7-128) ->
    (canvas uint8 [out_h, out_w, 3], random_idx (n_key,), min over pixels and keys of
    ||l^T E p| - 0.002| -- how close the canvas came to the threshold)."""
    kl = np.ascontiguousarray(key_left, np.float32).reshape(-1, 2)
    kr = np.ascontiguousarray(key_right, np.float32).reshape(-1, 2)
    e = np.ascontiguousarray(E, np.float64).reshape(9)
    out = np.zeros((out_h, out_w, 3), np.uint8)
    idx = np.zeros(max(n_key, 1), np.int32)
    mm = C.c_double(0)
    rc = lib().erpo_epipolar_draw(_p(kl), _p(kr), kl.shape[0], im_width, im_height, out_w, out_h,
                                  n_key, seed, offset, _p(e), _p(out), _p(idx), C.byref(mm))
    if rc:
        raise ValueError("epipolar_draw: invalid arguments")
    return out, idx[:n_key], mm.value


def epipolar_value(l, E, i: int, j: int, out_w: int, out_h: int) -> float:
    """l^T E p of canvas pixel (i, j) (src/epipolar_tool.cpp:100-105)"""
    lv = np.ascontiguousarray(l, np.float64).reshape(3)
    e = np.ascontiguousarray(E, np.float64).reshape(9)
    return lib().erpo_epipolar_value(_p(lv), _p(e), i, j, out_w, out_h)


def hsv2bgr(h: int, s: int, v: int) -> np.ndarray:
    o = np.zeros(3, np.uint8)
    lib().erpo_hsv2bgr(h, s, v, _p(o))
    return o


def draw_match(im_left: np.ndarray, im_right: np.ndarray, key_left, key_right) -> np.ndarray:
    """feature_matcher::draw_match (src/feature_matcher.cpp:61-86) with lines = the pixels
    within 2.5 of the segment between the rounded keypoints (parity with cv::line unpinned)."""
    a = np.ascontiguousarray(im_left, np.uint8)
    b = np.ascontiguousarray(im_right, np.uint8)
    kl = np.ascontiguousarray(key_left, np.float32).reshape(-1, 2)
    kr = np.ascontiguousarray(key_right, np.float32).reshape(-1, 2)
    H, W = a.shape[:2]
    out = np.zeros_like(a)
    lib().erpo_draw_match(_p(a), _p(b), W, H, _p(kl), _p(kr), kl.shape[0], _p(out))
    return out
