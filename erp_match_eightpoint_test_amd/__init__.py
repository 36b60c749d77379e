"""MI355X-native ERP matcher + spherical eight-point estimator.

Host-side mirror of the reference's hot-path classes (Kitsunetic/ERP_match_eightpoint_test):

* ``feature_matcher.match_two_image``  -- src/feature_matcher.cpp:42-59
* ``eight_point.find / initial_guess / eight_point_estimation`` -- src/eight_point.cpp:16-192
* ``erp_rotation`` / ``spherical_surf`` -- the ERP remaps either side of the path
  (src/erp_rotation.cpp:14-122, src/spherical_surf.cpp:16-133, src/automatic.cpp:50-79,148-152)
* ``epipolar_tool`` / ``feature_matcher.draw_match`` -- the visual outputs
  (src/epipolar_tool.cpp:7-128, src/feature_matcher.cpp:61-86)
* ``PairBatchRunner`` -- the batched hot path: match -> gather -> find for many ERP pairs,
  i.e. what src/automatic.cpp:117-126 runs per pair, as one sequence of gfx950 kernels.

Every call goes through the C ABI of ``lib/liberp_match.so`` (include/erp_match.h); there is
no CPU fallback.  Arrays are numpy (host, synchronous) or torch CUDA tensors (device,
asynchronous on torch's current stream).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi, synth
from .capi import (DMATCH_DTYPE, HYP_DTYPE, RESULT_DTYPE, Context, ErpError, check,
                   default_cfg)

__all__ = ["feature_matcher", "eight_point", "erp_rotation", "spherical_surf", "epipolar_tool",
           "PairBatchRunner", "Context", "ErpError",
           "default_cfg", "DMATCH_DTYPE", "HYP_DTYPE", "RESULT_DTYPE", "results_to_numpy",
           "hyps_to_numpy", "synth", "capi"]


def _np_ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class feature_matcher:  # noqa: N801  (reference class name)
    """feature_matcher (src/feature_matcher.hpp:26-51), hot-path subset.

    match_two_image(descriptor1, descriptor2) -> structured array of DMatch
    (queryIdx, trainIdx, imgIdx, distance), ascending queryIdx, kept when d0 < 0.3 * d1.
    """

    def __init__(self, device: int = 0, ctx: Context | None = None, method: int | None = None):
        self.ctx = ctx or Context(device)
        if method is not None:  # capi.MATCHER_MFMA_FILTER (default) / capi.MATCHER_VALU_EXACT
            self.ctx.set_matcher(method)

    def match_two_image(self, descriptor1, descriptor2, ratio: float = 0.3):
        try:
            import torch
            is_torch = isinstance(descriptor1, torch.Tensor)
        except ImportError:  # pragma: no cover
            is_torch = False
        if is_torch:
            return self._match_device(descriptor1, descriptor2, ratio)
        q = np.ascontiguousarray(descriptor1, np.float32)
        t = np.ascontiguousarray(descriptor2, np.float32)
        if q.ndim != 2 or t.ndim != 2 or q.shape[1] != t.shape[1]:
            raise ValueError("descriptors must be 2-D with equal columns")
        if abs(ratio - 0.3) > 0:
            tq = self._to_device(q)
            tt = self._to_device(t)
            return self._match_device(tq, tt, ratio).cpu().numpy().view(DMATCH_DTYPE).reshape(-1)
        out = np.zeros(max(q.shape[0], 1), DMATCH_DTYPE)
        n = C.c_int32(0)
        check(self.ctx.L.erp_match_two_image(self.ctx.h, _np_ptr(q), q.shape[0], _np_ptr(t),
                                             t.shape[0], q.shape[1], _np_ptr(out), C.byref(n)),
              "match_two_image")
        return out[:n.value].copy()

    # ---- SURF (src/feature_matcher.cpp:26-40, xfeatures2d::SURF::create() defaults) ----
    def surf(self, images, max_kp: int = 16384, **params):
        """detect_key_point + comput_descriptor on CUDA uint8 images [n, H, W] (gray) or
        [n, H, W, 3] (BGR); a single [H, W] / [H, W, 3] image is one image -> (keypoints list
        of KEYPOINT_DTYPE arrays, descriptor list of [k, 64] float32), per image, in OpenCV's
        KeypointGreater order.  Parity with OpenCV is unpinned (oracle/erp_surf.c)."""
        kp, desc, counts = self.surf_dev(images, max_kp, **params)
        c = int(counts.max()) if len(counts) else 0
        kps = kp[:, :c].cpu().numpy()
        ds = desc[:, :c].cpu().numpy()
        return ([kps[i, :counts[i]].reshape(-1).view(capi.KEYPOINT_DTYPE).copy()
                 for i in range(len(counts))],
                [ds[i, :counts[i]].copy() for i in range(len(counts))])

    def surf_dev(self, images, max_kp: int = 16384, **params):
        """surf() without leaving the device -> (keypoints uint8 [n, max_kp', 28] (view as
        float32 [.., 7]: x, y, size, angle, response, octave, class_id), descriptors float32
        [n, max_kp', 64], counts numpy int32 [n]); rows [0, counts[i]) of image i are valid.
        max_kp' >= max_kp grows when an image overflows (the call is repeated)."""
        import torch
        if images.dim() == 2 or (images.dim() == 3 and images.shape[-1] == 3):
            images = images.unsqueeze(0)  # one gray [H, W] or one BGR [H, W, 3] image
        if not (images.is_cuda and images.dtype == torch.uint8 and images.is_contiguous()):
            raise ValueError("images must be contiguous CUDA uint8 tensors")
        ch = 3 if images.dim() == 4 else 1
        n, H, W = images.shape[:3]
        prm = capi.SurfParams()
        self.ctx.L.erp_surf_params_default(C.byref(prm))
        for k, v in params.items():
            setattr(prm, k, v)
        st = torch.cuda.current_stream(images.device).cuda_stream
        while True:
            kp = torch.empty((n, max_kp, 28), dtype=torch.uint8, device=images.device)
            desc = torch.empty((n, max_kp, 64), dtype=torch.float32, device=images.device)
            cnt = torch.zeros(n, dtype=torch.int32, device=images.device)
            check(self.ctx.L.erp_surf_detect_compute_dev(self.ctx.h, images.data_ptr(), n, W, H, ch,
                                                         C.byref(prm), max_kp, kp.data_ptr(),
                                                         desc.data_ptr(), cnt.data_ptr(), st),
                  "erp_surf_detect_compute_dev")
            counts = cnt.cpu().numpy()
            if (counts >= 0).all():
                return kp, desc, counts
            max_kp = int(-counts.min()) + 16

    def draw_match(self, im_left, im_right, key_left, key_right):
        """draw_match (src/feature_matcher.cpp:61-86): CUDA uint8 BGR images [H, W, 3] and the
        matched keypoints (CUDA float32 [M, 2] or anything array-like of (pt.x, pt.y)) -> the
        overlay [H, W, 3]: grey left / right in channels 0 / 1, a 5-px line per match coloured
        HSV(i 180 / M, 180, 150), later matches on top."""
        import torch
        im_left, im_right = _img_dev(im_left), _img_dev(im_right)
        if im_left.shape != im_right.shape:
            raise ValueError("draw_match: the two images differ in size")
        if im_left.device != im_right.device or im_left.device.index != self.ctx.device:
            raise ValueError(f"draw_match: images must be on the context's device "
                             f"cuda:{self.ctx.device}")
        H, W = im_left.shape[:2]
        kl, kr = _keys_dev(key_left, im_left.device), _keys_dev(key_right, im_left.device)
        m = min(kl.shape[0], kr.shape[0])
        if kl.shape[0] != kr.shape[0]:
            raise ValueError("draw_match: key_left and key_right differ in length")
        out = torch.empty_like(im_left)
        check(self.ctx.L.erp_draw_match_dev(self.ctx.h, im_left.data_ptr(), im_right.data_ptr(),
                                            W, H, kl.data_ptr() if m else None,
                                            kr.data_ptr() if m else None, m, out.data_ptr(),
                                            torch.cuda.current_stream(im_left.device).cuda_stream),
              "draw_match")
        return out

    def _to_device(self, a):
        import torch
        return torch.from_numpy(a).to(f"cuda:{self.ctx.device}")

    def _match_device(self, q, t, ratio):
        """device path: torch float32 CUDA tensors -> torch int32 tensor [M, 4] (DMatch rows)."""
        import torch
        q = q.contiguous()
        t = t.contiguous()
        assert q.dtype == torch.float32 and t.dtype == torch.float32 and q.is_cuda and t.is_cuda
        out = torch.empty((max(q.shape[0], 1), 4), dtype=torch.int32, device=q.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=q.device)
        st = torch.cuda.current_stream(q.device).cuda_stream
        check(self.ctx.L.erp_match_knn2_ratio(self.ctx.h, q.data_ptr(), q.shape[0], t.data_ptr(),
                                              t.shape[0], q.shape[1], ratio, out.data_ptr(),
                                              cnt.data_ptr(), st), "match_knn2_ratio")
        return out[: int(cnt.item())]


class eight_point:  # noqa: N801  (reference class name)
    """eight_point (src/eight_point.hpp:8-28).  ``cfg`` holds the reference constants."""

    def __init__(self, device: int = 0, ctx: Context | None = None, **cfg):
        self.ctx = ctx or Context(device)
        self.cfg = default_cfg(**cfg)
        self.last_result = None

    def find(self, im_width: int, im_height: int, key_left, key_right, match_size: int | None = None):
        """-> (R_vec_out (3,) float32, T_vec_out (3,) float32); raises ErpError on the
        reference's undefined-behaviour cases (too few points, no valid hypothesis)."""
        kl = np.ascontiguousarray(key_left, np.float32).reshape(-1, 2)
        kr = np.ascontiguousarray(key_right, np.float32).reshape(-1, 2)
        m = kl.shape[0] if match_size is None else int(match_size)
        if m > kl.shape[0] or m > kr.shape[0]:
            raise ValueError("match_size larger than the keypoint arrays")
        kl = np.ascontiguousarray(kl[:m])
        kr = np.ascontiguousarray(kr[:m])
        R = np.zeros(3, np.float32)
        T = np.zeros(3, np.float32)
        res = capi.PairResult()
        st = self.ctx.L.erp_eight_point_find(self.ctx.h, im_width, im_height, _np_ptr(kl),
                                             _np_ptr(kr), m, C.byref(self.cfg), _np_ptr(R),
                                             _np_ptr(T), C.byref(res))
        self.last_result = np.frombuffer(bytes(res), RESULT_DTYPE)[0]
        check(st, "find")
        return R, T

    def initial_guess(self, im_width: int, im_height: int, key_point_left_rect,
                      key_point_right_rect, match_size: int | None = None):
        bl = np.ascontiguousarray(key_point_left_rect, np.float64).reshape(-1, 3)
        br = np.ascontiguousarray(key_point_right_rect, np.float64).reshape(-1, 3)
        m = bl.shape[0] if match_size is None else int(match_size)
        R = np.zeros(3, np.float32)
        T = np.zeros(3, np.float32)
        res = capi.PairResult()
        st = self.ctx.L.erp_initial_guess(self.ctx.h, _np_ptr(bl), _np_ptr(br), m,
                                          C.byref(self.cfg), _np_ptr(R), _np_ptr(T), C.byref(res))
        self.last_result = np.frombuffer(bytes(res), RESULT_DTYPE)[0]
        check(st, "initial_guess")
        return R, T

    def eight_point_estimation(self, im_width: int, im_height: int, key_point_left_rect,
                               key_point_right_rect, match_size: int | None = None):
        """-> (R1_vec, R2_vec, T_vec, R1_valid, R2_valid, E)"""
        bl = np.ascontiguousarray(key_point_left_rect, np.float64).reshape(-1, 3)
        br = np.ascontiguousarray(key_point_right_rect, np.float64).reshape(-1, 3)
        m = bl.shape[0] if match_size is None else int(match_size)
        h = capi.Hypothesis()
        check(self.ctx.L.erp_eight_point_estimation(self.ctx.h, _np_ptr(bl), _np_ptr(br), m,
                                                    C.byref(h)), "eight_point_estimation")
        r = np.frombuffer(bytes(h), HYP_DTYPE)[0]
        return (r["R1"].copy(), r["R2"].copy(), r["T"].copy(), bool(r["R1_valid"]),
                bool(r["R2_valid"]), r["E"].copy())


def _keys_dev(k, device):
    """(pt.x, pt.y) rows as a contiguous CUDA float32 tensor [n, 2]"""
    import torch
    if isinstance(k, torch.Tensor):
        t = k.to(device=device, dtype=torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(k, np.float32)).to(device)
    return t.reshape(-1, 2).contiguous()


def _keys_host(k) -> np.ndarray:
    try:
        import torch
        if isinstance(k, torch.Tensor):
            k = k.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.ascontiguousarray(k, np.float32).reshape(-1, 2)


class epipolar_tool:  # noqa: N801  (reference class name)
    """epipolar_tool (src/epipolar_tool.hpp:7-31, .cpp:7-128): picks test_key_num (<= 7) of the
    matched pairs with std::random_shuffle on the glibc rand() stream -- (seed, offset) = the
    process-global rand() state, (1, 0) in a fresh process -- and draws, for an essential
    matrix, the epipolar curves of their left keypoints and dots at their right keypoints on an
    output_width x output_height ERP canvas (a CUDA uint8 tensor [H, W, 3])."""

    def __init__(self, left_key, right_key, im_width: int, im_height: int, output_width: int,
                 output_height: int, test_key_num: int, seed: int = 1, offset: int = 0,
                 device: int = 0, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self.left_key, self.right_key = _keys_host(left_key), _keys_host(right_key)
        if self.left_key.shape != self.right_key.shape:
            raise ValueError("epipolar_tool: left_key and right_key differ in length")
        self.match_size = self.left_key.shape[0]
        self.n_key = int(test_key_num)
        self.im_width, self.im_height = int(im_width), int(im_height)
        self.epipole_mat_width, self.epipole_mat_height = int(output_width), int(output_height)
        self.seed, self.offset = int(seed), int(offset)
        if not (1 <= self.match_size and 0 <= self.n_key <= min(7, self.match_size)):
            raise ErpError(capi.ERP_INVALID_ARG,
                           "epipolar_tool: need 0 <= test_key_num <= min(7, match_size)")
        # the constructor's choice (src/epipolar_tool.cpp:13-16), available before any draw
        self.random_idx = np.zeros(self.n_key, np.int32)
        check(self.ctx.L.erp_random_shuffle_prefix(self.seed, self.offset, self.match_size,
                                                   self.n_key, _np_ptr(self.random_idx)),
              "random_shuffle_prefix")

    def draw_epipole(self, test_E_mat):  # noqa: N803  (reference argument name)
        import torch
        E = _m9(test_E_mat)
        dev = torch.device(f"cuda:{self.ctx.device}")
        out = torch.empty((self.epipole_mat_height, self.epipole_mat_width, 3), dtype=torch.uint8,
                          device=dev)
        check(self.ctx.L.erp_epipolar_draw_dev(
            self.ctx.h, _np_ptr(self.left_key), _np_ptr(self.right_key), self.match_size,
            self.im_width, self.im_height, self.epipole_mat_width, self.epipole_mat_height,
            self.n_key, self.seed, self.offset, _np_ptr(E), out.data_ptr(),
            _np_ptr(self.random_idx), torch.cuda.current_stream(dev).cuda_stream), "draw_epipole")
        return out


def _m9(a) -> np.ndarray:
    return np.ascontiguousarray(a, np.float64).reshape(9)


def _img_dev(im):
    import torch
    if not (isinstance(im, torch.Tensor) and im.is_cuda and im.dtype == torch.uint8
            and im.dim() == 3 and im.shape[2] == 3 and im.is_contiguous()):
        raise ValueError("images are contiguous CUDA uint8 tensors [H, W, 3] (CV_8UC3)")
    return im


class erp_rotation:  # noqa: N801  (reference class name)
    """erp_rotation (src/erp_rotation.hpp:9-19).  Matrices are host numpy (3, 3) float64;
    images are CUDA uint8 tensors [H, W, 3].  Output pixels whose source falls outside the
    image are not written (uninitialised in the reference): ``fill`` pre-fills them."""

    def __init__(self, device: int = 0, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self.L = self.ctx.L

    def eular2rot(self, theta) -> np.ndarray:
        th = np.ascontiguousarray(theta, np.float64).reshape(3)
        R = np.zeros(9, np.float64)
        self.L.erp_eular2rot(_np_ptr(th), _np_ptr(R))
        return R.reshape(3, 3)

    def rot2eular(self, R) -> np.ndarray:
        m = _m9(R)
        e = np.zeros(3, np.float64)
        self.L.erp_rot2eular(_np_ptr(m), _np_ptr(e))
        return e

    def rotate_image(self, im, rot_mat, fill: int = 0):
        import torch
        im = _img_dev(im)
        H, W = im.shape[:2]
        out = torch.full_like(im, fill)
        m = _m9(rot_mat)
        check(self.L.erp_rotate_image_dev(self.ctx.h, im.data_ptr(), W, H, _np_ptr(m),
                                          out.data_ptr(), torch.cuda.current_stream().cuda_stream),
              "rotate_image")
        return out

    def rot_from_vec(self, v1, v2) -> np.ndarray:
        a = np.ascontiguousarray(v1, np.float64).reshape(3)
        b = np.ascontiguousarray(v2, np.float64).reshape(3)
        R = np.zeros(9, np.float64)
        self.L.erp_rot_from_vec(_np_ptr(a), _np_ptr(b), _np_ptr(R))
        return R.reshape(3, 3)

    def inv(self, m) -> np.ndarray:
        """cv::Mat::inv() of a 3x3 double matrix"""
        a = _m9(m)
        o = np.zeros(9, np.float64)
        if not self.L.erp_inv3(_np_ptr(a), _np_ptr(o)):
            raise ErpError(capi.ERP_INVALID_ARG, "inv: singular")
        return o.reshape(3, 3)

    def rectify(self, im_left, im_right, rot_vec, t_vec, fill: int = 0):
        """rectify (src/automatic.cpp:66-79) -> (left_rectified, right_rectified)"""
        import torch
        im_left, im_right = _img_dev(im_left), _img_dev(im_right)
        H, W = im_left.shape[:2]
        lo, ro = torch.full_like(im_left, fill), torch.full_like(im_right, fill)
        rv = np.ascontiguousarray(rot_vec, np.float64).reshape(3)
        tv = np.ascontiguousarray(t_vec, np.float64).reshape(3)
        check(self.L.erp_rectify_dev(self.ctx.h, im_left.data_ptr(), im_right.data_ptr(), W, H,
                                     _np_ptr(rv), _np_ptr(tv), lo.data_ptr(), ro.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream), "rectify")
        return lo, ro

    def vertical_rotate(self, im, fill: int = 0):
        """src/automatic.cpp:148-151: rotate_image by eular2rot(RAD(89.999),0,0).inv(), then
        cv::rotate(ROTATE_90_CLOCKWISE) -> [W, H, 3]"""
        import torch
        im = _img_dev(im)
        H, W = im.shape[:2]
        out = torch.full((W, H, 3), fill, dtype=torch.uint8, device=im.device)
        check(self.L.erp_vertical_rotate_dev(self.ctx.h, im.data_ptr(), W, H, out.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream),
              "vertical_rotate")
        return out


class spherical_surf:  # noqa: N801  (reference class name)
    """spherical_surf (src/spherical_surf.hpp:11-29): the four de-distorted bands of an ERP
    image, SURF on every band, the keypoint un-rotation back to ERP pixels, the band
    concatenation, the match and the gather of the matched keypoints (do_all)."""

    PITCH = (45.0, 0.0, -45.0, -90.0)  # bands n0..n3 (src/spherical_surf.cpp:77-83)

    def __init__(self, device: int = 0, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self.L = self.ctx.L

    def crop_rotated_image(self, pitch_rot: float, im, fill: int = 0):
        import torch
        im = _img_dev(im)
        H, W = im.shape[:2]
        out = torch.full((H // 4, W, 3), fill, dtype=torch.uint8, device=im.device)
        check(self.L.erp_crop_rotated_image_dev(self.ctx.h, im.data_ptr(), W, H, pitch_rot,
                                                out.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream),
              "crop_rotated_image")
        return out

    def bands(self, ims, fill: int = 0):
        """ims: CUDA uint8 [n, H, W, 3] (or [H, W, 3]) -> [n, 4, H/4, W, 3]"""
        import torch
        single = ims.dim() == 3
        if single:
            ims = ims.unsqueeze(0)
        if not (ims.is_cuda and ims.dtype == torch.uint8 and ims.is_contiguous()
                and ims.dim() == 4 and ims.shape[3] == 3):
            raise ValueError("images are contiguous CUDA uint8 tensors [n, H, W, 3]")
        n, H, W = ims.shape[:3]
        out = torch.full((n, 4, H // 4, W, 3), fill, dtype=torch.uint8, device=ims.device)
        check(self.L.erp_spherical_bands_dev(self.ctx.h, ims.data_ptr(), n, W, H, out.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream), "bands")
        return out[0] if single else out

    def rotate_keypoint(self, pitch_rot_inv: float, key, width: int, height: int):
        """in place on a CUDA float32 tensor [n, 2] of (pt.x, pt.y)"""
        import torch
        check(self.L.erp_rotate_keypoints_dev(self.ctx.h, key.data_ptr(), key.shape[0],
                                              pitch_rot_inv, width, height,
                                              torch.cuda.current_stream().cuda_stream),
              "rotate_keypoint")
        return key

    def do_all(self, im_left, im_right, max_kp: int = 16384, fill: int = 0, draw: bool = False):
        """spherical_surf::do_all (src/spherical_surf.cpp:65-180) on two CUDA uint8 BGR ERP
        images [H, W, 3]: bands (:77-93) -> SURF on the 8 bands (:96-118) -> keypoint
        un-rotation + concatenation n0..n3 (:120-150) -> match_two_image (:153) -> gather
        (:155-162).  Returns (left_key [M, 2], right_key [M, 2]) CUDA float32 tensors of the
        matched ERP pixels, match_size and total_key_num (the left keypoints, :179); with
        draw=True also match_output (feature_matcher.draw_match of the two images, :173)."""
        import torch
        H, W = im_left.shape[:2]
        ims = torch.stack([_img_dev(im_left), _img_dev(im_right)]).contiguous()
        bands = self.bands(ims, fill=fill)                      # [2, 4, H/4, W, 3]
        fm = feature_matcher(ctx=self.ctx)
        kp, desc, counts = fm.surf_dev(bands.reshape(8, H // 4, W, 3), max_kp=max_kp)
        kxy = kp.view(torch.float32)[..., :2]                   # pt.x, pt.y of every row
        keys, dcat = [], []
        for side in range(2):
            c4 = [int(c) for c in counts[4 * side: 4 * side + 4]]
            key = torch.cat([kxy[4 * side + b, :c4[b]] for b in range(4)]).contiguous()
            if key.shape[0]:
                self.unrotate_band_keypoints(key, c4, W, H)
            keys.append(key)
            dcat.append(torch.cat([desc[4 * side + b, :c4[b]] for b in range(4)]).contiguous())
        m = fm._match_device(dcat[0], dcat[1], 0.3)            # [M, 4] int32 DMatch rows
        q, t = m[:, 0].long(), m[:, 1].long()
        kl, kr = keys[0][q], keys[1][t]
        if draw:
            return (kl, kr, int(m.shape[0]), int(keys[0].shape[0]),
                    fm.draw_match(im_left, im_right, kl, kr))
        return kl, kr, int(m.shape[0]), int(keys[0].shape[0])

    def unrotate_band_keypoints(self, key, counts, width: int, height: int):
        """do_all's keypoint step (src/spherical_surf.cpp:120-144), in place on the band
        keypoints concatenated n0, n1, n2, n3 (CUDA float32 [n, 2]); counts = 4 band sizes"""
        import torch
        c = np.ascontiguousarray(counts, np.int32).reshape(4)
        if int(c.sum()) != key.shape[0]:
            raise ValueError("counts do not sum to the keypoint count")
        check(self.L.erp_unrotate_band_keypoints_dev(self.ctx.h, key.data_ptr(), _np_ptr(c),
                                                     width, height,
                                                     torch.cuda.current_stream().cuda_stream),
              "unrotate_band_keypoints")
        return key


class PairBatchRunner:
    """The fused hot path over a batch of ERP pairs held in device memory (torch tensors).

    run(...) launches match -> gather -> find for every pair on torch's current stream and
    returns a torch uint8 tensor of erp_pair_result records (view with RESULT_DTYPE after
    .cpu()).  Optional debug outputs (matches, hyps, samples, rvec, tvec, dist) are allocated
    when requested.
    """

    def __init__(self, device: int = 0, ctx: Context | None = None, reuse_outputs: bool = False,
                 **cfg):
        """reuse_outputs: run() hands back the SAME output tensors for the same shape (copy them
        before the next call) -- what a HIP-graph replay (Context.set_graphs) needs, since the
        captured graph bakes the output pointers in"""
        self.ctx = ctx or Context(device)
        self.cfg = default_cfg(**cfg)
        self.device = self.ctx.device
        self.reuse_outputs = reuse_outputs
        self._outs = {}

    def reserve(self, n_pairs: int, max_nq: int, max_nt: int):
        check(self.ctx.L.erp_ctx_reserve(self.ctx.h, n_pairs, max_nq, max_nt, self.cfg.iters),
              "erp_ctx_reserve")

    def run(self, desc_l, desc_r, kp_l, kp_r, off_l, off_r, width, height, max_nq: int,
            max_nt: int, ratio: float = 0.3, want=(), stream=None):
        import torch
        n_pairs = off_l.shape[0] - 1
        dev = desc_l.device
        for t, dt in ((desc_l, torch.float32), (desc_r, torch.float32), (kp_l, torch.float32),
                      (kp_r, torch.float32), (off_l, torch.int64), (off_r, torch.int64),
                      (width, torch.int32), (height, torch.int32)):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise ValueError("batch tensors must be contiguous CUDA tensors of the C types")
        b = capi.PairBatch(n_pairs, desc_l.shape[1], max_nq, max_nt, desc_l.data_ptr(),
                           desc_r.data_ptr(), kp_l.data_ptr(), kp_r.data_ptr(), off_l.data_ptr(),
                           off_r.data_ptr(), width.data_ptr(), height.data_ptr())
        key = (n_pairs, max_nq, tuple(want), str(dev), self.cfg.iters)
        if self.reuse_outputs and key in self._outs:
            outs = self._outs[key]
            return self._launch(b, ratio, outs, stream, dev)
        outs = {"results": torch.empty((n_pairs, RESULT_DTYPE.itemsize), dtype=torch.uint8,
                                       device=dev)}
        iters = self.cfg.iters
        s_max = max(int(max_nq * self.cfg.sample_frac), 1)
        shapes = {"matches": (n_pairs, max_nq, 4, torch.int32),
                  "key_left": (n_pairs, max_nq, 2, torch.float32),
                  "key_right": (n_pairs, max_nq, 2, torch.float32),
                  "hyps": (n_pairs, iters, HYP_DTYPE.itemsize, torch.uint8),
                  "samples": (n_pairs, iters, s_max, torch.int32),
                  "rvec": (n_pairs, 2 * iters, 3, torch.float32),
                  "tvec": (n_pairs, 2 * iters, 3, torch.float32),
                  "dist": (n_pairs, 2 * iters, torch.float64)}
        for name in want:
            *shape, dt = shapes[name]
            outs[name] = torch.zeros(shape, dtype=dt, device=dev)
        if self.reuse_outputs:
            self._outs[key] = outs
        return self._launch(b, ratio, outs, stream, dev)

    def _launch(self, b, ratio, outs, stream, dev):
        import torch
        o = capi.BatchOutputs(*[outs[k].data_ptr() if k in outs else None
                                for k in ("results", "matches", "key_left", "key_right", "hyps",
                                          "samples", "rvec", "tvec", "dist")])
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        check(self.ctx.L.erp_pair_batch_run(self.ctx.h, C.byref(b), ratio, C.byref(self.cfg),
                                            C.byref(o), st), "erp_pair_batch_run")
        return outs


def results_to_numpy(t) -> np.ndarray:
    return t.cpu().numpy().view(RESULT_DTYPE).reshape(-1)


def hyps_to_numpy(t) -> np.ndarray:
    a = t.cpu().numpy()
    return a.reshape(a.shape[0], -1).view(HYP_DTYPE)
