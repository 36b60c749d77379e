"""MI355X-native ERP matcher + spherical eight-point estimator.

Host-side mirror of the reference's hot-path classes (Kitsunetic/ERP_match_eightpoint_test):

* ``feature_matcher.match_two_image``  -- src/feature_matcher.cpp:42-59
* ``eight_point.find / initial_guess / eight_point_estimation`` -- src/eight_point.cpp:16-192
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

__all__ = ["feature_matcher", "eight_point", "PairBatchRunner", "Context", "ErpError",
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


class PairBatchRunner:
    """The fused hot path over a batch of ERP pairs held in device memory (torch tensors).

    run(...) launches match -> gather -> find for every pair on torch's current stream and
    returns a torch uint8 tensor of erp_pair_result records (view with RESULT_DTYPE after
    .cpu()).  Optional debug outputs (matches, hyps, samples, rvec, tvec, dist) are allocated
    when requested.
    """

    def __init__(self, device: int = 0, ctx: Context | None = None, **cfg):
        self.ctx = ctx or Context(device)
        self.cfg = default_cfg(**cfg)
        self.device = self.ctx.device

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
