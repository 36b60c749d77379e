"""Multi-GPU partitioning of the hot path: one process per GPU, torch.distributed (RCCL on
the GPUs, gloo in the CPU tests).

Two partitions, each with a single collective at the end (no data-path exchange):

* pairs (configs[2]): independent ERP pairs are split into contiguous blocks per rank; each
  rank runs erp_pair_batch_run on its block; the 64-byte result records are all-gathered.
* hypothesis blocks (configs[4]): the `iters` initial_guess iterations of ONE find() are split
  into contiguous blocks [a, b) per rank.  Because the reference draws every iteration from one
  process-global glibc rand() stream (src/eight_point.hpp:57, M-1 draws per iteration), block
  [a, b) is exactly the single-process computation started at stream offset base + a*(M-1);
  the per-iteration records are all-gathered in rank order (= iteration order, so the
  R_vec_arr push order of src/eight_point.cpp:113-126 is preserved) and every rank runs the
  same consensus on the merged list.

The compute is pluggable: on GPUs it is the C ABI (`CapiShardBackend` for the device-resident
path `sharded_find`, `gpu_hypotheses` / `gpu_consensus` for the host variant); the gloo tests
plug in the oracle and run the very same collective code on CPU tensors.
"""
from __future__ import annotations

import numpy as np


def block_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """contiguous block [a, b) of n items for `rank` out of `world` (sizes differ by <= 1)."""
    return n * rank // world, n * (rank + 1) // world


def all_gather_rows(t, group=None):
    """all_gather of a tensor whose first dimension may differ per rank -> list per rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    mx = max(ns) if ns else 0
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    bufs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return [b[:k] for b, k in zip(bufs, ns)]


def valid_list(hyps: np.ndarray):
    """R_vec_arr / T_vec_arr of initial_guess: per iteration push R1 (if valid) then R2 (if
    valid), each with that iteration's T (src/eight_point.cpp:113-126)."""
    r = np.stack([hyps["R1"], hyps["R2"]], 1).reshape(-1, 3)
    t = np.stack([hyps["T"], hyps["T"]], 1).reshape(-1, 3)
    v = np.stack([hyps["R1_valid"] != 0, hyps["R2_valid"] != 0], 1).reshape(-1)
    return np.ascontiguousarray(r[v], np.float32), np.ascontiguousarray(t[v], np.float32)


def stream_offset(base: int, a: int, m: int, sampler: int = 0) -> int:
    """the erp_ransac_cfg.offset that starts iteration a of a run begun at `base`: the glibc
    replay consumes m-1 rand() draws per iteration (base + a (m-1)); the counter-based Philox
    sampler (ERP_SAMPLER_PHILOX) keys each iteration by its number (base + a)."""
    return base + a if sampler == 1 else base + a * (m - 1)


def find_hypothesis_sharded(hyp_fn, consensus_fn, m: int, iters: int, offset: int, group=None,
                            sampler: int = 0):
    """One find() with its iterations split over the ranks of `group`.

    hyp_fn(iters_local, offset_local) -> numpy structured array of per-iteration records (fields
    R1, R2, T, R1_valid, R2_valid, ...); consensus_fn(rvec, tvec) -> result.  Returns the
    result (identical on every rank) and the merged record array."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = block_range(iters, world, rank)
    local = hyp_fn(b - a, stream_offset(offset, a, m, sampler))
    raw = torch.from_numpy(np.ascontiguousarray(local).view(np.uint8).reshape(len(local), -1).copy())
    parts = all_gather_rows(raw, group)
    merged = np.concatenate([p.numpy().reshape(-1).view(local.dtype) for p in parts])
    rvec, tvec = valid_list(merged)
    return consensus_fn(rvec, tvec), merged


def padded_block(iters: int, world: int, rank: int) -> tuple[int, int, int]:
    """block size B = ceil(iters / world) and this rank's iterations [a, b) = [rank B, ..)."""
    blk = max(1, -(-iters // world))
    a = min(iters, rank * blk)
    return blk, a, min(iters, a + blk)


class CapiShardBackend:
    """the per-rank compute of the device-resident configs[4] path through the C ABI, all on
    one HIP stream `st` (hypotheses -> consensus or bounds shard -> finish)."""

    def __init__(self, ctx, W: int, H: int, d_kl, d_kr, m: int, cfg_kwargs: dict | None = None,
                 stream=None):
        import torch
        self.ctx, self.W, self.H, self.d_kl, self.d_kr, self.m = ctx, W, H, d_kl, d_kr, m
        self.cfg_kwargs = dict(cfg_kwargs or {})
        self.base = int(self.cfg_kwargs.pop("offset", 0))
        self.device = d_kl.device
        self.st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream

    def stream(self):
        """context manager: torch's current stream = the compute stream, so the collectives
        (issued on torch's current stream) are ordered after the kernels that fill their
        inputs, and the kernels after the collectives that fill theirs."""
        import contextlib

        import torch
        if self.st == torch.cuda.current_stream(self.device).cuda_stream:
            return contextlib.nullcontext()  # already torch's current stream
        return torch.cuda.stream(torch.cuda.ExternalStream(self.st, device=self.device))

    def _cfg(self, **kw):
        from .capi import default_cfg
        return default_cfg(**dict(self.cfg_kwargs, **kw))

    def hyps(self, a: int, b: int, out):
        import ctypes as C

        from .capi import check
        cfg = self._cfg(iters=b - a, offset=stream_offset(self.base, a, self.m,
                                                          self.cfg_kwargs.get("sampler", 0)))
        check(self.ctx.L.erp_eight_point_hypotheses_dev(
            self.ctx.h, self.W, self.H, self.d_kl.data_ptr(), self.d_kr.data_ptr(), self.m,
            C.byref(cfg), out.data_ptr(), self.st), "erp_eight_point_hypotheses_dev")

    def consensus(self, merged, iters: int, res):
        import ctypes as C

        from .capi import check
        cfg = self._cfg(iters=iters)
        check(self.ctx.L.erp_consensus_hyps_dev(self.ctx.h, self.m, merged.data_ptr(),
                                                merged.shape[0], C.byref(cfg), res.data_ptr(),
                                                self.st), "erp_consensus_hyps_dev")

    def shard(self, merged, iters: int, sh: int, nsh: int, part):
        import ctypes as C

        from .capi import check
        cfg = self._cfg(iters=iters)
        check(self.ctx.L.erp_consensus_hyps_shard_dev(
            self.ctx.h, self.m, merged.data_ptr(), merged.shape[0], C.byref(cfg), sh, nsh,
            part[0].data_ptr(), part[1].data_ptr(), part[2].data_ptr(), self.st),
            "erp_consensus_hyps_shard_dev")

    def finish(self, merged, iters: int, bounds, res):
        import ctypes as C

        from .capi import check
        cfg = self._cfg(iters=iters)
        check(self.ctx.L.erp_consensus_hyps_finish_dev(
            self.ctx.h, self.m, merged.data_ptr(), merged.shape[0], C.byref(cfg),
            bounds[0].data_ptr(), bounds[1].data_ptr(), bounds[2].data_ptr(), res.data_ptr(),
            self.st), "erp_consensus_hyps_finish_dev")


def sharded_find(backend, iters: int, group=None, shard_consensus: bool = True,
                 emulate_world: int = 0):
    """The collective skeleton of configs[4] (hypothesis blocks), independent of where the
    compute runs: rank r computes iterations [r B, (r+1) B) (B = ceil(iters / world)) into a
    zero-padded block of B records, the blocks are all_gather_into_tensor'ed in rank order
    (= iteration order; zero records push nothing, so R_vec_arr's order is the single-process
    one, src/eight_point.cpp:113-126), and every rank runs the valid-list compaction +
    consensus on the merged records.  With shard_consensus the K^2 bounds pass is split too:
    rank r bounds its rows, one all_reduce(SUM) over the [LB, UB] doubles and one over the
    boundary-bin words (two int32 per row, summed as int64 words: one rank writes each row,
    the others hold 0, so the sums are exact), and every rank finishes the selection.
    emulate_world > 1 (one process): run every shard locally in turn and sum them, as the
    all_reduce would.  `backend` supplies device, stream() and the compute (hyps, consensus,
    shard, finish): CapiShardBackend on GPUs, the oracle in the gloo tests.
    Returns (result record tensor [64] uint8, merged records [world B, 120] uint8)."""
    import torch
    import torch.distributed as dist

    from .capi import HYP_DTYPE, RESULT_DTYPE
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    blk, a, b = padded_block(iters, world, rank)
    dev = backend.device
    with backend.stream():
        local = torch.zeros((blk, HYP_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        if b > a:
            backend.hyps(a, b, local)
        if world > 1:
            merged = torch.empty((world * blk, HYP_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            dist.all_gather_into_tensor(merged, local, group=group)
        else:
            merged = local
        res = torch.zeros(RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        n = merged.shape[0]
        nsh = world if world > 1 else max(emulate_world, 1)
        if not shard_consensus or nsh == 1:
            backend.consensus(merged, iters, res)
            return res, merged
        bounds = torch.zeros((3, 2 * n), dtype=torch.float64, device=dev)  # lb, ub, bsel (2 x i32)
        part = torch.empty_like(bounds)
        for sh in ([rank] if world > 1 else range(nsh)):
            backend.shard(merged, iters, sh, nsh, part)
            if world > 1:
                bounds = part
            else:  # emulation: the same sums the all_reduce does
                bounds[:2] += part[:2]
                bounds[2].view(torch.int64).add_(part[2].view(torch.int64))
        if world > 1:
            dist.all_reduce(bounds[:2], group=group)
            dist.all_reduce(bounds[2].view(torch.int64), group=group)
        backend.finish(merged, iters, bounds, res)
    return res, merged


def find_hypothesis_sharded_dev(ctx, W: int, H: int, d_kl, d_kr, m: int, iters: int,
                                cfg_kwargs: dict | None = None, group=None, stream=None,
                                shard_consensus: bool = True, emulate_world: int = 0):
    """configs[4] on GPUs, device-resident end to end (sharded_find over the C ABI:
    erp_eight_point_hypotheses_dev at offset stream_offset(base, r B, m), RCCL all_gather of the
    blocks, erp_consensus_hyps_dev, or erp_consensus_hyps_shard_dev + RCCL all_reduce +
    erp_consensus_hyps_finish_dev) -- the same result as the unsharded
    erp_eight_point_find_dev.  Everything, collectives included, is ordered on `stream`.
    Returns (result record tensor [64] uint8, merged)."""
    be = CapiShardBackend(ctx, W, H, d_kl, d_kr, m, cfg_kwargs, stream)
    return sharded_find(be, iters, group, shard_consensus, emulate_world)


def gather_records(local, group=None):
    """the pair path's only collective (configs[1]/[2], the "best-model gather"): every rank's
    [B, 64] block of erp_pair_result records, concatenated in rank order with one
    all_gather_into_tensor (RCCL on the GPUs).  Equal B on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


def min_idx_agrees(got: int, want: int, r1_valid=None, r2_valid=None) -> tuple[bool, bool]:
    """(agrees, is_swap) for a consensus winner index `got` against the oracle's `want` in
    R_vec_arr order (src/eight_point.cpp:113-126: R1 then R2 per iteration).  Equal indices
    agree.  Indices one apart agree ONLY when both rows are the two rotations of one iteration
    (R1 and R2 both valid there): the R1 / R2 order follows the sign of a noise-level singular
    vector inside decomposeEssentialMat, so the push order of that iteration may
    differ while the winning rotation is the same.  r1_valid / r2_valid: the oracle's
    per-iteration validity flags (needed to map rows to iterations; without them a +-1 is a
    mismatch)."""
    got, want = int(got), int(want)
    if got == want:
        return True, False
    if abs(got - want) != 1 or r1_valid is None or r2_valid is None:
        return False, False
    v1 = np.asarray(r1_valid).astype(bool)
    v2 = np.asarray(r2_valid).astype(bool)
    # row k belongs to the iteration whose [start, start + count) covers k
    cnt = v1.astype(np.int64) + v2.astype(np.int64)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    lo = min(got, want)
    it = int(np.searchsorted(start, lo, side="right")) - 1
    same = 0 <= it < len(cnt) and cnt[it] == 2 and start[it] == lo
    return bool(same), bool(same)


def check_gathered(gathered, per_rank: int, world: int, rerun_fn, oracle_fn=None) -> dict:
    """rank 0's self-check of the pair path's gathered records (outside the timed region):
    for every rank r, the first pair of r's block is recomputed on rank 0 alone
    (rerun_fn(r) -> 64-byte record as uint8[64]) and compared byte for byte with the record
    rank r contributed (gathered[r * per_rank]); with oracle_fn(r) -> the oracle's find() of
    that pair (dict with M, K, min_idx, R, T), the gathered record is also checked against the
    CPU restatement (src/eight_point.cpp:152-192: K equal, min_idx equal by min_idx_agrees --
    given the oracle's per-iteration validity flags o["hyp"] when present -- and R / T within
    1e-6)."""
    from .capi import RESULT_DTYPE
    g = np.ascontiguousarray(np.asarray(gathered, np.uint8)).reshape(-1, RESULT_DTYPE.itemsize)
    bad_bytes, bad_oracle, swaps = [], [], []
    for r in range(world):
        rec = g[r * per_rank]
        if not np.array_equal(np.asarray(rerun_fn(r), np.uint8).reshape(-1), rec):
            bad_bytes.append(r)
        if oracle_fn is not None:
            o = oracle_fn(r)
            x = rec.view(RESULT_DTYPE)[0]
            hy = o.get("hyp")
            agree, swap = min_idx_agrees(x["min_idx"], o["min_idx"],
                                         None if hy is None else hy["R1_valid"],
                                         None if hy is None else hy["R2_valid"])
            if swap:
                swaps.append(r)
            ok = (int(x["status"]) == 0 and int(x["M"]) == int(o["M"]) and
                  int(x["K"]) == int(o["K"]) and agree and
                  float(np.abs(x["R"] - o["R"]).max()) <= 1e-6 and
                  float(np.abs(x["T"] - o["T"]).max()) <= 1e-6)
            if not ok:
                bad_oracle.append(r)
    out = {"ranks_checked": world, "records_identical": not bad_bytes,
           "mismatched_ranks": bad_bytes}
    if oracle_fn is not None:
        out["oracle_all_equal"] = not bad_oracle
        out["oracle_mismatched_ranks"] = bad_oracle
        out["r1r2_order_swaps"] = swaps
    return out


def shard_pairs(n_pairs: int, group=None) -> range:
    import torch.distributed as dist
    a, b = block_range(n_pairs, dist.get_world_size(group), dist.get_rank(group))
    return range(a, b)


# ----------------------------------------------------------------------- GPU callables
def gpu_hypotheses(ctx, W: int, H: int, d_kl, d_kr, m: int, cfg_kwargs: dict):
    """hyp_fn for find_hypothesis_sharded on a GPU (erp_eight_point_hypotheses_dev)."""
    import ctypes as C

    import torch

    from .capi import HYP_DTYPE, check, default_cfg

    def fn(iters_local: int, offset_local: int):
        cfg = default_cfg(**dict(cfg_kwargs, iters=max(iters_local, 1), offset=offset_local))
        out = torch.zeros((max(iters_local, 1), HYP_DTYPE.itemsize), dtype=torch.uint8,
                          device=d_kl.device)
        check(ctx.L.erp_eight_point_hypotheses_dev(ctx.h, W, H, d_kl.data_ptr(), d_kr.data_ptr(),
                                                   m, C.byref(cfg), out.data_ptr(),
                                                   torch.cuda.current_stream().cuda_stream),
              "erp_eight_point_hypotheses_dev")
        return out.cpu().numpy().reshape(-1).view(HYP_DTYPE)[:iters_local]
    return fn


def gpu_consensus(ctx, device, trim_lo: float = 0.2, trim_hi: float = 0.8):
    """consensus_fn for find_hypothesis_sharded on a GPU (erp_consensus_dev)."""
    import torch

    from .capi import RESULT_DTYPE, check

    def fn(rvec: np.ndarray, tvec: np.ndarray):
        K = rvec.shape[0]
        dr = torch.from_numpy(np.ascontiguousarray(rvec) if K else np.zeros((1, 3), np.float32)).to(device)
        dt = torch.from_numpy(np.ascontiguousarray(tvec) if K else np.zeros((1, 3), np.float32)).to(device)
        res = torch.zeros(RESULT_DTYPE.itemsize, dtype=torch.uint8, device=device)
        check(ctx.L.erp_consensus_dev(ctx.h, dr.data_ptr(), dt.data_ptr(), K, trim_lo, trim_hi,
                                      res.data_ptr(), torch.cuda.current_stream().cuda_stream),
              "erp_consensus_dev")
        return res.cpu().numpy().view(RESULT_DTYPE)[0]
    return fn
