"""Multi-process partition logic on CPU (gloo, world_size 2 and 3): hypothesis-block sharding
(configs[4]) and pair sharding (configs[2]) reproduce the single-process result exactly.  The
per-shard compute is the oracle here; on GPUs the same functions take the C-ABI callables."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from erp_match_eightpoint_test_amd import dist as D
from erp_match_eightpoint_test_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _hyp_worker(rank, world, port, q):
    import oracle as O
    dist = _init(rank, world, port)
    c = synth.make_correspondences(31, m=100, outlier_frac=0.6)
    bl = O.pixel_to_bearing(c["W"], c["H"], c["kp_l"])
    br = O.pixel_to_bearing(c["W"], c["H"], c["kp_r"])

    def hyp_fn(iters_local, offset_local):
        r = O.initial_guess(bl, br, O.make_cfg(iters=iters_local, offset=offset_local), detail=True)
        return r["hyp"]

    def cons_fn(rvec, tvec):
        rc, mi, d = O.consensus(rvec)
        return mi, rvec[mi], tvec[mi], len(rvec)

    res, merged = D.find_hypothesis_sharded(hyp_fn, cons_fn, 100, 300, 0)
    if rank == 0:
        q.put((res[0], res[1].tolist(), res[2].tolist(), res[3]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hypothesis_block_sharding_gloo(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hyp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    c = synth.make_correspondences(31, m=100, outlier_frac=0.6)
    ref = oracle.find(c["W"], c["H"], c["kp_l"], c["kp_r"], oracle.make_cfg(iters=300))
    mi, R, T, K = got
    assert K == ref["K"] and mi == ref["min_idx"]
    assert np.array_equal(np.float32(R), ref["R"]) and np.array_equal(np.float32(T), ref["T"])


def _pair_worker(rank, world, port, q):
    import torch

    import oracle as O
    dist = _init(rank, world, port)
    n_pairs = 5
    out = []
    for i in D.shard_pairs(n_pairs):
        p = synth.make_pair(500 + i, n_kpts=256)
        mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"])
        r = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                   O.make_cfg(iters=40))
        out.append(np.concatenate([[i, len(mt)], r["R"], r["T"]]).astype(np.float64))
    t = torch.from_numpy(np.array(out).reshape(-1, 8))
    parts = D.all_gather_rows(t)
    if rank == 0:
        q.put(torch.cat(parts).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_pair_sharding_gloo(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pair_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [int(x) for x in got[:, 0]] == list(range(5))  # rank order = pair order
    for row in got:
        p = synth.make_pair(500 + int(row[0]), n_kpts=256)
        mt, _, _, _ = oracle.match_two_image(p["desc_l"], p["desc_r"])
        r = oracle.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                        oracle.make_cfg(iters=40))
        assert int(row[1]) == len(mt)
        assert np.array_equal(np.float32(row[2:5]), r["R"]) and np.array_equal(np.float32(row[5:8]), r["T"])


def test_block_range_partition():
    for n in (0, 1, 7, 100, 10001):
        for w in (1, 2, 3, 8):
            blocks = [D.block_range(n, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1


# ------------------------------------------------------------------------------------------
# The device-resident configs[4] path (dist.sharded_find) and the pair path's record gather
# (dist.gather_records): the SAME collective code the GPU ranks run over RCCL, here over gloo
# on CPU tensors with the oracle as the per-rank compute.
class _OracleShardBackend:
    """dist.sharded_find's compute on CPU: hypotheses from the oracle's initial_guess at the
    block's glibc offset, written as 120-byte erp_hypothesis records; the bounds shard gives
    its rows [K sh / nsh, K (sh+1) / nsh) of the valid list LB = UB = the oracle's exact trimmed
    mean and a distinctive int32 pair as the boundary-bin words (so the int64-word all_reduce
    must carry them exactly); finish checks those words and takes the first argmin."""

    def __init__(self, bl, br, m):
        import torch
        self.bl, self.br, self.m = bl, br, m
        self.device = torch.device("cpu")

    def stream(self):
        import contextlib
        return contextlib.nullcontext()

    def hyps(self, a, b, out):
        import torch

        import oracle as O
        r = O.initial_guess(self.bl, self.br, O.make_cfg(iters=b - a, offset=a * (self.m - 1)),
                            detail=True)
        from erp_match_eightpoint_test_amd.capi import HYP_DTYPE
        rec = np.zeros(b - a, HYP_DTYPE)  # the oracle's record also carries E_corr
        for f in HYP_DTYPE.names:
            rec[f] = r["hyp"][f]
        out[: b - a] = torch.from_numpy(rec.view(np.uint8).reshape(b - a, -1).copy())

    def _valid(self, merged):
        from erp_match_eightpoint_test_amd.capi import HYP_DTYPE
        h = merged.numpy().reshape(-1).view(HYP_DTYPE)
        return D.valid_list(h)

    def _result(self, res, rvec, tvec, mi, K, d):
        import torch

        from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
        rec = np.zeros(1, RESULT_DTYPE)
        rec["R"], rec["T"], rec["K"], rec["min_idx"] = rvec[mi], tvec[mi], K, mi
        rec["min_dist"] = d
        res[:] = torch.from_numpy(rec.view(np.uint8).copy())

    def consensus(self, merged, iters, res):
        import oracle as O
        rvec, tvec = self._valid(merged)
        rc, mi, dist = O.consensus(rvec)
        self._result(res, rvec, tvec, mi, len(rvec), dist[mi])

    def shard(self, merged, iters, sh, nsh, part):
        import oracle as O
        rvec, _ = self._valid(merged)
        K = len(rvec)
        _, _, dist = O.consensus(rvec)
        a, b = K * sh // nsh, K * (sh + 1) // nsh
        part.zero_()
        part[0, a:b] = part.new_tensor(dist[a:b])
        part[1, a:b] = part.new_tensor(dist[a:b])
        import torch
        w = part[2].view(torch.int32)
        rows = np.arange(a, b)
        w[2 * a:2 * b:2] = w.new_tensor(rows + 1)
        w[2 * a + 1:2 * b:2] = w.new_tensor(-(rows + 1))

    def finish(self, merged, iters, bounds, res):
        import torch
        rvec, tvec = self._valid(merged)
        K = len(rvec)
        w = bounds[2].view(torch.int32).numpy()
        assert np.array_equal(w[0:2 * K:2], np.arange(1, K + 1))
        assert np.array_equal(w[1:2 * K:2], -np.arange(1, K + 1))
        assert not w[2 * K:].any()
        ub = bounds[1].numpy()[:K]
        assert np.array_equal(bounds[0].numpy()[:K], ub)
        mi = int(np.argmin(ub))  # std::min_element: the first minimum
        self._result(res, rvec, tvec, mi, K, ub[mi])


def _sharded_find_worker(rank, world, port, iters, shard_consensus, q):
    import oracle as O
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    dist = _init(rank, world, port)
    c = synth.make_correspondences(37, m=100, outlier_frac=0.6)
    bl = O.pixel_to_bearing(c["W"], c["H"], c["kp_l"])
    br = O.pixel_to_bearing(c["W"], c["H"], c["kp_r"])
    res, merged = D.sharded_find(_OracleShardBackend(bl, br, 100), iters,
                                 shard_consensus=shard_consensus)
    r = res.numpy().view(RESULT_DTYPE)[0]
    blk = D.padded_block(iters, world, rank)[0]
    q.put((rank, int(r["K"]), int(r["min_idx"]), r["R"].tolist(), r["T"].tolist(),
           merged.shape[0] == world * blk))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,iters,shard", [(2, 301, True), (2, 300, False), (3, 250, True)])
def test_sharded_find_collectives_gloo(oracle, world, iters, shard):
    """padded blocks (iters not divisible by world: zero records in the last block) gathered
    with all_gather_into_tensor, the consensus bounds all_reduce'd as doubles + int64 words:
    every rank ends with the single-process find()'s K, min_idx, R and T."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_find_worker, args=(r, world, port, iters, shard, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    c = synth.make_correspondences(37, m=100, outlier_frac=0.6)
    ref = oracle.find(c["W"], c["H"], c["kp_l"], c["kp_r"], oracle.make_cfg(iters=iters))
    assert ref["K"] > 0
    for rank, K, mi, R, T, shape_ok in got:
        assert shape_ok
        assert K == ref["K"] and mi == ref["min_idx"], (rank, K, mi, ref["K"], ref["min_idx"])
        assert np.array_equal(np.float32(R), ref["R"]) and np.array_equal(np.float32(T), ref["T"])


def _gather_worker(rank, world, port, q):
    import torch

    import oracle as O
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    dist = _init(rank, world, port)
    B = 3
    rec = np.zeros(B, RESULT_DTYPE)
    for j in range(B):
        i = rank * B + j
        p = synth.make_pair(700 + i, n_kpts=192)
        mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"])
        r = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                   O.make_cfg(iters=30))
        rec[j]["R"], rec[j]["T"], rec[j]["M"], rec[j]["K"] = r["R"], r["T"], len(mt), r["K"]
        rec[j]["min_idx"] = r["min_idx"]
    local = torch.from_numpy(rec.view(np.uint8).reshape(B, 64).copy())
    g = D.gather_records(local)
    if rank == 0:
        # the bench's rank-0 self-check of the gathered records (first pair of every rank's
        # block recomputed on rank 0, byte for byte, and against the oracle)
        def rerun(r):
            return local.numpy()[0] if r == 0 else _oracle_record(O, 700 + r * B)

        def ora(r):
            p = synth.make_pair(700 + r * B, n_kpts=192)
            mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"])
            o = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                       O.make_cfg(iters=30))
            return dict(o, M=len(mt))
        chk = D.check_gathered(g.numpy(), B, world, rerun, ora)
        # a corrupted record of rank 1 must be caught
        bad = g.numpy().copy()
        bad[B, 40] ^= 1
        chk_bad = D.check_gathered(bad, B, world, rerun, None)
        q.put((g.numpy().copy(), chk, chk_bad))
    dist.barrier()
    dist.destroy_process_group()


def _oracle_record(O, seed):
    """the 64-byte record _gather_worker builds for pair `seed`"""
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    rec = np.zeros(1, RESULT_DTYPE)
    p = synth.make_pair(seed, n_kpts=192)
    mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"])
    r = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
               O.make_cfg(iters=30))
    rec[0]["R"], rec[0]["T"], rec[0]["M"], rec[0]["K"] = r["R"], r["T"], len(mt), r["K"]
    rec[0]["min_idx"] = r["min_idx"]
    return rec.view(np.uint8).reshape(64)


def test_gather_records_gloo(oracle):
    """the bench's per-step best-model gather: rank-ordered 64-byte records, every pair's
    record equal to a single-process oracle run of that pair."""
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, chk, chk_bad = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert chk["records_identical"] and chk["oracle_all_equal"] and chk["ranks_checked"] == 2
    assert not chk_bad["records_identical"] and chk_bad["mismatched_ranks"] == [1]
    recs = got.reshape(-1).view(RESULT_DTYPE)
    assert len(recs) == 6
    for i, r in enumerate(recs):
        p = synth.make_pair(700 + i, n_kpts=192)
        mt, _, _, _ = oracle.match_two_image(p["desc_l"], p["desc_r"])
        o = oracle.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                        oracle.make_cfg(iters=30))
        assert int(r["M"]) == len(mt) and int(r["K"]) == o["K"] and int(r["min_idx"]) == o["min_idx"]
        assert np.array_equal(r["R"], o["R"]) and np.array_equal(r["T"], o["T"])


def test_min_idx_agrees_rule():
    """the parity checks' consensus-index rule (bench.parity_check and dist.check_gathered):
    equal indices agree; indices one apart agree only when they are the R1 / R2 rows of ONE
    iteration (R1 then R2 pushed per iteration, src/eight_point.cpp:113-126); anything else,
    or a +-1 without the validity flags, is a mismatch"""
    from erp_match_eightpoint_test_amd.dist import min_idx_agrees
    r1 = np.array([1, 0, 1, 1, 0, 1])
    r2 = np.array([1, 1, 0, 1, 0, 1])
    # rows: it0 -> 0, 1; it1 -> 2; it2 -> 3; it3 -> 4, 5; it4 -> none; it5 -> 6, 7
    assert min_idx_agrees(3, 3, r1, r2) == (True, False)
    assert min_idx_agrees(0, 1, r1, r2) == (True, True)
    assert min_idx_agrees(5, 4, r1, r2) == (True, True)
    assert min_idx_agrees(7, 6, r1, r2) == (True, True)
    assert min_idx_agrees(1, 2, r1, r2) == (False, False)   # different iterations
    assert min_idx_agrees(2, 3, r1, r2) == (False, False)
    assert min_idx_agrees(5, 6, r1, r2) == (False, False)
    assert min_idx_agrees(0, 2, r1, r2) == (False, False)   # two apart
    assert min_idx_agrees(0, 1) == (False, False)           # no flags: strict
