"""The bench's shipped execution shape on the GPU: the sub-batches of one step, each on its own
context and HIP stream, enqueued at once (bench.py call()).  Compared byte for byte with the
same sub-batches run one after the other, and against the oracle on one pair of every
sub-batch (src/eight_point.cpp:129-149 is a deterministic sort + accumulate + min_element, so
the answer must not depend on which kernels share the CUs).

Round 4 shipped a library whose overlapped records differed from the serial ones: binned_rows
on ~10 % of the pairs and, at ~2e-4 per pair, min_idx / R / T.  The cause was packed-FP32
results corrupted while other streams' int8 MFMA Gram kernels ran on the same CUs (DESIGN.md
5d).  These tests pin the fix."""
from __future__ import annotations

import os

import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu

S, PER, ITERS, KPTS = 6, 48, 10000, 4096


@pytest.fixture(scope="module")
def overlap_setup():
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner
    pairs = bench.make_batch(0, S * PER, KPTS, 20200423)
    subs = []
    for i in range(S):
        b = bench.to_device(pairs[i * PER:(i + 1) * PER], "cuda")
        subs.append(dict(b=b, run=PairBatchRunner(ctx=Context(0), iters=ITERS),
                         st=torch.cuda.Stream()))
    return pairs, subs


def _run(sb, want=()):
    import torch
    b = sb["b"]
    with torch.cuda.stream(sb["st"]):
        o = sb["run"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"],
                          b["width"], b["height"], b["max_nq"], b["max_nt"], want=want,
                          stream=sb["st"].cuda_stream)
    return o


def _overlapped(subs):
    import torch
    outs = [_run(sb)["results"] for sb in subs]  # every sub-batch enqueued before any finishes
    torch.cuda.synchronize()
    return np.concatenate([o.cpu().numpy() for o in outs])


def _serial(subs, want=()):
    import torch
    outs = []
    for sb in subs:
        outs.append(_run(sb, want))
        torch.cuda.synchronize()
    return outs


def test_overlapped_streams_equal_serial(overlap_setup):
    """three overlapped runs of the 6-stream step, each byte-identical to the serial run"""
    _, subs = overlap_setup
    ser = np.concatenate([o["results"].cpu().numpy() for o in _serial(subs)])
    for rep in range(3):
        ovl = _overlapped(subs)
        diff = np.nonzero(np.any(ovl != ser, axis=1))[0]
        assert diff.size == 0, f"run {rep}: {diff.size} of {len(ser)} records differ: {diff[:10]}"
    assert np.array_equal(np.concatenate([o["results"].cpu().numpy() for o in _serial(subs)]), ser)


def test_overlapped_streams_against_oracle(overlap_setup, oracle):
    """one pair of every sub-batch (a different position in each) of an overlapped run against
    the oracle: status, M, K, min_idx, R and T, and the match list bit-exact"""
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    pairs, subs = overlap_setup
    res = np.ascontiguousarray(_overlapped(subs)).view(RESULT_DTYPE).reshape(-1)
    matches = [o["matches"].cpu().numpy() for o in _serial(subs, want=("matches",))]
    nthreads = max(1, min(16, len(os.sched_getaffinity(0))))
    picks = [i * PER + (7 * i) % PER for i in range(S)]
    ora = [bench.oracle_pair(pairs[k], ITERS, nthreads) for k in picks]
    got = np.stack([res[k] for k in picks])
    mt = np.stack([matches[k // PER][k % PER] for k in picks])
    par = bench.parity_check(got, mt, ora)
    assert par["all_equal"], par


def test_lite_estimates_equal_records(overlap_setup):
    """the batch pipeline's lite estimates (R1, R2, T as f32 SoA + per-wave counts, placed by
    valid_place_kernel; no 120-B records) against the record path (taken whenever the caller
    asks for the records): the consensus inputs (rvec, tvec in push order) and every result
    record byte-identical"""
    import torch
    _, subs = overlap_setup
    sb = subs[1]
    lite = _run(sb, want=("rvec", "tvec"))
    torch.cuda.synchronize()
    lite = {k: v.cpu().numpy() for k, v in lite.items()}
    rec = _run(sb, want=("rvec", "tvec", "hyps"))
    torch.cuda.synchronize()
    rec = {k: v.cpu().numpy() for k, v in rec.items()}
    for k in ("results", "rvec", "tvec"):
        assert np.array_equal(lite[k].view(np.uint8), rec[k].view(np.uint8)), k


def test_lite_estimates_equal_records_one_pair(overlap_setup):
    """the one-pair launch takes estimate_lite_kernel<true> (the eigen leftovers inlined: launches
    of <= 1024 waves) -- against the record path on the same pair, byte for byte"""
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner
    pairs, _ = overlap_setup
    sb = dict(b=bench.to_device(pairs[:1], "cuda"),
              run=PairBatchRunner(ctx=Context(0), iters=ITERS), st=torch.cuda.Stream())
    lite = _run(sb, want=("rvec", "tvec"))
    torch.cuda.synchronize()
    lite = {k: v.cpu().numpy() for k, v in lite.items()}
    rec = _run(sb, want=("rvec", "tvec", "hyps"))
    torch.cuda.synchronize()
    rec = {k: v.cpu().numpy() for k, v in rec.items()}
    for k in ("results", "rvec", "tvec"):
        assert np.array_equal(lite[k].view(np.uint8), rec[k].view(np.uint8)), k


def test_gram_row_tiles_identical(overlap_setup):
    """the Gram kernel with one or two 32-iteration row tiles per wave (ERP_OPT_GRAM_TILES 1 / 2;
    the launcher picks 2 for launches of >= 512 wide blocks) on the same 48-pair sub-batch: the
    hypothesis records (E included), the sample sets and the result records byte-identical"""
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner
    _, subs = overlap_setup
    outs = {}
    for wt in (1, 2):
        c = Context(0)
        c.set_option("gram_tiles", wt)
        sb = dict(b=subs[3]["b"], run=PairBatchRunner(ctx=c, iters=ITERS), st=torch.cuda.Stream())
        o = _run(sb, want=("hyps", "samples"))
        torch.cuda.synchronize()
        outs[wt] = {k: v.cpu().numpy() for k, v in o.items()}
    for k in ("results", "hyps", "samples"):
        assert np.array_equal(outs[1][k].view(np.uint8), outs[2][k].view(np.uint8)), k


def test_small_batch_route_equals_pruning_route(overlap_setup):
    """a batch of <= ERP_OPT_SMALL_BATCH pairs bins every row (no pre-pruning: the single-pair
    latency route); the same pairs through the pruning route give every result field equal
    (only the work counts binned_rows / survivors may differ)"""
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy
    pairs, _ = overlap_setup
    b = bench.to_device(pairs[:6], "cuda")
    args = (b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
            b["height"], b["max_nq"], b["max_nt"])
    res = {}
    for route, limit in (("all_rows", 8), ("prune", 0)):
        c = Context(0)
        c.set_option("small_batch", limit)
        out = PairBatchRunner(ctx=c, iters=ITERS).run(*args)
        torch.cuda.synchronize()
        res[route] = results_to_numpy(out["results"])
    a, c = res["all_rows"], res["prune"]
    for f in a.dtype.names:
        if f not in ("binned_rows", "survivors"):
            assert np.array_equal(a[f], c[f]), f
    assert np.all(a["binned_rows"] == a["K"]) and np.all(c["binned_rows"] < c["K"])


def test_survivor_zoom_equals_no_zoom(overlap_setup):
    """the survivors' zoom stage (ERP_OPT_ZOOM_LEVELS = 1, the default until r05; 2 = a second level)
    only tightens bounds before the refine: every result field equals the default route's (0),
    only the work count `survivors` may differ -- on a 48-pair sub-batch through the pruning
    route"""
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy
    _, subs = overlap_setup
    b = subs[2]["b"]
    args = (b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
            b["height"], b["max_nq"], b["max_nt"])
    res = {}
    for zl in ("0", "1", "2"):
        c = Context(0)
        c.set_option("zoom_levels", int(zl))
        out = PairBatchRunner(ctx=c, iters=ITERS).run(*args)
        torch.cuda.synchronize()
        res[zl] = results_to_numpy(out["results"])
    for zl in ("1", "2"):
        for f in res["0"].dtype.names:
            if f != "survivors":
                assert np.array_equal(res["0"][f], res[zl][f]), (zl, f)
