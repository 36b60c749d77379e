#!/usr/bin/env python3
"""Run-to-run and overlap determinism probes of the pair pipeline (GPU box).  Every kernel's
output is a function of its inputs, so records must be byte-identical between runs and between
the overlapped and the serial execution of the bench step (the -m gpu twin of the second probe is
tests/test_gpu_overlap.py; DESIGN.md 5d has the round-4 history these probes localised).

    python scripts/dev/determinism.py repeat  [--pairs 64] [--runs 3] [--twin] [--fresh-ctx]
        one batch through the pipeline --runs times: the record fields that differ
    python scripts/dev/determinism.py streams [--subs 6] [--pairs 768] [--want rvec,tvec,hyps]
                                              [--repeat N] [--same]
        the bench step's sub-batches on their own contexts / streams at once (bench.py call())
        against the same sub-batches one after the other: records and per-iteration outputs;
        --repeat N more overlapped runs counted against the serial records (round 5: 0 of
        30 720 with --repeat 40, profiles/r05c_determinism_rvec_repeat40.txt)
    python scripts/dev/determinism.py bounds  [--pair 6] [--overlap 1] [--reps 4] [--twin]
        the consensus bounds phase (erp_consensus_hyps_shard_dev, one shard) of one pair, run
        --reps times on --overlap contexts / streams at once: rows whose lb / ub / bsel differ
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

ITERS = 10000


def _pairs(n: int, twin: bool):
    import bench
    from erp_match_eightpoint_test_amd import synth
    if twin:  # two-cluster configs[1]-shaped pairs (R1 and R2 both valid in every iteration)
        seeds = json.load(open(os.path.join(ROOT, "scripts", "twin_seeds.json")))["seeds"][:n]
        return [synth.make_pair(s, n_kpts=4096, inlier_frac=0.98) for s in seeds]
    return bench.make_batch(0, n, 4096, 20200423)


def _field_diffs(a, c, names):
    out = {}
    for f in names:
        ne = np.nonzero(np.any((a[f] != c[f]).reshape(len(a), -1), axis=1))[0]
        if len(ne):
            out[f] = ne
    return out


def cmd_repeat(args):
    import torch

    import bench
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    b = bench.to_device(_pairs(args.pairs, args.twin), "cuda")
    batch = (b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
             b["height"], b["max_nq"], b["max_nt"])
    run0 = PairBatchRunner(ctx=Context(0), iters=ITERS)
    outs = []
    for _ in range(args.runs):
        r = PairBatchRunner(ctx=Context(0), iters=ITERS) if args.fresh_ctx else run0
        o = r.run(*batch)
        torch.cuda.synchronize()
        outs.append(results_to_numpy(o["results"]).copy())
    for k in range(1, args.runs):
        d = _field_diffs(outs[0], outs[k], RESULT_DTYPE.names)
        for f, ne in d.items():
            print(f"run {k}: field {f} differs on {len(ne)} pairs, first {ne[:12].tolist()}")
        print(f"run {k}: identical = {np.array_equal(outs[0].view(np.uint8), outs[k].view(np.uint8))}")
    print("survivors", outs[0]["survivors"][:24].tolist())
    print("binned_rows", outs[0]["binned_rows"][:24].tolist())


def cmd_streams(args):
    import torch

    import bench
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner
    from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE
    S, B = args.subs, args.pairs
    want = tuple(w for w in args.want.split(",") if w)
    pairs = bench.make_batch(0, B, 4096, 20200423)
    subs = []
    for i in range(S):
        j = 0 if args.same else i  # --same: every sub-batch the same pairs
        sb = bench.to_device(pairs[j * B // S:(j + 1) * B // S], "cuda")
        subs.append(dict(b=sb, run=PairBatchRunner(ctx=Context(0), iters=ITERS),
                         st=torch.cuda.Stream()))

    def run_one(sb):
        b = sb["b"]
        with torch.cuda.stream(sb["st"]):
            o = sb["run"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                              b["off_r"], b["width"], b["height"], b["max_nq"], b["max_nt"],
                              want=want, stream=sb["st"].cuda_stream)
            return {k: v.clone() for k, v in o.items()}

    def gather(outs):
        return {k: torch.cat([o[k] for o in outs]).cpu().numpy() for k in outs[0]}

    def overlapped():
        outs = [run_one(sb) for sb in subs]  # every sub-batch enqueued before any finishes
        torch.cuda.synchronize()
        return gather(outs)

    def serial():
        outs = []
        for sb in subs:
            outs.append(run_one(sb))
            torch.cuda.synchronize()
        return gather(outs)

    r = {"ser0": serial(), "ovl0": overlapped(), "ovl1": overlapped(), "ser1": serial()}
    a0 = r["ser0"]["results"].view(RESULT_DTYPE).reshape(-1)
    for k in ("ser1", "ovl0", "ovl1"):
        for name in r["ser0"]:
            if name == "results":
                c = r[k]["results"].view(RESULT_DTYPE).reshape(-1)
                d = _field_diffs(a0, c, RESULT_DTYPE.names)
                for f, ne in d.items():
                    print(f"{k}: results.{f} differs on {len(ne)} pairs, first {ne[:8].tolist()}")
                print(f"{k}: records identical to ser0: {not d}")
                continue
            a, c = r["ser0"][name], r[k][name]
            dd = np.any((a != c).reshape(a.shape[0], a.shape[1], -1), axis=2)
            np_ = np.nonzero(dd.any(axis=1))[0]
            print(f"{k}: {name} differs on {len(np_)} pairs ({int(dd.sum())} iterations)")
    if args.same:
        for k in ("ser0", "ovl0", "ovl1"):
            br = r[k]["results"].view(RESULT_DTYPE).reshape(-1)["binned_rows"].reshape(S, -1)
            print(k, "sub-batches with binned_rows unlike sub-batch 0:",
                  [i for i in range(1, S) if not np.array_equal(br[i], br[0])])
    if args.repeat:
        res_fields = [f for f in RESULT_DTYPE.names if f not in ("binned_rows", "survivors")]
        nbad = nbr = 0
        for _ in range(args.repeat):
            c = overlapped()["results"].view(RESULT_DTYPE).reshape(-1)
            bad = np.zeros(len(a0), bool)
            for f in res_fields:
                bad |= np.any((a0[f] != c[f]).reshape(len(a0), -1), axis=1)
            nbad += int(bad.sum())
            nbr += int((a0["binned_rows"] != c["binned_rows"]).sum())
            if bad.any():
                print("result fields differ on pairs", np.nonzero(bad)[0].tolist())
        print(f"REPEAT {args.repeat}: {args.repeat * len(a0)} overlapped records, {nbad} with a "
              f"result field unlike the serial run's, {nbr} with other binned_rows")


def cmd_bounds(args):
    import torch

    import oracle as O  # (the matcher, for the pair's keypoint lists only)
    from erp_match_eightpoint_test_amd import Context
    from erp_match_eightpoint_test_amd.capi import HYP_DTYPE
    from erp_match_eightpoint_test_amd.dist import CapiShardBackend
    p = _pairs(1, True)[0] if args.twin else _pairs(10, False)[args.pair]
    mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=16)
    kl = torch.from_numpy(np.ascontiguousarray(p["kp_l"][mt["queryIdx"]])).cuda()
    kr = torch.from_numpy(np.ascontiguousarray(p["kp_r"][mt["trainIdx"]])).cuda()
    hy = torch.zeros((ITERS, HYP_DTYPE.itemsize), dtype=torch.uint8, device="cuda")
    CapiShardBackend(Context(0), p["W"], p["H"], kl, kr, len(mt), {}).hyps(0, ITERS, hy)
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream() for _ in range(args.overlap)]
    bes = [CapiShardBackend(Context(0), p["W"], p["H"], kl, kr, len(mt), {}, stream=st.cuda_stream)
           for st in sts]
    outs = []
    for _ in range(args.reps):
        parts = [torch.zeros((3, 2 * ITERS), dtype=torch.float64, device="cuda") for _ in bes]
        for be, part in zip(bes, parts):
            be.shard(hy, ITERS, 0, 1, part)
        torch.cuda.synchronize()
        outs += [x.cpu().numpy() for x in parts]
    ref = outs[0]
    nd = 0
    for i, o in enumerate(outs[1:], 1):
        d = np.nonzero(np.any(o.view(np.uint64) != ref.view(np.uint64), axis=0))[0]
        if len(d):
            nd += 1
            print(f"output {i}: {len(d)} rows differ, e.g. {d[:6].tolist()}")
            for r in d[:4]:
                print(f"   row {r}: lb {ref[0, r]!r} vs {o[0, r]!r}; ub {ref[1, r]!r} vs {o[1, r]!r}; "
                      f"bsel {ref[2].view(np.int32)[2 * r:2 * r + 2]} vs "
                      f"{o[2].view(np.int32)[2 * r:2 * r + 2]}")
    print(f"{len(outs)} outputs, {nd} differ from the first; rows with ub != 0: "
          f"{int((ref[1] != 0).sum())}")


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    sp = ap.add_subparsers(dest="cmd", required=True)
    a = sp.add_parser("repeat")
    a.add_argument("--pairs", type=int, default=64)
    a.add_argument("--runs", type=int, default=3)
    a.add_argument("--twin", action="store_true")
    a.add_argument("--fresh-ctx", action="store_true", help="a new context per run")
    a = sp.add_parser("streams")
    a.add_argument("--subs", type=int, default=6)
    a.add_argument("--pairs", type=int, default=768)
    a.add_argument("--want", default="rvec,tvec,hyps")
    a.add_argument("--repeat", type=int, default=0)
    a.add_argument("--same", action="store_true")
    a = sp.add_parser("bounds")
    a.add_argument("--pair", type=int, default=6)
    a.add_argument("--overlap", type=int, default=1)
    a.add_argument("--reps", type=int, default=4)
    a.add_argument("--twin", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    {"repeat": cmd_repeat, "streams": cmd_streams, "bounds": cmd_bounds}[args.cmd](args)


if __name__ == "__main__":
    main()
