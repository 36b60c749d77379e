"""Probe: the bench step's sub-batches on S contexts / streams at once against the same
sub-batches one after the other, comparing the per-iteration debug outputs (WANT, default
rvec,tvec,hyps) as well as the records: does the overlap change the consensus inputs?"""
import os
import sys

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy  # noqa: E402
from erp_match_eightpoint_test_amd.capi import RESULT_DTYPE  # noqa: E402

S, B = 6, 768
WANT = tuple(w for w in os.environ.get("WANT", "rvec,tvec,hyps").split(",") if w)
pairs = bench.make_batch(0, B, 4096, 20200423)
subs = []
for i in range(S):
    b = bench.to_device(pairs[i * B // S:(i + 1) * B // S], "cuda")
    subs.append(dict(b=b, run=PairBatchRunner(ctx=Context(0), iters=10000), st=torch.cuda.Stream()))


def run_one(sb):
    b = sb["b"]
    with torch.cuda.stream(sb["st"]):
        o = sb["run"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"],
                          b["width"], b["height"], b["max_nq"], b["max_nt"], want=WANT,
                          stream=sb["st"].cuda_stream)
        return {k: v.clone() for k, v in o.items()}


def gather(outs):
    return {k: torch.cat([o[k] for o in outs]).cpu().numpy() for k in outs[0]}


def overlapped():
    outs = [run_one(sb) for sb in subs]
    torch.cuda.synchronize()
    return gather(outs)


def serial():
    outs = []
    for sb in subs:
        outs.append(run_one(sb))
        torch.cuda.synchronize()
    return gather(outs)


r = {"ser0": serial()}
L = subs[0]["run"].ctx.L
if os.environ.get("ERP_ALLOC_PAD"):
    print("canaries overwritten after the serial run:", L.erp_debug_check_pads())
r.update(ovl0=overlapped(), ovl1=overlapped(), ser1=serial())
# REPEAT = n: n more overlapped runs, counting the records whose result fields (everything but
# the work diagnostics binned_rows / survivors) differ from the serial run's
rep = int(os.environ.get("REPEAT", "0"))
if rep:
    a0 = r["ser0"]["results"].view(RESULT_DTYPE).reshape(-1)
    res_fields = [f for f in RESULT_DTYPE.names if f not in ("binned_rows", "survivors")]
    nbad = nbr = 0
    for _ in range(rep):
        c = overlapped()["results"].view(RESULT_DTYPE).reshape(-1)
        bad = np.zeros(len(a0), bool)
        for f in res_fields:
            bad |= np.any((a0[f] != c[f]).reshape(len(a0), -1), axis=1)
        nbad += int(bad.sum())
        nbr += int((a0["binned_rows"] != c["binned_rows"]).sum())
        if bad.any():
            print("result fields differ on pairs", np.nonzero(bad)[0].tolist())
    print(f"REPEAT {rep}: {rep * len(a0)} overlapped records, {nbad} with a result field unlike the "
          f"serial run's, {nbr} with other binned_rows")
if os.environ.get("ERP_ALLOC_PAD"):
    print("canaries overwritten after all runs:", L.erp_debug_check_pads())
for k in ("ser1", "ovl0", "ovl1"):
    for name in r["ser0"]:
        a, c = r["ser0"][name], r[k][name]
        if name == "results":
            a, c = a.view(RESULT_DTYPE).reshape(-1), c.view(RESULT_DTYPE).reshape(-1)
            for f in RESULT_DTYPE.names:
                ne = np.nonzero(np.any((a[f] != c[f]).reshape(len(a), -1), axis=1))[0]
                if len(ne):
                    print(f"{k}: results.{f} differs on {len(ne)} pairs, first {ne[:8].tolist()}")
            continue
        d = np.any((a != c).reshape(a.shape[0], a.shape[1], -1), axis=2)
        np_ = np.nonzero(d.any(axis=1))[0]
        print(f"{k}: {name} differs on {len(np_)} pairs ({int(d.sum())} iterations)"
              + (f", e.g. pair {np_[0]} iterations {np.nonzero(d[np_[0]])[0][:8].tolist()}" if len(np_) else ""))

# ERP_DEBUG_SNAP=1: lb / ub / first-stage counts right after the bounds pass, per sub-batch
if os.environ.get("ERP_DEBUG_SNAP") == "1":
    import ctypes as C
    L.erp_debug_snapshot.restype = C.c_longlong
    L.erp_debug_snapshot.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]

    def snaps():
        out = []
        for sb in subs:
            h = sb["run"].ctx.h
            n = L.erp_debug_snapshot(h, None, 0)
            buf = np.empty(n, np.uint8)
            assert L.erp_debug_snapshot(h, buf.ctypes.data, n) == n
            P = 128
            nrow = P * 20000
            cap = 20000 // 4 + 64
            lb = buf[:nrow * 8].view(np.float64).reshape(P, -1)
            ub = buf[nrow * 8:nrow * 16].view(np.float64).reshape(P, -1)
            o = nrow * 16
            cnt = buf[o:o + 4 * P].view(np.int32)
            o += 4 * P
            lref = buf[o:o + P * cap * 16].view(np.float32).reshape(P, cap, 4)
            o += P * cap * 16
            lU = buf[o:o + 8 * P].view(np.float64)
            lcnt = buf[o + 8 * P:o + 12 * P].view(np.int32)
            rvend = buf[o + 12 * P:].view(np.float32).reshape(P, 3, -1) if n > o + 12 * P else None
            out.append((lb, ub, cnt, lref, lU, lcnt, rvend))
        return out

    def run_and_snap(f):
        res = f()
        return res, snaps()

    (_, s0) = run_and_snap(serial)
    (_, s1) = run_and_snap(overlapped)
    (_, s2) = run_and_snap(serial)
    for name, sx in (("ovl", s1), ("ser", s2)):
        for i in range(len(subs)):
            lb0, ub0, c0 = s0[i][:3]
            lb1, ub1, c1 = sx[i][:3]
            K = r["ser0"]["results"].view(RESULT_DTYPE).reshape(-1)["K"][i * 128:(i + 1) * 128]
            dc = np.nonzero(c0 != c1)[0]
            msg = []
            for p in dc[:3]:
                k = int(K[p])
                ref = np.arange(0, k, 32)
                dl = np.nonzero(lb0[p, :k] != lb1[p, :k])[0]
                du = np.nonzero(ub0[p, :k] != ub1[p, :k])[0]
                msg.append(f"pair {p}: count {c0[p]} vs {c1[p]}, K {k}; lb differs on {len(dl)} rows "
                           f"({np.isin(dl, ref).sum()} refs, first {dl[:4].tolist()}), ub on {len(du)} "
                           f"({np.isin(du, ref).sum()} refs); ref lb/ub equal: "
                           f"{np.array_equal(lb0[p, ref], lb1[p, ref]) and np.array_equal(ub0[p, ref], ub1[p, ref])}")
                if len(dl):
                    j = dl[0]
                    msg.append(f"   row {j}: lb {lb0[p, j]!r} vs {lb1[p, j]!r}, ub {ub0[p, j]!r} vs {ub1[p, j]!r}")
            print(f"snap {name} sub-batch {i}: counts differ on {len(dc)} pairs", *msg, sep="\n  ")

    # the consensus's SoA rotation vectors at the end of the run: equal to the AOS rvec output
    # (written by the same compaction) in every run?
    for name, sx, rk in (("ser", s0, "ser0"), ("ovl", s1, None)):
        for i in range(len(subs)):
            rvend = sx[i][6]
            if rvend is None:
                continue
            K = r["ser0"]["results"].view(RESULT_DTYPE).reshape(-1)["K"][i * 128:(i + 1) * 128]
            nb = 0
            for p in range(128):
                k = int(K[p])
                aos = r["ser0"]["rvec"][i * 128 + p, :k] if "rvec" in WANT else None
                if aos is not None and not np.array_equal(rvend[p, :, :k].T, aos):
                    nb += 1
                    if nb <= 2:
                        d = np.nonzero(np.any(rvend[p, :, :k].T != aos, axis=1))[0]
                        print(f"  {name} sub {i} pair {p}: {len(d)} rows of rv changed, first {d[:4].tolist()}")
            print(f"rv at the end, {name} sub-batch {i}: {nb} pairs with rv unlike the rvec output")

    # the first-stage Lipschitz test of the rows whose pruning differs, redone on the host from
    # the serial snapshot (kernels.hip consensus_lip_refs_kernel / lip_prune_rows, M = 1e-6)
    if "rvec" in WANT:
        M = 1e-6
        for i in range(len(subs)):
            lb0, ub0, c0, lr0, lU0, lc0 = s0[i][:6]
            lb1, ub1, c1, lr1, lU1, lc1 = s1[i][:6]
            K = r["ser0"]["results"].view(RESULT_DTYPE).reshape(-1)["K"][i * 128:(i + 1) * 128]
            for p in np.nonzero(c0 != c1)[0][:2]:
                k = int(K[p])
                X = r["ser0"]["rvec"][i * 128 + p, :k].astype(np.float32)
                ref = np.arange(0, k, 32)
                U = ub0[p, ref].min()
                a = lb0[p, ref] * (1 - M) - U * (1 + M)
                live = a > 0
                thr = (a[live] * a[live] * (1 - M)).astype(np.float32)
                R = X[ref[live]]
                for j in np.nonzero((lb0[p, :k] != lb1[p, :k]))[0][:2]:
                    d = X[j] - R
                    s2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]).astype(np.float32)
                    q = np.argmin(s2 - thr)
                    rr = ref[live][q]
                    def has(lr, lc):  # the pruning reference among the kernel's staged ones
                        e = lr[p, :lc[p]]
                        return int(((e[:, 0] == X[rr, 0]) & (e[:, 1] == X[rr, 1]) & (e[:, 2] == X[rr, 2])).sum())
                    sset = lambda lr, lc: sorted(map(tuple, lr[p, :lc[p]].tolist()))
                    print(f"  lcnt {lc0[p]} vs {lc1[p]}, lU {lU0[p]!r} vs {lU1[p]!r}, pruning ref staged "
                          f"{has(lr0, lc0)} vs {has(lr1, lc1)} times, staged sets equal: {sset(lr0, lc0) == sset(lr1, lc1)}")
                    print(f"sub {i} pair {p} row {j}: U {U!r}, serial LB/U {lb0[p, j] / U!r}; "
                          f"{int(live.sum())} refs; min (s2 - thr) {float(s2[q] - thr[q])!r} at ref row "
                          f"{ref[live][q]} (thr {float(thr[q])!r}); rows with s2 < thr: {int((s2 < thr).sum())}")
