"""Probe (round 5): which pipeline stage perturbs kernels running beside it on other streams?

Part 1 (GUARD=1): the LDS guard kernel (scripts/dev/lds_guard.hip) on a stream of its own while
one stage group of the pipeline (ERP_OPT_DEBUG_STAGES mask) runs on S sub-batch streams: every LDS
word of a guard workgroup that changes under it was written by another workgroup.

Part 2 (PAIRS=1): the victim = sub-batch 0's consensus alone (mask 16), the aggressors = the other
sub-batches running one stage group each, overlapped; the victim's records against its records
from a run with nothing beside it.

Env: SAMPLER (0 glibc / 1 philox), S (sub-batches, default 6), REPS, MASKS (comma list)."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy  # noqa: E402

SAMPLER = int(os.environ.get("SAMPLER", "0"))
S = int(os.environ.get("S", "6"))
REPS = int(os.environ.get("REPS", "10"))
MASKS = [int(m, 0) for m in os.environ.get("MASKS", "1,2,4,8,16,31").split(",")]
B = 128 * S
pairs = bench.make_batch(0, B, 4096, 20200423)
subs = []
for i in range(S):
    b = bench.to_device(pairs[i * 128:(i + 1) * 128], "cuda")
    subs.append(dict(b=b, run=PairBatchRunner(ctx=Context(0), iters=10000, sampler=SAMPLER),
                     st=torch.cuda.Stream()))


def run_one(sb, mask):
    sb["run"].ctx.set_option("debug_stages", mask)  # (ERP_OPT_DEBUG_STAGES)
    b = sb["b"]
    with torch.cuda.stream(sb["st"]):
        o = sb["run"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"],
                          b["width"], b["height"], b["max_nq"], b["max_nt"],
                          stream=sb["st"].cuda_stream)
    return o["results"]


# one full serial pass: every context's scratch holds valid intermediate results
for sb in subs:
    run_one(sb, -1)
    torch.cuda.synchronize()
for _sb in subs:
    _sb["run"].ctx.set_option("debug_stages", -1)
print("sampler", SAMPLER, "sub-batches", S, "lib", os.environ.get("ERP_LIB_PATH", "in-tree"), flush=True)

if os.environ.get("GUARD", "1") == "1":
    G = C.CDLL(os.path.join(ROOT, "scripts", "dev", "liblds_guard.so"))
    G.lds_guard_launch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_longlong, C.c_uint32,
                                   C.c_void_p, C.c_int]
    MAXREC = 4096
    out = torch.zeros(16 + 8 * MAXREC, dtype=torch.int32, device="cuda")
    gst = torch.cuda.Stream()
    NW = int(os.environ.get("GUARD_NW", "16"))  # 16 KB per guard workgroup
    NBLK = int(os.environ.get("GUARD_BLOCKS", "512"))
    for mask in MASKS:
        # the stage group's duration alone (sub-batches overlapped), to size the guard's spin
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for sb in subs:
            run_one(sb, mask)
        torch.cuda.synchronize()
        t_stage = time.perf_counter() - t0
        out.zero_()
        torch.cuda.synchronize()
        spin = max(2e-3, 0.25 * t_stage)
        n_guard = int(REPS * t_stage / spin) + 2
        if os.environ.get("GUARD_AFTER") == "1":
            # the stage's workgroups first, then a guard launch behind each round of them: the
            # guard workgroups take the LDS the stage's finished workgroups free, between its
            # running ones
            n_guard = REPS
            spin = max(1e-3, 0.8 * t_stage)
            for r in range(REPS):
                for sb in subs:
                    run_one(sb, mask)
                rc = G.lds_guard_launch(gst.cuda_stream, NBLK, NW, int(spin * 1e8), 0x1234567 + r,
                                        out.data_ptr(), MAXREC)
                assert rc == 0, rc
        else:
            for g in range(n_guard):  # guard kernels back to back on their own stream
                rc = G.lds_guard_launch(gst.cuda_stream, NBLK, NW, int(spin * 1e8), 0x1234567 + g,
                                        out.data_ptr(), MAXREC)
                assert rc == 0, rc
            for r in range(REPS):
                for sb in subs:
                    run_one(sb, mask)
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        nbad, nrec, ndone, rounds = int(o[0]), int(o[1]), int(o[2]), int(o[3])
        print(f"GUARD mask {mask:#x}: stage {t_stage * 1e3:.2f} ms x {REPS}, {n_guard} guard "
              f"launches of {spin * 1e3:.1f} ms ({ndone} workgroups done, {rounds} check rounds): "
              f"{nbad} changed LDS words", flush=True)
        recs = o[16:16 + 8 * min(nrec, MAXREC)].reshape(-1, 8)
        for r in recs[:12]:
            blk, idx, got, exp, hw, xcc, dt, _ = (int(x) for x in r)
            print(f"   blk {blk} word {idx} got {got:#010x} expected {exp:#010x} "
                  f"(cleared {exp & ~got:#010x}, set {got & ~exp:#010x}) hw_id {hw:#x} xcc {xcc:#x} "
                  f"t+{dt / 100:.0f} us", flush=True)
    for _sb in subs:
        _sb["run"].ctx.set_option("debug_stages", -1)

if os.environ.get("PK", "0") == "1":
    # the packed-f32 pruning test against scalar f32 (scripts/dev/lds_guard.hip pk_probe_kernel)
    # beside each stage group, and alone (mask 0)
    G = C.CDLL(os.path.join(ROOT, "scripts", "dev", "liblds_guard.so"))
    G.pk_probe_launch.argtypes = [C.c_void_p, C.c_int, C.c_longlong, C.c_uint32, C.c_void_p, C.c_int]
    MAXREC = 4096
    out = torch.zeros(16 + 8 * MAXREC, dtype=torch.int32, device="cuda")
    gst = torch.cuda.Stream()
    NBLK = int(os.environ.get("PK_BLOCKS", "512"))
    for mask in [0] + MASKS:
        t_stage = 4e-3
        if mask:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for sb in subs:
                run_one(sb, mask)
            torch.cuda.synchronize()
            t_stage = time.perf_counter() - t0
        out.zero_()
        torch.cuda.synchronize()
        spin = max(1e-3, 0.8 * t_stage)
        for r in range(REPS):
            if mask:
                for sb in subs:
                    run_one(sb, mask)
            rc = G.pk_probe_launch(gst.cuda_stream, NBLK, int(spin * 1e8), 0x2345 + r, out.data_ptr(), MAXREC)
            assert rc == 0, rc
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        print(f"PK mask {mask:#x}: {REPS} probe launches of {spin * 1e3:.1f} ms ({int(o[2])} workgroups, "
              f"{int(o[3])} rounds): {int(o[0])} packed results unlike scalar", flush=True)
        for r in o[16:16 + 8 * min(int(o[1]), 8)].reshape(-1, 8):
            blk, tid, q, d0, t0s, d1, t1s, dt = (int(x) for x in r)
            print(f"   blk {blk} tid {tid} ref {q}: lo {d0:#010x} vs {t0s:#010x}, hi {d1:#010x} vs {t1s:#010x}, t+{dt / 100:.0f} us",
                  flush=True)
    for _sb in subs:
        _sb["run"].ctx.set_option("debug_stages", -1)

if os.environ.get("PAIRS", "1") == "1":
    vic = subs[0]

    def victim_alone():
        r = run_one(vic, 16)
        torch.cuda.synchronize()
        return results_to_numpy(r)

    L = vic["run"].ctx.L
    dbg = np.zeros(64, np.uint32)
    verify = L.erp_debug_lip_counters(dbg.ctypes.data) == 0

    def lip_counters(tag):
        if not verify:
            return
        L.erp_debug_lip_counters(dbg.ctypes.data)
        print(f"   LIP_VERIFY {tag}: refs differing {int(dbg[0])}, rows differing {int(dbg[1])}", flush=True)
        for k in range(min(int(dbg[2]), 14)):
            kind, a, b, c = (int(x) for x in dbg[8 + 4 * k:12 + 4 * k])
            print(f"      kind {kind} a {a} b {b:#010x} c {c:#010x}", flush=True)

    base = victim_alone()
    lip_counters("victim alone")
    again = victim_alone()
    print("PAIRS victim alone twice identical:", np.array_equal(base.view(np.uint8), again.view(np.uint8)),
          flush=True)
    for mask in MASKS:
        nd = 0
        nres = 0
        for r in range(REPS):
            for sb in subs[1:]:
                run_one(sb, mask)
            for sb in subs[1:]:
                run_one(sb, mask)
            rv = run_one(vic, 16)
            torch.cuda.synchronize()
            res = results_to_numpy(rv)
            d = base.view(np.uint8).reshape(len(base), -1) != res.view(np.uint8).reshape(len(res), -1)
            nd += int(np.any(d, axis=1).sum())
            for f in res.dtype.names:
                if f not in ("binned_rows", "survivors"):
                    nres += int(np.any((res[f] != base[f]).reshape(len(res), -1), axis=1).sum())
        print(f"PAIRS aggressor mask {mask:#x}: {nd} of {REPS * len(base)} victim records differ "
              f"({nres} result-field differences)", flush=True)
        lip_counters(f"aggressor mask {mask:#x}")
