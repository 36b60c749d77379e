#!/usr/bin/env python3
"""Benchmark of the ERP hot path on MI355X: ERP image-pairs/sec (4k x 4k kpts, 10k RANSAC iters).

Workload (BASELINE.json configs[1] shape): synthetic ERP pairs of 4096 x 4096 64-D SURF-like
descriptors + keypoints (W x H = 5376 x 2688), exact k=2 + ratio-0.3 match -> gather ->
eight_point::find with 10 000 initial_guess iterations (glibc-replay sampler, reference
defaults otherwise).  A step = B such pairs resident in HBM, split into S independent
sub-batches (own context + HIP stream each, so one sub-batch's latency-bound kernels overlap
the other's); every step recomputes everything (no cached outputs).  Defaults B = 768, S = 6 (six
sub-batches of 128 on six HIP streams: the latency-bound consensus / eigen kernels of one
overlap the VALU- and MFMA-bound kernels of the others; r03 sweep on one MI355X, 8 steps each,
profiles/r03n_step_sweep.txt: 768 x 4 34.8-35.0k pairs/s, 768 x 6 35.7-36.5k, 768 x 8
34.9-35.2k, 1024 x 4 35.1k, 1536 x 4 34.6k, 1536 x 6 35.6k; the r02m sweep had 768 x 4 ahead of
768 x 3 and 384 x 3, profiles/r02m_streamsweep.txt).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs B] [--streams S] [--iters I]

N > 1: launched by torch.distributed.run, one rank per GPU; each rank runs its own B pairs
(weak scaling, independent pairs = the reference's per-pair process) and the per-pair result
records are all-gathered over RCCL every step (the "best-model gather" of configs[2]).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_VALU_UNFUSED = 157.3 / 2  # TFLOP/s: 157.3 counts an FMA as 2; sub/mul/add are 1 each
PEAK_FP64_VALU = 78.6               # TFLOP/s (MI355X spec, FMA = 2)
PEAK_HBM = 8000.0                   # GB/s
PEAK_BF16_MFMA = 2516.6             # TFLOP/s dense (256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz)
PEAK_I8_MFMA = 2 * PEAK_BF16_MFMA   # TOP/s dense (32x32x32 i8 = the cycles of 32x32x16 bf16)
# VALU lane-op peak (MI355X_MICROARCH.md "Wave scheduling": a wave64 VALU instruction issues
# over 2 cycles on a SIMD-32, i.e. 32 lanes / cycle / SIMD): 256 CU x 4 SIMD x 32 x 2.4 GHz
PEAK_VALU_OPS = 256 * 4 * 32 * 2.4e9 / 1e12          # 78.6 T lane-ops/s
PEAK_VALU_OPS_4CYC = PEAK_VALU_OPS / 2                # secondary: every op at 4 cycles (39.3)
# profiles/<tag>_pmc_<stage>.json of the shipped step (768 pairs, 6 sub-batches = 128-pair
# launches): the HBM bytes per launch that roofline.traffic reports
PROFILE_TAG = "r06ap"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=768, help="pairs per step per GPU")
    ap.add_argument("--streams", type=int, default=6,
                    help="independent sub-batches (own context + HIP stream) per step")
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--kpts", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=20200423)
    ap.add_argument("--inlier-frac", type=float, default=0.8,
                    help="pairs workload: fraction of left keypoints with a true partner")
    ap.add_argument("--sigma", type=float, default=0.03,
                    help="pairs workload: descriptor noise of the true partners")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--main-batch", choices=["default", "worst"], default="default",
                    help="pairs workload: 'worst' makes the timed batch itself the worst-case "
                         "batch (for stage profiles of it; not the headline)")
    ap.add_argument("--sampler", choices=["glibc", "philox"], default="glibc",
                    help="glibc: the reference's rand() replay (the headline); philox: the "
                         "counter-based mode (SURVEY 8b), parity against the oracle in that mode")
    ap.add_argument("--worst-steps", type=int, default=3,
                    help="pairs workload: timed steps of the worst-case batch (every pair a "
                         "two-cluster consensus pair -- R1 and R2 both valid, K ~ 2 x iters -- "
                         "at inlier fraction 0.98, so M ~ 4k; scripts/twin_seeds.json)")
    ap.add_argument("--hard-steps", type=int, default=3,
                    help="pairs workload: timed steps of a second, harder batch (half the left "
                         "keypoints without a partner, descriptor noise 0.035, 30%% of the true "
                         "matches at wrong positions) reported beside the headline; 0 = off")
    ap.add_argument("--cpu-seconds", type=float, default=30.0)  # (~48 oracle pairs: the parity sample)
    ap.add_argument("--profile-tag", default=PROFILE_TAG,
                    help="profiles/<tag>_pmc_<stage>.json: HBM bytes per launch (roofline.traffic)")
    ap.add_argument("--matcher", choices=["mfma", "valu"], default="mfma",
                    help="exact k=2 method: bf16-MFMA filter + rescoring, or the packed-FP32 sweep")
    ap.add_argument("--no-shard-consensus", action="store_true",
                    help="manual workload: replicate the consensus on every rank")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: the process group's backend.  nccl (= RCCL) is the product path, "
                         "one rank per GPU; gloo (collectives on host copies) with "
                         "--ranks-on-device lets several ranks share one GPU, to rehearse the "
                         "multi-rank launcher, gather and checks on a 1-GPU box (not a scaling "
                         "number)")
    ap.add_argument("--ranks-on-device", type=int, default=-1,
                    help="N > 1, development: every rank uses this HIP device instead of "
                         "LOCAL_RANK's (with --dist-backend gloo: RCCL refuses two ranks on one GPU)")
    ap.add_argument("--ctx-option", action="append", default=[], metavar="NAME=VALUE",
                    help="erp_ctx_set_option on every context the bench makes (route options, "
                         "capi.OPTIONS: same results, for A/B runs; e.g. lip2=0)")
    ap.add_argument("--workload", choices=["pairs", "dense", "manual", "remap", "e2e"],
                    default="pairs",
                    help="pairs: configs[1] (the metric; configs[2] with --kpts 2048); dense: "
                         "configs[3], one N x N match (--kpts, default 16384) on both matcher "
                         "methods; manual: configs[4], one find() of --iters (default 100k) on "
                         "100 manual-pickup correspondences (60%% outliers), hypothesis blocks "
                         "sharded over the ranks; remap: section 8f, the spherical band remap "
                         "and rectification of 5376 x 2688 ERP images; e2e: the whole reference "
                         "pipeline per pair from 5376 x 2688 images (do_all + find)")
    return ap.parse_args()


def make_batch(rank: int, B: int, kpts: int, seed: int, inlier_frac: float = 0.8,
               sigma: float = 0.03, mismatch_frac: float = 0.0):
    from erp_match_eightpoint_test_amd import synth
    pairs = [synth.make_pair(seed + 1000 * rank + i, n_kpts=kpts, inlier_frac=inlier_frac,
                             sigma=sigma, mismatch_frac=mismatch_frac) for i in range(B)]
    return pairs


def make_worst_batch(rank: int, B: int, kpts: int, sigma: float):
    """the worst-case batch: two-cluster consensus pairs (scripts/twin_seeds.json: R1 and R2
    both valid) at inlier fraction 0.98"""
    from erp_match_eightpoint_test_amd import synth
    seeds = json.load(open(os.path.join(ROOT, "scripts", "twin_seeds.json")))["seeds"]
    return [synth.make_pair(seeds[(rank * B + i) % len(seeds)], n_kpts=kpts, inlier_frac=0.98,
                            sigma=sigma) for i in range(B)]


def to_device(pairs, dev):
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ol = np.concatenate([[0], np.cumsum([len(p["desc_l"]) for p in pairs])]).astype(np.int64)
    orr = np.concatenate([[0], np.cumsum([len(p["desc_r"]) for p in pairs])]).astype(np.int64)
    return dict(desc_l=t(np.concatenate([p["desc_l"] for p in pairs])),
                desc_r=t(np.concatenate([p["desc_r"] for p in pairs])),
                kp_l=t(np.concatenate([p["kp_l"] for p in pairs])),
                kp_r=t(np.concatenate([p["kp_r"] for p in pairs])),
                off_l=t(ol), off_r=t(orr),
                width=t(np.array([p["W"] for p in pairs], np.int32)),
                height=t(np.array([p["H"] for p in pairs], np.int32)),
                max_nq=int(np.diff(ol).max()), max_nt=int(np.diff(orr).max()))


def stage_work(stage, B, kpts, iters, res):
    """algorithmic work of ONE launch of `stage` over the batch:
    returns (amount, unit, peak, bound, note)."""
    M = res["M"].astype(np.float64)
    K = res["K"].astype(np.float64)
    if stage in ("knn2_filter", "knn2_candidates"):
        flops = 2.0 * kpts * kpts * 64 * B  # one bf16 product qh.th per (query, train) pair
        return flops, "TFLOP/s", PEAK_BF16_MFMA, "mfma", "2*N*T*64 bf16 MFMA flops per pair"
    if stage == "knn2_exact":
        ops = 3.0 * kpts * kpts * 64 * B  # sub, mul, add per element, flann::L2 order
        return ops, "Top/s", PEAK_FP32_VALU_UNFUSED, "valu", "3*N*T*64 fp32 ops per pair"
    if stage == "gram":
        nb = np.floor((M - 1) / 31) + 1  # selection words (31 rows + 1 pad each)
        ops = float(np.sum(2.0 * iters * 32 * nb * 216))  # 6 int8 limbs x 36 Gram entries
        return ops, "TOP/s", PEAK_I8_MFMA, "mfma", "2*I*32*nb*216 int8 MFMA ops per pair"
    if stage == "consensus_bounds":
        # binned rows x K squared distances (the reference rows + the rows that Lipschitz
        # pre-pruning kept; the pruning test itself is not counted)
        nb = res["binned_rows"].astype(np.float64)
        flops = float(np.sum(nb * K * 8.0))  # 3 sub, 3 mul, 2 add per squared distance
        return flops, "TFLOP/s", PEAK_FP32_VALU_UNFUSED, "valu", \
            "8 fp32 ops per binned squared distance (binned_rows x K)"
    if stage == "sampler" and SAMPLER == 1:
        s = np.floor(M * 0.25)
        ops = float(np.sum(s * iters * 27.0))
        return ops, "Top/s", PEAK_VALU_OPS, "valu", \
            "27 int lane-ops per Philox draw (10 rounds x ~10 ops per 4 draws + mulhi, test-and-" \
            "set); peak = wave64 2-cycle VALU issue"
    if stage == "sampler":
        ops = float(np.sum((M - 1) * iters * 4.0))  # per draw: recurrence, shift, remainder, test
        return ops, "Top/s", PEAK_VALU_OPS, "valu", \
            "4 int/fp64 lane-ops per rand() draw (floor); peak = wave64 2-cycle VALU issue"
    return None


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_share():
    """(threads to use, record): the CPUs this process may run on (sched_getaffinity) capped
    by the cgroup v2 CPU quota (cpu.max "quota period"; "max" = no cap).  os.cpu_count() is
    the whole machine's count on the GPU box, where a job gets a share of it."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cpu_max = None
    quota_cpus = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                cpu_max = f.read().strip()
            q, per = cpu_max.split()[:2]
            if q != "max":
                quota_cpus = max(1, int(-(-int(q) // int(per))))
        except (OSError, ValueError):
            pass
    threads = min(aff, quota_cpus) if quota_cpus else aff
    return threads, {"affinity_cpus": aff, "cgroup_cpu_max": cpu_max,
                     "cgroup_quota_cpus": quota_cpus, "host_cpus": os.cpu_count(),
                     "threads_basis": "min(sched_getaffinity, cgroup cpu.max quota)"}


SAMPLER = 0  # erp_ransac_cfg.sampler of every run (--sampler): 0 glibc replay, 1 Philox
CTX_OPTIONS: dict = {}  # --ctx-option: applied to every context by make_ctx


def make_ctx(device: int, **extra):
    """a Context with the --ctx-option route options (and `extra`) applied"""
    from erp_match_eightpoint_test_amd import Context
    ctx = Context(device)
    for k, v in {**CTX_OPTIONS, **extra}.items():
        ctx.set_option(k, v)
    return ctx


def oracle_pair(p, iters, nthreads):
    """one pair through the oracle (exact k=2 match + find), with its match list and the
    per-iteration validity flags (for the R1 / R2 order rule of parity_check)"""
    import oracle as O
    mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=nthreads)
    r = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
               O.make_cfg(iters=iters, sampler=SAMPLER), detail=True)
    r["matches"] = mt
    r["hyp"] = {"R1_valid": r["hyp"]["R1_valid"].copy(), "R2_valid": r["hyp"]["R2_valid"].copy()}
    for k in ("samples", "rvec", "tvec", "dist"):
        r.pop(k, None)
    return r


def cpu_baseline(pairs, iters, budget_s):
    """the oracle (CPU restatement, exact brute force + OpenCV-style SVD) on host cores: whole
    pairs of the same workload, as many as fit in ~budget_s (at least one), with OpenMP over
    the box's CPU share (the matcher is the parallel part; find() is serial like the
    reference's), then ONE pair again on a single thread.  Returns (record, oracle results of
    the pairs it ran) -- the results are the parity check of the timed workload (main())."""
    import oracle as O
    O.build()
    threads, share = host_cpu_share()
    os.environ["OMP_NUM_THREADS"] = str(threads)

    def one(p, nth):
        return oracle_pair(p, iters, nth)

    t0 = time.perf_counter()
    got = []
    for p in pairs:
        got.append(one(p, threads))
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    n = len(got)
    t1 = time.perf_counter()
    one(pairs[0], 1)
    dt1 = time.perf_counter() - t1
    rec = {"value": n / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
           "sample": f"{n} whole pair(s) of the bench workload ({len(pairs[0]['desc_l'])}x"
                     f"{len(pairs[0]['desc_r'])} kpts, {iters} iters) through oracle/ "
                     f"(exact-BF CPU restatement, OpenMP {threads} threads), {dt:.1f} s",
           "value_1core": 1.0 / dt1,
           "sample_1core": f"pair 0 again on 1 thread, {dt1:.2f} s",
           "cpu_model": _cpu_model(), **share}
    return rec, got


def parity_check(gpu_res, gpu_matches, ora):
    """the timed workload against the oracle, pair by pair (the pairs cpu_baseline ran): M, K
    and status equal, min_idx equal (dist.min_idx_agrees: one apart only when both rows are the
    R1 / R2 of ONE iteration, from the oracle's validity flags), R / T within 1e-6, the match list
    (queryIdx, trainIdx, distance bits) bit-exact.  gpu_res: result records of the timed step
    (same pairs, same order); gpu_matches: [pairs, max_nq, 4] int32 from an untimed pass with the
    matches out."""
    from erp_match_eightpoint_test_amd.dist import min_idx_agrees
    bad, swaps = [], []
    for i, o in enumerate(ora):
        r = gpu_res[i]
        M = len(o["matches"])
        hy = o.get("hyp")
        agree, swap = min_idx_agrees(r["min_idx"], o["min_idx"],
                                     None if hy is None else hy["R1_valid"],
                                     None if hy is None else hy["R2_valid"])
        if swap:
            swaps.append(i)
        ok = (int(r["status"]) == o["status"] == 0 and int(r["M"]) == M and int(r["K"]) == o["K"]
              and agree
              and float(np.abs(r["R"] - o["R"]).max()) <= 1e-6
              and float(np.abs(r["T"] - o["T"]).max()) <= 1e-6
              and np.array_equal(gpu_matches[i, :M].view(np.uint32).reshape(-1)[: 4 * M],
                                 o["matches"].view(np.uint32).reshape(-1)))
        if not ok:
            bad.append(i)
    return {"pairs_checked": len(ora), "all_equal": not bad, "mismatched_pairs": bad,
            "r1r2_order_swaps": swaps,
            "fields": "status, M, K equal; min_idx equal (or, listed in r1r2_order_swaps, the "
                      "other rotation of the SAME iteration with the same R); R, T within 1e-6; "
                      "matches bit-exact"}


def load_pmc(tag, stage):
    """(HBM bytes per launch of `stage` from profiles/<tag>_pmc_<stage>.json, that path).  A
    missing file is reported loudly (stderr) and in the line (roofline.traffic_missing), never
    as a silent null."""
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_{stage}.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    print(f"bench.py: WARNING: no PMC traffic file {os.path.relpath(path, ROOT)} for the "
          f"dominant kernel '{stage}' (--profile-tag {tag}); roofline.traffic is null",
          file=sys.stderr)
    return None, None


def run_dense(args):
    """configs[3]: one dense N x N exact k=2 + ratio match on one GPU with both methods (bf16
    MFMA filter + exact rescoring vs the LDS-tiled packed-FP32 sweep), HIP-event stage times,
    each against its own roof; the two match lists must be identical."""
    import torch
    from erp_match_eightpoint_test_amd import Context, capi, feature_matcher, synth
    n = args.kpts if args.kpts != 4096 else 16384
    dev = torch.device("cuda:0")
    p = synth.make_pair(args.seed, n_kpts=n)
    q = torch.from_numpy(p["desc_l"]).to(dev)
    t = torch.from_numpy(p["desc_r"]).to(dev)
    methods = {}
    outs = {}
    for name, m in (("mfma", capi.MATCHER_MFMA_FILTER), ("valu", capi.MATCHER_VALU_EXACT)):
        ctx = make_ctx(0)
        fm = feature_matcher(ctx=ctx, method=m)
        for _ in range(args.warmup):
            out = fm._match_device(q, t, 0.3)
        torch.cuda.synchronize()
        ctx.set_profiling(True)
        ctx.stage_times()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = fm._match_device(q, t, 0.3)  # (reads the match count: one sync per call)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.steps
        st = {k: v[0] / args.steps for k, v in ctx.stage_times().items() if v[1] > 0}
        ctx.set_profiling(False)
        outs[name] = out.cpu().numpy()
        if name == "mfma":
            kern = st.get("knn2_filter", 0)
            work = 2.0 * n * n * 64  # ONE bf16 MFMA pass: 2 N T 64 flops
            roof = {"bound": "mfma", "kernels": "knn2_filter", "peak": PEAK_BF16_MFMA,
                    "unit": "TFLOP/s", "achieved": work / (kern / 1e3) / 1e12}
        else:
            kern = st.get("knn2_exact", 0)
            work = 3.0 * n * n * 64  # sub, mul, add per element (flann::L2 order, no FMA)
            roof = {"bound": "valu", "kernels": "knn2_exact", "peak": PEAK_FP32_VALU_UNFUSED,
                    "unit": "Top/s", "achieved": work / (kern / 1e3) / 1e12}
        roof["frac"] = roof["achieved"] / roof["peak"]
        methods[name] = {"ms_per_match": el * 1e3, "stages_ms": st, "roofline": roof,
                         "M": int(outs[name].shape[0])}
    same = outs["mfma"].shape == outs["valu"].shape and np.array_equal(outs["mfma"], outs["valu"])
    best = min(methods, key=lambda k: methods[k]["ms_per_match"])
    line = {"metric": f"dense {n}x{n} exact k=2 + ratio match (configs[3]); match-set bit-exact",
            "value": 1e3 / methods[best]["ms_per_match"], "unit": "matches/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": methods[best]["ms_per_match"], "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": "f32 (bf16 MFMA filter)",
            "data": "synthetic (seeded SURF-like descriptors, synth.make_pair)",
            "config": {"workload": f"configs[3]: one pair, {n} x {n} 64-D descriptors",
                       "kpts": n, "faster": best},
            "methods": methods, "check": {"identical_matches": bool(same)}}
    print(json.dumps(line))


def run_manual(args):
    """configs[4]: ONE find() with I = 100k initial_guess iterations on the manual-pickup regime
    (100 integer-pixel correspondences on 2048 x 1024, 60 % outliers), its iterations split into
    contiguous hypothesis blocks over the ranks (glibc jump-ahead per block), records
    all-gathered over RCCL, consensus on the merged list (strong scaling: the work is fixed)."""
    import torch
    from erp_match_eightpoint_test_amd import Context, dist as D, results_to_numpy, synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    iters = args.iters if args.iters != 10000 else 100000
    c = synth.make_correspondences(args.seed, m=100, outlier_frac=0.6)
    kl = torch.from_numpy(c["kp_l"]).to(dev)
    kr = torch.from_numpy(c["kp_r"]).to(dev)
    ctx = make_ctx(local)

    def step():
        return D.find_hypothesis_sharded_dev(ctx, c["W"], c["H"], kl, kr, 100, iters,
                                             shard_consensus=not args.no_shard_consensus)[0]

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    ctx.set_profiling(True)
    ctx.stage_times()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = {k: v[0] / args.steps for k, v in ctx.stage_times().items() if v[1] > 0}
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    r = results_to_numpy(res.view(1, -1))[0]
    emu = {}
    if world == 1 and not args.no_shard_consensus:
        # the row-sharded consensus of an N-rank run, every shard on this GPU in turn (outside
        # the timed region): the bounds stage per shard ~ one rank's share of it at N ranks
        for nsh in (2, 8):
            D.find_hypothesis_sharded_dev(ctx, c["W"], c["H"], kl, kr, 100, iters, emulate_world=nsh)
            torch.cuda.synchronize()
            ctx.stage_times()
            res_e = D.find_hypothesis_sharded_dev(ctx, c["W"], c["H"], kl, kr, 100, iters,
                                                  emulate_world=nsh)[0]
            torch.cuda.synchronize()
            se = {k: v[0] for k, v in ctx.stage_times().items() if v[1] > 0}
            re_ = results_to_numpy(res_e.view(1, -1))[0]
            emu[f"shards{nsh}"] = {
                "bounds_ms_per_shard": se.get("consensus_bounds", 0.0) / nsh,
                "stages_ms_all_shards": se,
                "same_winner": bool(re_["min_idx"] == r["min_idx"] and
                                    np.array_equal(re_["R"], r["R"]))}
    if rank == 0:
        # the unsharded find() on this GPU must give the same winner (outside the timed region)
        from erp_match_eightpoint_test_amd import eight_point
        ep = eight_point(ctx=make_ctx(local), iters=iters)
        R1, T1 = ep.find(c["W"], c["H"], c["kp_l"], c["kp_r"])
        line = {"metric": f"find() calls/sec, {iters // 1000}k-iteration RANSAC on 100 manual-pickup "
                          "correspondences (60% outliers), hypothesis blocks sharded (configs[4])",
                "value": args.steps / elapsed, "unit": "finds/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64+f32",
                "data": "synthetic (synth.make_correspondences, seeded)",
                "config": {"workload": "configs[4]", "iters": iters, "m": 100,
                           "parallelism": f"hypothesis blocks x{world}",
                           "iterations_per_s": iters * args.steps / elapsed},
                "stages_ms_rank0": st,
                "row_shard_emulation": emu,
                "check": {"status": int(r["status"]), "K": int(r["K"]),
                          "min_idx": int(r["min_idx"]), "survivors": int(r["survivors"]),
                          "same_as_unsharded": bool(np.array_equal(r["R"], R1) and
                                                    np.array_equal(r["T"], T1))}}
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def run_remap(args):
    """section 8f: do_all's band remap (4 bands of each image: crop_rotated_image at 45 / -45 /
    -90 degrees + the unrotated band) and rectify (two full-image rotate_image) on 5376 x 2688
    CV_8UC3 images resident in HBM.  Roofline: HBM at 6 algorithmic bytes per output pixel
    (3-byte gather + 3-byte store), reported beside the FP64 VALU work (acos + atan2 per pixel)."""
    import torch
    from erp_match_eightpoint_test_amd import Context, erp_rotation, spherical_surf
    dev = torch.device("cuda:0")
    H, W, B = 2688, 5376, 16
    g = torch.Generator(device="cpu").manual_seed(args.seed)
    ims = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g).to(dev)
    ctx = make_ctx(0)
    ss, er = spherical_surf(ctx=ctx), erp_rotation(ctx=ctx)
    bands = torch.zeros((B, 4, H // 4, W, 3), dtype=torch.uint8, device=dev)
    L = ctx.L
    st = torch.cuda.current_stream().cuda_stream
    rv = np.array([0.05, -0.12, 0.03])
    tv = np.array([0.6, 0.1, -0.79])
    tv /= np.linalg.norm(tv)
    outs = [torch.zeros_like(ims[0]) for _ in range(2)]

    def do_bands():
        L.erp_spherical_bands_dev(ctx.h, ims.data_ptr(), B, W, H, bands.data_ptr(), st)

    def do_rectify():
        for i in range(0, B, 2):
            er.L.erp_rectify_dev(ctx.h, ims[i].data_ptr(), ims[i + 1].data_ptr(), W, H,
                                 rv.ctypes.data, tv.ctypes.data, outs[0].data_ptr(),
                                 outs[1].data_ptr(), st)

    res = {}
    for name, fn, px in (("bands", do_bands, B * 3 * (H // 4) * W),
                         ("rectify", do_rectify, B * H * W)):
        for _ in range(args.warmup):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        gbs = px * 6 / (ms / 1e3) / 1e9
        res[name] = {"ms_per_batch": ms, "images_per_s": B / (ms / 1e3),
                     "remapped_pixels_per_s": px / (ms / 1e3),
                     "roofline": {"bound": "hbm (algorithmic) / fp64 valu (actual)",
                                  "achieved": gbs, "peak": PEAK_HBM, "unit": "GB/s",
                                  "frac": gbs / PEAK_HBM, "bytes_per_pixel": 6}}
    line = {"metric": "ERP band remap + rectification, 5376x2688 images/s (section 8f)",
            "value": res["bands"]["images_per_s"], "unit": "images/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["bands"]["ms_per_batch"],
            "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8+f64",
            "data": "synthetic random CV_8UC3 images", "config": {"workload": "section 8f",
                                                                "images_per_batch": B},
            "stages": res}
    print(json.dumps(line))


def run_e2e(args):
    """automatic.cpp:117-126 per pair from the images: spherical_surf::do_all (4 bands per
    image, SURF on the 8 bands, un-rotation, concat, match, gather) then eight_point::find with
    --iters iterations, on synthetic 5376 x 2688 BGR ERP pairs (a blob texture rendered on the
    sphere; the right image = rotate_image of the left by a known small rotation).  Stage
    times from HIP events around each stage (torch's stream)."""
    import torch
    from erp_match_eightpoint_test_amd import (Context, eight_point, erp_rotation, feature_matcher,
                                                spherical_surf, synth)
    dev = torch.device("cuda:0")
    H, W, B = 2688, 5376, 4
    rng = np.random.default_rng(args.seed)
    ctx = make_ctx(0)
    ss, er, fm = spherical_surf(ctx=ctx), erp_rotation(ctx=ctx), feature_matcher(ctx=ctx)
    ep = eight_point(ctx=ctx, iters=args.iters)
    lefts, rights = [], []
    for b in range(B):
        lo = synth.sphere_texture(args.seed + b, H // 4, W // 4)
        t = torch.from_numpy(lo).to(dev).permute(2, 0, 1)[None].float()
        up = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)
        up = (up + torch.randn(up.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(b)) * 3)
        left = up.clamp(0, 255).round().to(torch.uint8)[0].permute(1, 2, 0).contiguous()
        R = er.eular2rot(np.radians(rng.uniform(0, 15, 3)))
        lefts.append(left)
        rights.append(er.rotate_image(left, er.inv(R)))
    torch.cuda.synchronize()

    def one(b):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        kl, kr, M, total = ss.do_all(lefts[b], rights[b])
        ev[1].record()
        R, T = ep.find(W, H, kl.cpu().numpy(), kr.cpu().numpy())
        ev[2].record()
        return ev, M, total

    for b in range(min(args.warmup, B)):
        one(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    recs = []
    for s_ in range(args.steps):
        recs.append(one(s_ % B))
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    do_ms = float(np.mean([e[0].elapsed_time(e[1]) for e, _, _ in recs]))
    find_ms = float(np.mean([e[1].elapsed_time(e[2]) for e, _, _ in recs]))
    # SURF alone on the 8 bands of one pair (device time)
    bands = ss.bands(torch.stack([lefts[0], rights[0]])).reshape(8, H // 4, W, 3)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fm.surf_dev(bands)
    e0.record()
    for _ in range(3):
        fm.surf_dev(bands)
    e1.record()
    torch.cuda.synchronize()
    line = {"metric": "ERP image pairs/sec through the whole reference pipeline (do_all + find), "
                      "5376x2688 images", "value": 1.0 / el, "unit": "pairs/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3,
            "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8+f32+f64",
            "data": "synthetic ERP images (sphere blob texture, known rotation)",
            "config": {"workload": "e2e, one pair per step", "iters": args.iters},
            "stages_ms": {"do_all (bands + SURF x 8 + concat + match + gather)": do_ms,
                          "find": find_ms, "surf_8_bands_device": e0.elapsed_time(e1) / 3},
            "check": {"M": [int(r[1]) for r in recs], "total_key_num": [int(r[2]) for r in recs]}}
    print(json.dumps(line))


def _launch_ranks(args) -> int:
    """--gpus N > 1 without a torch.distributed launcher: start N ranks (one process per GPU)
    via torch.distributed.run as a CHILD process -- before anything here touches the GPU -- and
    return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr)
    return subprocess.call(cmd)


def check_world(args) -> int:
    """the world size this process runs in; fails loudly when it disagrees with --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch with "
                         f"torch.distributed.run --nproc-per-node {args.gpus} (or without a "
                         "launcher and let bench.py start the ranks)")
    return world


def main():
    args = parse()
    global SAMPLER
    SAMPLER = 1 if args.sampler == "philox" else 0
    for kv in args.ctx_option:
        k, v = kv.split("=", 1)
        CTX_OPTIONS[k] = int(v)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args))
    check_world(args)
    if args.gpus > 1 and args.workload in ("dense", "remap", "e2e"):
        raise SystemExit(f"bench.py: workload {args.workload} is single-GPU (--gpus 1)")
    import torch
    if args.ranks_on_device >= 0 and args.dist_backend != "gloo":
        raise SystemExit("bench.py: --ranks-on-device needs --dist-backend gloo (RCCL refuses "
                         "two ranks on one GPU)")
    need = args.ranks_on_device + 1 if args.ranks_on_device >= 0 else args.gpus
    if torch.cuda.device_count() < need:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} "
                         "HIP device(s) visible")
    if args.workload == "dense":
        return run_dense(args)
    if args.workload == "manual":
        return run_manual(args)
    if args.workload == "remap":
        return run_remap(args)
    if args.workload == "e2e":
        return run_e2e(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.ranks_on_device >= 0:
        local = args.ranks_on_device
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
        world = dist.get_world_size()  # the world actually formed
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy
    from erp_match_eightpoint_test_amd import dist as D
    if args.main_batch == "worst":
        pairs = make_worst_batch(rank, args.pairs, args.kpts, args.sigma)
    else:
        pairs = make_batch(rank, args.pairs, args.kpts, args.seed, args.inlier_frac, args.sigma)
    S = max(1, min(args.streams, args.pairs))
    parts = [pairs[i * args.pairs // S:(i + 1) * args.pairs // S] for i in range(S)]
    subs = []
    for part in parts:  # one context (scratch) and one HIP stream per sub-batch
        b = to_device(part, dev)
        ctx = make_ctx(local)
        ctx.set_matcher(0 if args.matcher == "mfma" else 1)
        runner = PairBatchRunner(ctx=ctx, iters=args.iters, sampler=SAMPLER)
        runner.reserve(len(part), b["max_nq"], b["max_nt"])
        subs.append(dict(b=b, ctx=ctx, runner=runner, stream=torch.cuda.Stream(dev),
                         res=torch.empty((len(part), 64), dtype=torch.uint8, device=dev)))

    coll_dev = torch.device("cpu") if args.dist_backend == "gloo" else dev

    def gather(o):  # the records' all-gather (host copies under gloo)
        return D.gather_records(o.to(coll_dev))

    def call(batch=None):
        for i, sb in enumerate(subs):
            b = sb["b"] if batch is None else batch[i]
            with torch.cuda.stream(sb["stream"]):
                out = sb["runner"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                                       b["off_r"], b["width"], b["height"], b["max_nq"],
                                       b["max_nt"], stream=sb["stream"].cuda_stream)
                sb["res"].copy_(out["results"])
        for sb in subs:
            torch.cuda.current_stream(dev).wait_stream(sb["stream"])
        return torch.cat([sb["res"] for sb in subs])

    gathered = None
    def call_serial():  # the sub-batches one after the other (no stream overlap)
        for sb in subs:
            b = sb["b"]
            with torch.cuda.stream(sb["stream"]):
                o = sb["runner"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                                     b["off_r"], b["width"], b["height"], b["max_nq"],
                                     b["max_nt"], stream=sb["stream"].cuda_stream)
                sb["res"].copy_(o["results"])
            sb["stream"].synchronize()

    for _ in range(args.warmup):
        if args.steps == 0:  # profile-only run: keep every launch standalone
            call_serial()
            continue
        out = call()
        if dist is not None:
            gathered = gather(out)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = call()
        if dist is not None:
            gathered = gather(out)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    timed_out = out  # the last timed step's records (torch.cat: a tensor of its own)
    # per-kernel durations: one more step AFTER the timed region, its sub-batches run one after
    # the other with HIP events around every kernel (standalone kernel times; inside the timed
    # region the sub-batches overlap, so events there would also count queueing behind the
    # other streams).  stages[k] = (total ms, launches) over the whole step.
    stages = {}
    for sb in subs:
        sb["ctx"].set_profiling(True)
        sb["ctx"].stage_times()  # clear
    call_serial()
    for sb in subs:
        for k, (ms, n) in sb["ctx"].stage_times().items():
            a = stages.get(k, (0.0, 0))
            stages[k] = (a[0] + ms, a[1] + n)
        sb["ctx"].set_profiling(False)
    elapsed = t1 - t0
    serial_out = torch.cat([sb["res"] for sb in subs])  # the serial pass recomputed the step
    out = timed_out if timed_out is not None else serial_out
    timed_identical = (None if timed_out is None else
                       bool(torch.equal(timed_out.cpu(), serial_out.cpu())))
    # the same comparison on the result fields only (binned_rows / survivors are work counts):
    # the pairs whose answer under 6-stream overlap differs from the serial pass's (DESIGN.md
    # 5c item 2: ~2e-4 of overlapped records in round 4's measurement)
    timed_result_diff = None
    if timed_out is not None:
        a = results_to_numpy(timed_out).reshape(-1)
        c = results_to_numpy(serial_out).reshape(-1)
        bad = np.zeros(len(a), bool)
        for f in a.dtype.names:
            if f not in ("binned_rows", "survivors"):
                bad |= np.any((a[f] != c[f]).reshape(len(a), -1), axis=1)
        timed_result_diff = np.nonzero(bad)[0].tolist()
    ranks_timed = None
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # every rank's timed-vs-serial comparison, not only rank 0's: [ranks whose timed
        # records differ from their serial pass, ranks whose RESULT fields differ, total pairs
        # whose result fields differ]
        flags = torch.tensor([0 if timed_identical is not False else 1,
                              1 if timed_result_diff else 0,
                              len(timed_result_diff or [])], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(flags, op=dist.ReduceOp.SUM)
        f = [int(x) for x in flags.tolist()]
        ranks_timed = {"ranks": world, "ranks_records_differ": f[0],
                       "ranks_result_fields_differ": f[1], "pairs_result_fields_differ": f[2],
                       "timed_records_identical": f[0] == 0}
    res = results_to_numpy(out)
    ok = bool(np.all(res["status"] == 0))
    err_deg = [float(np.degrees(np.abs(r["R"] - p["euler_gt"])).mean()) for r, p in zip(res, pairs)]
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    total_pairs = world * args.pairs * args.steps
    # --steps 0: profile-only run (the serial profile pass alone, e.g. under rocprofv3)
    value = total_pairs / elapsed if args.steps > 0 else None
    # dominant kernel roofline from the live HIP-event stage times
    dom = max((k for k in stages if stages[k][1] > 0), key=lambda k: stages[k][0])
    roof = None
    w = stage_work(dom, args.pairs, args.kpts, args.iters, res)
    if w is not None:
        amount, unit, peak, bound, note = w
        amount /= stages[dom][1]  # the step's work over its launches (one per sub-batch)
        avg_s = stages[dom][0] / stages[dom][1] / 1e3
        achieved = amount / avg_s / 1e12
        traffic, tsrc = load_pmc(args.profile_tag, dom)
        roof = {"bound": bound, "kernel": dom, "achieved": achieved, "peak": peak, "unit": unit,
                "frac": achieved / peak, "traffic": traffic,
                "traffic_source": tsrc if tsrc else None,
                "avg_launch_ms": avg_s * 1e3, "work_per_launch": amount, "work_note": note,
                "launch_pairs": args.pairs // S}
        if tsrc is None:
            roof["traffic_missing"] = f"profiles/{args.profile_tag}_pmc_{dom}.json"
        if peak == PEAK_VALU_OPS:
            roof["frac_vs_4cycle_issue"] = achieved / PEAK_VALU_OPS_4CYC
        sol = os.path.join(ROOT, "profiles", "r06b_sampler_sol.json")
        if dom == "sampler" and SAMPLER == 0 and os.path.exists(sol):
            # the measured floor of the same replay (scripts/dev/sampler_sol.hip: the backwards
            # ring + magic modulo alone, same launch shape), same-box run
            with open(sol) as f:
                so = json.load(f)
            v = so["variants"]
            roof["speed_of_light_probe"] = {
                "source": os.path.relpath(sol, ROOT),
                "generator_ms": v["V0"]["ms"], "generator_modulo_ms": v["V1"]["ms"],
                "plus_bitmap_bookkeeping_ms": v["V2"]["ms"],
                "sampler_kernel_ms_same_box": so["real_sampler_kernel_ms"],
                "sampler_over_generator_modulo": so["real_over_floor_V1"]}
    stage_roofs = {}
    for k in stages:
        w = stage_work(k, args.pairs, args.kpts, args.iters, res)
        if w is None or stages[k][1] == 0:
            continue
        amount, unit, peak, bound, note = w
        amount /= stages[k][1]
        avg_s = stages[k][0] / stages[k][1] / 1e3
        stage_roofs[k] = {"bound": bound, "achieved": amount / avg_s / 1e12, "peak": peak,
                          "unit": unit, "frac": amount / avg_s / 1e12 / peak,
                          "avg_launch_ms": avg_s * 1e3}
    # latency of ONE pair alone through the same pipeline (the reference's per-pair use,
    # src/automatic.cpp:117-126): a batch of 1, median of 20 synchronous runs (not `value`)
    lat = None
    if args.steps > 0:
        b1 = to_device(pairs[:1], dev)

        def lat_run(graphs: bool) -> tuple:
            ctx1 = make_ctx(local)
            ctx1.set_matcher(0 if args.matcher == "mfma" else 1)
            ctx1.set_graphs(graphs)  # erp_ctx_set_graphs: replay the captured launch sequence
            run1 = PairBatchRunner(ctx=ctx1, iters=args.iters, sampler=SAMPLER,
                                   reuse_outputs=graphs)
            run1.reserve(1, b1["max_nq"], b1["max_nt"])
            st1 = torch.cuda.Stream(dev) if graphs else None  # (capture needs a non-NULL stream)
            ts, rec = [], None
            for k in range(23):
                torch.cuda.synchronize()
                ta = time.perf_counter()
                o = run1.run(b1["desc_l"], b1["desc_r"], b1["kp_l"], b1["kp_r"], b1["off_l"],
                             b1["off_r"], b1["width"], b1["height"], b1["max_nq"], b1["max_nt"],
                             stream=st1.cuda_stream if st1 is not None else None)
                torch.cuda.synchronize()
                if k >= 3:
                    ts.append(time.perf_counter() - ta)
                rec = o["results"].cpu().numpy().tobytes()
            return float(np.median(ts)) * 1e3, rec

        eager_ms, eager_rec = lat_run(False)
        graph_ms, graph_rec = lat_run(True)
        lat = {"single_pair_ms": min(eager_ms, graph_ms),
               "single_pair_ms_eager": eager_ms, "single_pair_ms_graph": graph_ms,
               "graph_record_equals_eager": graph_rec == eager_rec,
               "note": f"one {args.kpts}x{args.kpts} pair, {args.iters} iterations, batch of 1, "
                       "host-timed (sync before and after each call), median of 20; eager = "
                       "launches enqueued per call, graph = the context's captured HIP graph "
                       "replayed (erp_ctx_set_graphs); single_pair_ms = the faster of the two"}
    # a harder batch through the same contexts and streams (beside the headline, not `value`):
    # half the left keypoints without a true partner, more descriptor noise (0.035: much more
    # and the 0.3 ratio test rejects the true partners too), 30 % of the true matches at wrong
    # positions (outliers the consensus must reject)
    hard = None
    if args.steps > 0 and args.hard_steps > 0:
        hpairs = make_batch(rank, args.pairs, args.kpts, args.seed + 7777, 0.5, 0.035, 0.3)
        hparts = [hpairs[i * args.pairs // S:(i + 1) * args.pairs // S] for i in range(S)]
        hb = [to_device(part, dev) for part in hparts]
        for sb, b in zip(subs, hb):
            sb["runner"].reserve(len(b["width"]), b["max_nq"], b["max_nt"])
        call(hb)
        torch.cuda.synchronize()
        th0 = time.perf_counter()
        for _ in range(args.hard_steps):
            hout = call(hb)
        torch.cuda.synchronize()
        th = (time.perf_counter() - th0) / args.hard_steps
        hres = results_to_numpy(hout)
        hard = {"value": args.pairs / th, "unit": "pairs/s", "ms_per_step": th * 1e3,
                "steps": args.hard_steps, "inlier_frac": 0.5, "sigma": 0.035,
                "mismatch_frac": 0.3,
                "mean_abs_euler_err_deg_max": max(
                    float(np.degrees(np.abs(r["R"] - p["euler_gt"])).mean())
                    for r, p in zip(hres, hpairs)),
                "all_status_ok": bool(np.all(hres["status"] == 0)),
                "M_mean": float(hres["M"].mean()), "K_mean": float(hres["K"].mean()),
                "survivors_mean": float(hres["survivors"].mean()),
                "survivors_max": int(hres["survivors"].max()),
                "binned_rows_mean": float(hres["binned_rows"].mean())}
        if world == 1 and not args.no_cpu_baseline:
            # the harder regime against the oracle too: the first pairs of the hard batch
            # (30 % wrong matches exercise a different consensus regime), matches out
            threads, _ = host_cpu_share()
            n_h = 3
            ora_h = [oracle_pair(p, args.iters, threads) for p in hpairs[:n_h]]
            sb = subs[0]
            b = hb[0]
            o = sb["runner"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                                 b["off_r"], b["width"], b["height"], b["max_nq"], b["max_nt"],
                                 want=("matches",))
            torch.cuda.synchronize()
            hard["parity"] = parity_check(hres, o["matches"][:n_h].cpu().numpy(), ora_h)
    # the worst case beside it: every pair a two-cluster consensus pair (the pose makes R1 and
    # R2 both valid, src/eight_point.cpp:71-85: K ~ 2 x iters, every trimmed mean within ~1 % of
    # the minimum) at inlier fraction 0.98 (M ~ 4k: the most sampler / Gram work per pair)
    worst = None
    if args.steps > 0 and args.worst_steps > 0:
        wpairs = make_worst_batch(rank, args.pairs, args.kpts, args.sigma)
        wparts = [wpairs[i * args.pairs // S:(i + 1) * args.pairs // S] for i in range(S)]
        wb = [to_device(part, dev) for part in wparts]
        for sb, b in zip(subs, wb):
            sb["runner"].reserve(len(b["width"]), b["max_nq"], b["max_nt"])
        call(wb)
        torch.cuda.synchronize()
        tw0 = time.perf_counter()
        for _ in range(args.worst_steps):
            wout = call(wb)
        torch.cuda.synchronize()
        tw = (time.perf_counter() - tw0) / args.worst_steps
        wres = results_to_numpy(wout)
        worst = {"value": args.pairs / tw, "unit": "pairs/s", "ms_per_step": tw * 1e3,
                 "steps": args.worst_steps, "inlier_frac": 0.98, "sigma": args.sigma,
                 "seeds": "scripts/twin_seeds.json (R1 and R2 both valid)",
                 "all_status_ok": bool(np.all(wres["status"] == 0)),
                 "M_mean": float(wres["M"].mean()), "M_max": int(wres["M"].max()),
                 "K_mean": float(wres["K"].mean()), "K_min": int(wres["K"].min()),
                 "survivors_mean": float(wres["survivors"].mean()),
                 "survivors_max": int(wres["survivors"].max()),
                 "binned_rows_mean": float(wres["binned_rows"].mean())}
        if world == 1 and not args.no_cpu_baseline:
            threads, _ = host_cpu_share()
            n_w = min(3, len(wb[0]["width"]))  # (the first is a two-cluster pair, K = 2 iters)
            ora_w = [oracle_pair(p, args.iters, threads) for p in wpairs[:n_w]]
            sb = subs[0]
            b = wb[0]
            o = sb["runner"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                                 b["off_r"], b["width"], b["height"], b["max_nq"], b["max_nt"],
                                 want=("matches",))
            torch.cuda.synchronize()
            worst["parity"] = parity_check(wres, o["matches"][:n_w].cpu().numpy(), ora_w)
    cpu = None
    parity = None
    multi = None
    if world > 1 and gathered is not None:
        # rank 0's self-check of the timed step's RCCL-gathered records (outside the timed
        # region): the first pair of every rank's block recomputed here alone, byte for byte,
        # and against the oracle (the CPU baseline itself runs at N = 1 only)
        import oracle as O
        O.build()
        threads, _ = host_cpu_share()
        b1cache = {}

        def first_pair(r):
            if r not in b1cache:
                b1cache[r] = make_batch(r, 1, args.kpts, args.seed, args.inlier_frac, args.sigma)[0]
            return b1cache[r]

        # (the pruning route, as the gathered batch took: the small-batch route -- and the
        # automatic pruning options, which a launch of fewer than 8 pairs resolves to off
        # (capi.hip pruning_opts) -- would change the work counts binned_rows / survivors of the
        # record, not its result fields; so the sub-batch's own resolution is set explicitly)
        few = len(parts[0]) < 8  # (each rank's first pair is in its sub-batch 0)
        auto = {"lip2": 0 if few else 1, "lipg": 0 if few else 1, "flat_refs": 0 if few else 25,
                "refine_hint": 0 if few else 1}
        ctx_c = make_ctx(local, small_batch=0,
                         **{k: v for k, v in auto.items() if k not in CTX_OPTIONS})
        ctx_c.set_matcher(0 if args.matcher == "mfma" else 1)
        run_c = PairBatchRunner(ctx=ctx_c, iters=args.iters, sampler=SAMPLER)

        def rerun(r):
            b = to_device([first_pair(r)], dev)
            o = run_c.run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"],
                          b["width"], b["height"], b["max_nq"], b["max_nt"])
            torch.cuda.synchronize()
            return o["results"][0].cpu().numpy()

        def ora(r):
            p = first_pair(r)
            mt, _, _, _ = O.match_two_image(p["desc_l"], p["desc_r"], nthreads=threads)
            o = O.find(p["W"], p["H"], p["kp_l"][mt["queryIdx"]], p["kp_r"][mt["trainIdx"]],
                       O.make_cfg(iters=args.iters, sampler=SAMPLER), detail=True)
            return dict(o, M=len(mt))
        multi = D.check_gathered(gathered.cpu().numpy(), args.pairs, world, rerun, ora)
        multi["gathered_rows"] = int(gathered.shape[0])
        parity = {"pairs_checked": world, "all_equal": bool(multi["records_identical"] and
                                                            multi["oracle_all_equal"]),
                  "fields": "first pair of every rank's block: gathered record byte-identical "
                            "to a rank-0 recomputation; status, M, K, min_idx equal and R, T "
                            "within 1e-6 of the oracle",
                  # every rank's timed step == its own serial pass, all-reduced (all pairs)
                  "timed_records_identical": ranks_timed["timed_records_identical"],
                  "timed_all_ranks": ranks_timed}
        multi["dist_backend"] = args.dist_backend
        multi["ranks_on_device"] = args.ranks_on_device if args.ranks_on_device >= 0 else None
    if world == 1 and not args.no_cpu_baseline:
        # the oracle's pairs: the first pair of every sub-batch, then the second of every
        # sub-batch, ... (every stream of the timed step is checked, not just sub-batch 0)
        starts = [i * args.pairs // S for i in range(S)]
        sizes = [len(p) for p in parts]
        order = [starts[i] + k for k in range(max(sizes)) for i in range(S) if k < sizes[i]]
        cpu, ora = cpu_baseline([pairs[k] for k in order], args.iters, args.cpu_seconds)
        picked = order[:len(ora)]
        # untimed pass of every sub-batch with the match lists out; its records must also equal
        # the timed step's (nothing cached between runs)
        rr, mts = [], []
        for sb in subs:
            b = sb["b"]
            o = sb["runner"].run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"],
                                 b["off_r"], b["width"], b["height"], b["max_nq"], b["max_nt"],
                                 want=("matches",))
            torch.cuda.synchronize()
            rr.append(results_to_numpy(o["results"]))
            mts.append(o["matches"].cpu().numpy())
        rerun = np.concatenate(rr)
        sub_of = np.searchsorted(np.asarray(starts), np.asarray(picked), side="right") - 1
        gm = np.stack([mts[s_][k - starts[s_]] for s_, k in zip(sub_of, picked)])
        parity = parity_check(res[picked], gm, ora)
        parity["pairs"] = [int(k) for k in picked]
        parity["sub_batches_checked"] = sorted({int(x) for x in sub_of})
        parity["rerun_records_identical"] = bool(
            np.array_equal(rerun.view(np.uint8), res.view(np.uint8)))
        # the parity-checked records ARE the timed step's; the serial profile pass after the
        # timed region must reproduce them byte for byte
        parity["timed_records_identical"] = timed_identical
        parity["timed_result_fields_differ_on"] = timed_result_diff
        if timed_result_diff:
            # a timed answer that differs from the serial pass's: which of the two is the
            # oracle's (up to 8 such pairs), and the line is not exact either way
            threads, _ = host_cpu_share()
            sres = results_to_numpy(serial_out)
            judged = []
            for k in timed_result_diff[:8]:
                o_ = oracle_pair(pairs[k], args.iters, threads)
                s_ = int(np.searchsorted(np.asarray(starts), k, side="right") - 1)
                m_ = mts[s_][k - starts[s_]][None]
                judged.append({"pair": int(k),
                               "timed_matches_oracle": parity_check(res[k:k + 1], m_, [o_])["all_equal"],
                               "serial_matches_oracle": parity_check(sres[k:k + 1], m_, [o_])["all_equal"]})
            parity["timed_result_diff_oracle"] = judged
            parity["all_equal"] = False
    line = {
        "metric": "ERP image-pairs/sec (4k x 4k kpts, 10k RANSAC iters); match-set bit-exact",
        "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32+f64",
        "data": "synthetic (seeded SURF-like descriptors + ERP keypoints, synth.make_pair)",
        "config": {"workload": (("configs[1] shape" if args.kpts == 4096 else
                                 "configs[2] shape" if args.kpts == 2048 else "custom shape") +
                                f": {args.kpts}x{args.kpts} kpts/pair, {args.iters} initial_guess "
                                f"iters, batch of {args.pairs} independent pairs per step per GPU"),
                   "kpts": args.kpts, "iters": args.iters, "pairs_per_step_per_gpu": args.pairs,
                   "streams": S, "matcher": args.matcher,
                   "parallelism": f"pair-sharded x{world}", "sampler": ("glibc replay (seed 1)" if SAMPLER == 0
                               else "Philox4x32-10 + Floyd (seed 1; no reference counterpart)"),
                   "rccl_world": world if dist is not None and args.dist_backend == "nccl" else None,
                   "dist_backend": args.dist_backend if dist is not None else None,
                   "ctx_options": CTX_OPTIONS or None,
                   "ranks_on_device": args.ranks_on_device if args.ranks_on_device >= 0 else None,
                   "profile_tag": args.profile_tag,
                   "inlier_frac": args.inlier_frac, "sigma": args.sigma},
        "roofline": roof,
        "roofline_stages": stage_roofs,
        "cpu_baseline": cpu,
        "latency": lat,
        "hard_data": hard,
        "worst_case": worst,
        "stages_ms_serial_step": {k: v[0] for k, v in stages.items()},
        # the streams' overlap: the step's kernels run one after another (HIP events, serial
        # pass) against the timed, 4-stream step
        "overlap": {"kernel_sum_ms": sum(v[0] for v in stages.values()),
                    "step_ms": elapsed / max(args.steps, 1) * 1e3},
        # exact: every parity comparison of the line held and the timed records equal the
        # serial pass's and a re-run's byte for byte (False marks the line non-exact)
        "exact": (None if parity is None else bool(
            parity["all_equal"] and parity.get("timed_records_identical", True) is not False
            and parity.get("rerun_records_identical", True) is not False)),
        "check": {"all_status_ok": ok, "mean_abs_euler_err_deg_max": max(err_deg),
                  "M_mean": float(res["M"].mean()), "K_mean": float(res["K"].mean()),
                  "consensus_survivors": {"mean": float(res["survivors"].mean()),
                                          "max": int(res["survivors"].max()),
                                          "pairs_over_8": np.nonzero(res["survivors"] > 8)[0].tolist()},
                  "near_ties": {"total": int(res["near_ties"].sum()),
                                "pairs": np.nonzero(res["near_ties"])[0].tolist()},
                  "parity": parity,
                  "gathered_records": None if gathered is None else int(gathered.shape[0]),
                  "multi_rank": multi},
    }
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
