#!/usr/bin/env python3
"""Speed-of-light probe of the glibc-replay sampler (scripts/dev/sampler_sol.hip), on the GPU.

One 128-pair sub-batch of the bench workload (bench.make_batch, configs[1] shape) goes through
the library once with stage timing on: that gives the batch's match counts M and the real
sampler_kernel's time for the launch.  The probe variants then run on the same counts, the same
grid and 10k iterations:
  V0 generator only, V1 generator + modulo (the floor), V2 + the i >= s bookkeeping on every step,
  V3 V2 with constant magic shifts, V4 V3 with the carry-accumulated selection bit.
Prints one JSON line: ms per launch and cycles per wave-draw per SIMD at the measured clock.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC scripts/dev/sampler_sol.hip \
      -o scripts/dev/libs/sol/libsampler_sol.so
  python scripts/dev/sampler_sol.py [--pairs 128] [--reps 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def magic_table(n=65539):
    """m_d | (l_d - 1) << 32 with l_d = ceil(log2 d), m_d = ceil(2^(31 + l_d) / d): the
    library's build_magic_table (kernels.hip), restated"""
    t = np.zeros(n, np.uint64)
    for d in range(2, n):
        l = (d - 1).bit_length()
        m = -(-(1 << (31 + l)) // d)
        assert m < (1 << 32) and m * d - (1 << (31 + l)) <= (1 << l)
        t[d] = m | ((l - 1) << 32)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=os.path.join(ROOT, "scripts", "dev", "libs", "sol",
                                                  "libsampler_sol.so"))
    a = ap.parse_args()
    import torch
    import bench
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy
    dev = torch.device("cuda:0")
    pairs = bench.make_batch(0, a.pairs, 4096, 20200423)
    b = bench.to_device(pairs, dev)
    ctx = Context(0)
    run = PairBatchRunner(ctx=ctx, iters=a.iters)
    run.reserve(a.pairs, b["max_nq"], b["max_nt"])
    args = (b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
            b["height"], b["max_nq"], b["max_nt"])
    run.run(*args)
    torch.cuda.synchronize()
    ctx.set_profiling(True)
    ctx.stage_times()
    real = []
    for _ in range(3):
        o = run.run(*args)
        torch.cuda.synchronize()
        st = ctx.stage_times()
        real.append(st["sampler"][0] / st["sampler"][1])
    M = results_to_numpy(o["results"])["M"].astype(np.int64)
    s = (M * 0.25).astype(np.int64)
    counts = torch.from_numpy(M.astype(np.int32)).to(dev)
    mt = torch.from_numpy(magic_table().view(np.int64)).to(dev)
    nwaves = (a.iters + 63) // 64
    nbw = int((M.max() - 1) // 31 + 2)
    nalloc = int(s.max() >> 5) + 1
    out = torch.empty(a.pairs * nwaves * nbw * 64, dtype=torch.int32, device=dev)
    L = C.CDLL(a.lib)
    L.sol_run.restype = C.c_float
    L.sol_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p,
                          C.c_void_p, C.c_int, C.c_int, C.c_int]
    draws = float(np.sum(M - 1)) * nwaves * 64          # lane-draws per launch (incl. idle lanes)
    wave_draws_per_simd = draws / 64 / 1024
    res = {}
    for v in range(5):
        L.sol_run(v, counts.data_ptr(), a.pairs, a.iters, 0.25, mt.data_ptr(), out.data_ptr(),
                  nbw, nalloc, 2)
        ms = [L.sol_run(v, counts.data_ptr(), a.pairs, a.iters, 0.25, mt.data_ptr(),
                        out.data_ptr(), nbw, nalloc, a.reps) for _ in range(3)]
        if min(ms) < 0:
            raise SystemExit(f"variant {v}: launch failed")
        res[f"V{v}"] = {"ms": min(ms), "ms_all": ms}
    real_ms = min(real)
    clk = 2.4e9
    line = {"probe": "sampler speed of light (scripts/dev/sampler_sol.hip)",
            "pairs": a.pairs, "iters": a.iters, "M_mean": float(M.mean()), "s_mean": float(s.mean()),
            "wave_draws_per_simd": wave_draws_per_simd,
            "real_sampler_kernel_ms": real_ms, "real_all": real,
            "variants": res,
            "cycles_per_wave_draw_at_2.4GHz": {k: v["ms"] * 1e-3 * clk / wave_draws_per_simd
                                               for k, v in res.items()},
            "real_cycles_per_wave_draw_at_2.4GHz": real_ms * 1e-3 * clk / wave_draws_per_simd,
            "real_over_floor_V1": real_ms / res["V1"]["ms"],
            "notes": "V0 generator; V1 generator + magic modulo (floor); V2 + i>=s bookkeeping on "
                     "every step; V3 V2 + constant shifts; V4 V3 + carry-accumulated bits"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
