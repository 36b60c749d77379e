"""Probe (round 5): packed-f32 results (pk_probe_kernel) beside synthetic aggressor kernels of one
instruction class each (scripts/dev/lds_guard.hip aggressor_kernel): which class corrupts them?"""
import ctypes as C
import os

import numpy as np
import torch

torch.cuda.init()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
G = C.CDLL(os.path.join(ROOT, "scripts", "dev", "liblds_guard.so"))
G.pk_probe_launch.argtypes = [C.c_void_p, C.c_int, C.c_longlong, C.c_uint32, C.c_void_p, C.c_int]
G.aggressor_launch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_longlong, C.c_void_p]
out = torch.zeros(16 + 8 * 64, dtype=torch.int32, device="cuda")
dummy = torch.zeros(16, dtype=torch.int32, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
NAMES = {-1: "none", 0: "mfma_i32_32x32x32_i8", 1: "mfma_f32_32x32x16_bf16", 2: "fma_f64",
         3: "mfma_i32_16x16x64_i8", 4: "mfma_f64_16x16x4f64"}
AB = int(os.environ.get("AGG_BLOCKS", "512"))
for kind in [-1, 0, 1, 2, 3, 4]:
    out.zero_()
    torch.cuda.synchronize()
    for r in range(int(os.environ.get("REPS", "5"))):
        if kind >= 0:
            assert G.aggressor_launch(sa.cuda_stream, AB, kind, int(10e-3 * 1e8), dummy.data_ptr()) == 0
        assert G.pk_probe_launch(sb.cuda_stream, 512, int(8e-3 * 1e8), 77 + r, out.data_ptr(), 64) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    print(f"PKSYNTH aggressor {NAMES[kind]}: {int(o[2])} probe workgroups, {int(o[3])} rounds: "
          f"{int(o[0])} packed results unlike scalar", flush=True)
    for r in o[16:16 + 8 * min(int(o[1]), 3)].reshape(-1, 8):
        blk, tid, q, d0, t0s, d1, t1s, dt = (int(x) for x in r)
        print(f"   blk {blk} tid {tid} ref {q}: lo {d0:#010x} vs {t0s:#010x}, hi {d1:#010x} vs {t1s:#010x}", flush=True)

# part 2: golden checksums per instruction class (valu_gold_kernel) beside the aggressors
G.valu_gold_launch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_longlong, C.c_void_p, C.c_void_p]
MODES = {0: "packed f32", 1: "scalar f32", 2: "fp64", 3: "int32", 4: "packed f16"}
NB = 512
gold = torch.zeros(NB * 256 * 2, dtype=torch.int32, device="cuda")
for mode in MODES:
    out.zero_()
    assert G.valu_gold_launch(sb.cuda_stream, NB, mode, 1, 0, gold.data_ptr(), out.data_ptr()) == 0
    torch.cuda.synchronize()
    for kind in [-1, 0, 1]:
        out.zero_()
        torch.cuda.synchronize()
        for r in range(int(os.environ.get("REPS", "5"))):
            if kind >= 0:
                assert G.aggressor_launch(sa.cuda_stream, AB, kind, int(10e-3 * 1e8), dummy.data_ptr()) == 0
            assert G.valu_gold_launch(sb.cuda_stream, NB, mode, 0, int(8e-3 * 1e8), gold.data_ptr(),
                                      out.data_ptr()) == 0
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        print(f"GOLD {MODES[mode]:11s} beside {NAMES[kind]:24s}: "
              f"rounds with a wrong lo checksum {int(o[0])}, hi {int(o[1])} ({int(o[2])} workgroups, {int(o[3])} rounds)",
              flush=True)
