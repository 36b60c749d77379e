#!/usr/bin/env python3
"""Time the f4 visual outputs (csrc/viz.hip) at the reference's sizes on one MI355X:
draw_match on 5376 x 2688 and 2048 x 1024 BGR pairs with M matched lines, and draw_epipole on a
1920 x 960 canvas with 7 keys.  HIP events on torch's current stream (the API launches there).

  python scripts/dev/viz_time.py > gpurun_out/viz_time.txt
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from erp_match_eightpoint_test_amd import Context, epipolar_tool, feature_matcher  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ctx = Context(0)
    fm = feature_matcher(ctx=ctx)
    rng = np.random.default_rng(0)
    for W, H, M in ((5376, 2688, 2000), (2048, 1024, 300)):
        a = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda")
        b = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda")
        kl = torch.from_numpy(rng.uniform(0, [W, H], (M, 2)).astype(np.float32)).cuda()
        kr = kl + torch.from_numpy(rng.normal(0, 40, (M, 2)).astype(np.float32)).cuda()
        ms = timed(lambda: fm.draw_match(a, b, kl, kr))
        # algorithmic bytes: 2 x 3 B in + 3 B out per pixel (+ 4 B of line stamps read)
        px = W * H
        print(f"draw_match {W}x{H} M={M}: {ms * 1e3:.1f} us/call, "
              f"{9 * px / ms / 1e6:.0f} GB/s algorithmic (9 B/pixel), "
              f"{13 * px / ms / 1e6:.0f} GB/s with the line stamps")
    W, H, ow, oh = 5376, 2688, 1920, 960
    kl = rng.uniform(0, [W, H], (500, 2)).astype(np.float32)
    kr = rng.uniform(0, [W, H], (500, 2)).astype(np.float32)
    E = np.array([[0, -0.3, 0.1], [0.3, 0, -0.9], [-0.1, 0.9, 0]])
    tool = epipolar_tool(kl, kr, W, H, ow, oh, 7, ctx=ctx)
    ms = timed(lambda: tool.draw_epipole(E))
    print(f"draw_epipole {ow}x{oh} 7 keys: {ms * 1e3:.1f} us/call "
          f"({ow * oh / ms / 1e6:.2f} Gpixel/s; includes the host shuffle of 500 indices)")


if __name__ == "__main__":
    main()
