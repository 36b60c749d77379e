"""SURF timing probe: 8 bands (672 x 5376) of a synthetic ERP pair through fm.surf."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
from erp_match_eightpoint_test_amd import Context, feature_matcher, spherical_surf, synth
ctx = Context(0)
fm, ss = feature_matcher(ctx=ctx), spherical_surf(ctx=ctx)
H, W = 2688, 5376
lo = synth.sphere_texture(1, H // 4, W // 4)
t = torch.from_numpy(lo).cuda().permute(2, 0, 1)[None].float()
up = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear").clamp(0, 255).round().to(torch.uint8)[0].permute(1, 2, 0).contiguous()
bands = ss.bands(torch.stack([up, up])).reshape(8, H // 4, W, 3)
for _ in range(3):
    torch.cuda.synchronize(); t0 = time.time(); k, d = fm.surf(bands, max_kp=int(sys.argv[1]) if len(sys.argv) > 1 else 4096); torch.cuda.synchronize()
    print("surf 8 bands", time.time() - t0, [len(x) for x in k])
