#!/usr/bin/env python3
"""Real-image fixtures from the reference's own data files (run in the build container, where
/root/reference exists; the GPU box only reads the committed outputs).

  python tests/golden/gen_real.py

* tests/golden/real/left_building.jpg, right_building.jpg: the reference's input pair
  (/root/reference/build/*.jpg, 5376 x 2688, copied byte for byte: data files, not source).
* tests/golden/real/ref_rectified_{left,right}.jpg: the reference's own OUTPUT of the automatic
  pipeline (src/automatic.cpp:117-157, rectify) on that pair at 2048 x 1024
  (/root/reference/build/output_20200423/rectified_*.png), re-encoded as JPEG quality 95 to keep
  the repository small (the test compares geometry -- a residual rotation from matched SURF
  features -- not pixel values).  The pairing output_20200423 <-> *_building.jpg was checked:
  the rectified left image differs from left_building.jpg resized to 2048 x 1024 by 14.0 grey
  levels on average, from left_building2.jpg by 42.8 (output_20200423_2 <-> building2: 10.2 /
  40.7).
* tests/golden/real/ref_rectified_left.png, ref_rectified_left_vertical.png: the reference's
  own rectified left image of that pair and its vertical view (src/automatic.cpp:148-157:
  rotate_image by eular2rot(89.999 deg, 0, 0).inv(), then cv::rotate 90 degrees clockwise),
  copied byte for byte (lossless PNG): the vertical view of the first is the second, pixel for
  pixel, except the pixels the reference never writes (uninitialised memory in its output).
* tests/golden/real/left_building2_2048.jpg, right_building2_2048.jpg: the second pair of the
  reference's data (build/*_building2.jpg, the pair its config_file.ini names), resized to the
  pipeline's 2048 x 1024 (resize_input, config_file.ini) with PIL's bilinear filter and
  stored as JPEG quality 95; ref_rectified_{left,right}_2.jpg: the reference's automatic
  output on that pair (output_20200423_2, re-encoded as JPEG quality 95).
* tests/golden/real/ref_rectified_right.png, ref_rectified_{left,right}_2.png +
  vertical_views.json: the other three rectified outputs (lossless) and their vertical views
  pinned by the sha256 of the decoded BGR bytes (plus the one unwritten pixel's bytes), so all
  four of the reference's vertical views are checked pixel for pixel.
* tests/golden/real/MANIFEST.json: sha256 of every source and output file.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys

from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

REF = "/root/reference/build"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "real")


def sha(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    os.makedirs(OUT, exist_ok=True)
    man = {"sources": {}, "outputs": {}}
    for name in ("left_building.jpg", "right_building.jpg"):
        src = os.path.join(REF, name)
        shutil.copyfile(src, os.path.join(OUT, name))
        man["sources"][name] = sha(src)
    for side in ("left", "right"):
        src = os.path.join(REF, "output_20200423", f"rectified_{side}.png")
        dst = os.path.join(OUT, f"ref_rectified_{side}.jpg")
        Image.open(src).convert("RGB").save(dst, quality=95, subsampling=0)
        man["sources"][f"output_20200423/rectified_{side}.png"] = sha(src)
    for name in ("rectified_left.png", "rectified_left_vertical.png"):
        src = os.path.join(REF, "output_20200423", name)
        shutil.copyfile(src, os.path.join(OUT, "ref_" + name))
        man["sources"]["output_20200423/" + name] = sha(src)
    for side in ("left", "right"):
        src = os.path.join(REF, f"{side}_building2.jpg")
        Image.open(src).convert("RGB").resize((2048, 1024), Image.BILINEAR).save(
            os.path.join(OUT, f"{side}_building2_2048.jpg"), quality=95, subsampling=0)
        man["sources"][f"{side}_building2.jpg"] = sha(src)
        src = os.path.join(REF, "output_20200423_2", f"rectified_{side}.png")
        Image.open(src).convert("RGB").save(os.path.join(OUT, f"ref_rectified_{side}_2.jpg"),
                                            quality=95, subsampling=0)
        man["sources"][f"output_20200423_2/rectified_{side}.png"] = sha(src)
    # the other three vertical views (src/automatic.cpp:148-157): the rectified image as a
    # lossless input, the reference's vertical view pinned by the sha256 of its decoded BGR
    # bytes plus the bytes of the pixels the remap never writes (uninitialised there); the
    # view itself (3 MB each) is not stored
    vert = {}
    for od, suffix in (("output_20200423", ""), ("output_20200423_2", "_2")):
        for side in ("left", "right"):
            src = os.path.join(REF, od, f"rectified_{side}.png")
            name = f"ref_rectified_{side}{suffix}.png"
            if not os.path.exists(os.path.join(OUT, name)):
                shutil.copyfile(src, os.path.join(OUT, name))
            man["sources"][f"{od}/rectified_{side}.png"] = sha(src)
            vsrc = os.path.join(REF, od, f"rectified_{side}_vertical.png")
            man["sources"][f"{od}/rectified_{side}_vertical.png"] = sha(vsrc)
            import numpy as np
            import oracle as O
            O.build()
            im = np.ascontiguousarray(np.asarray(Image.open(src).convert("RGB"))[..., ::-1])
            want = np.ascontiguousarray(np.asarray(Image.open(vsrc).convert("RGB"))[..., ::-1])
            a, b = O.vertical_rotate(im, fill=0), O.vertical_rotate(im, fill=255)
            un = np.argwhere((a != b).any(-1))
            vert[name] = {"reference_file": f"{od}/rectified_{side}_vertical.png",
                          "shape": list(want.shape),
                          "sha256_bgr": hashlib.sha256(want.tobytes()).hexdigest(),
                          "unwritten": [[int(r), int(c), want[r, c].tolist()] for r, c in un]}
    with open(os.path.join(OUT, "vertical_views.json"), "w") as f:
        json.dump(vert, f, indent=1)
    for name in sorted(os.listdir(OUT)):
        if name.endswith(".jpg") or name.endswith(".png") or name == "vertical_views.json":
            man["outputs"][name] = sha(os.path.join(OUT, name))
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(man, f, indent=1)
    print(json.dumps(man, indent=1))


if __name__ == "__main__":
    main()
