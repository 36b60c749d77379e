"""The oracle against the reference's own outputs (no GPU): the vertical view.

The reference's automatic pipeline writes rectified_left.png and its vertical view
rectified_left_vertical.png (src/automatic.cpp:148-157: rotate_image by
eular2rot(89.999 deg, 0, 0).inv(), then cv::rotate 90 degrees clockwise).  Both are committed
byte for byte under tests/golden/real/ (tests/golden/gen_real.py), so the restated remap
(oracle/erp_oracle.c erpo_vertical_rotate) is pinned to the reference binary's output: every
pixel it writes must equal the reference's, and the pixels it leaves unwritten (source outside
the image; the reference leaves them uninitialised, so their bytes are whatever its Mat held)
are identified by running it with two fill values.  Measured: 1 unwritten pixel of 2 097 152,
every other pixel equal.  (tests/test_gpu_real.py runs the device path the same way.)
"""
from __future__ import annotations

import os

import numpy as np
import pytest

REAL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "real")


def _bgr(name):
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(os.path.join(REAL, name)).convert("RGB"))[..., ::-1])


def test_oracle_vertical_view_equals_reference_output(oracle):
    src = _bgr("ref_rectified_left.png")
    want = _bgr("ref_rectified_left_vertical.png")
    assert src.shape == (1024, 2048, 3) and want.shape == (2048, 1024, 3)
    a = oracle.vertical_rotate(src, fill=0)
    b = oracle.vertical_rotate(src, fill=255)
    unwritten = (a != b).any(-1)
    assert int(unwritten.sum()) <= 4, int(unwritten.sum())
    assert np.array_equal(a[~unwritten], want[~unwritten])


@pytest.mark.parametrize("name", ["ref_rectified_left.png", "ref_rectified_right.png",
                                  "ref_rectified_left_2.png", "ref_rectified_right_2.png"])
def test_oracle_vertical_views_all_four(oracle, name):
    """all four of the reference's vertical views (both building pairs, left and right): the
    oracle's view of the reference's rectified image, with the remap's unwritten pixels taken
    from the reference, has the sha256 of the reference's own decoded vertical view
    (tests/golden/real/vertical_views.json, tests/golden/gen_real.py)"""
    import hashlib
    import json
    meta = json.load(open(os.path.join(REAL, "vertical_views.json")))[name]
    src = _bgr(name)
    a = oracle.vertical_rotate(src, fill=0)
    b = oracle.vertical_rotate(src, fill=255)
    un = np.argwhere((a != b).any(-1))
    assert [[int(r), int(c)] for r, c in un] == [u[:2] for u in meta["unwritten"]]
    for r, c, v in meta["unwritten"]:
        a[r, c] = v
    assert list(a.shape) == meta["shape"]
    assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == meta["sha256_bgr"]
