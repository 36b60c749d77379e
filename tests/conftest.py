"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu; everything else runs on CPU."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_sessionfinish(session, exitstatus):
    """ERP_PARITY_OUT=<path>: the measured parity deviations of the run (tests/parity_log.py)"""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import parity_log
    parity_log.dump()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def harness():
    """host build of erp_match_eightpoint_test_amd/csrc/erp_device.hpp (tests/host_math)."""
    import ctypes as C
    src = os.path.join(ROOT, "tests", "host_math", "harness.cpp")
    out = os.path.join(ROOT, "tests", "host_math", "libharness.so")
    hdr = os.path.join(ROOT, "erp_match_eightpoint_test_amd", "csrc", "erp_device.hpp")
    if (not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src)
            or os.path.getmtime(out) < os.path.getmtime(hdr)):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                        "-o", out, src], check=True)
    L = C.CDLL(out)
    P = C.c_void_p
    L.erph_estimate.argtypes = [P, P, C.c_int32, C.c_double, P]
    L.erph_gram36.argtypes = [P, P, C.c_int32, P]
    L.erph_svd3.argtypes = [P, P, P, P]
    L.erph_pixel_to_bearing.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, P]
    L.erph_rotate_pixel.argtypes = [C.c_int32, C.c_int32, P, C.c_int32, C.c_int32, P]
    return L


@pytest.fixture(scope="session")
def gpu_lib():
    """the product library on a GPU box (fails loudly if it is not built)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test scheduled but no HIP device is visible")
    from erp_match_eightpoint_test_amd import capi
    return capi.load()
