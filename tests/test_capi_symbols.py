"""The C-ABI library loads without a GPU and exports every symbol include/erp_match.h declares
(no compute calls here)."""
from __future__ import annotations

import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "erp_match.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(erp_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from erp_match_eightpoint_test_amd import _build, capi
    _build.build()
    return capi.load()


def test_every_declared_symbol_exported(lib):
    from erp_match_eightpoint_test_amd import capi
    names = _declared()
    assert len(names) >= 13
    assert sorted(names) == sorted(capi.EXPORTED)
    for n in names:
        assert hasattr(lib, n), n


def test_non_compute_entry_points(lib):
    from erp_match_eightpoint_test_amd import capi
    assert lib.erp_abi_version() == 2
    cfg = capi.RansacCfg()
    lib.erp_ransac_cfg_default(C.byref(cfg))
    assert (cfg.iters, cfg.sample_frac, cfg.trim_lo, cfg.trim_hi, cfg.valid_abs, cfg.seed) == \
        (80, 0.25, 0.2, 0.8, 1.57, 1)
    assert lib.erp_status_string(3) == b"no valid rotation hypothesis"


def test_null_ctx_rejected(lib):
    assert lib.erp_ctx_destroy(None) == 1
    assert lib.erp_match_two_image(None, None, 0, None, 0, 64, None, None) == 1
    assert lib.erp_ctx_set_option(None, 0, 0) == 1
    v = C.c_int32()
    assert lib.erp_ctx_get_option(None, 0, C.byref(v)) == 1


def test_release_library_reads_no_environment():
    """route choices are context options (erp_ctx_set_option), not environment variables: the
    release library imports no getenv / secure_getenv at all (VERDICT r05 "next" 6)"""
    from erp_match_eightpoint_test_amd import _build
    out = os.popen(f"nm -D --undefined-only {_build.LIB_PATH}").read()
    assert "getenv" not in out, [ln for ln in out.splitlines() if "getenv" in ln]


def test_option_names_match_header():
    """capi.OPTIONS mirrors the erp_ctx_option enum of include/erp_match.h"""
    from erp_match_eightpoint_test_amd import capi
    src = open(os.path.join(ROOT, "include", "erp_match.h")).read()
    enum = dict((m.group(1).lower(), int(m.group(2)))
                for m in re.finditer(r"ERP_OPT_([A-Z0-9_]+) = (\d+),", src))
    enum.pop("count", None)
    assert enum == capi.OPTIONS


def test_cpp_class_api_symbols():
    """the C++ class API (include/erp/*.hpp) is compiled into the same library."""
    from erp_match_eightpoint_test_amd import _build
    out = os.popen(f"nm -DC {_build.LIB_PATH}").read()
    for sym in ["erp::feature_matcher::match_two_image", "erp::eight_point::find",
                "erp::eight_point::initial_guess", "erp::eight_point::eight_point_estimation"]:
        assert sym in out, sym


def test_gfx950_code_object():
    from erp_match_eightpoint_test_amd import _build
    data = open(_build.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _device_isa(lib_path, tmp_path):
    """disassembly of the library's gfx950 code object (llvm-objdump --offloading extracts the
    bundles next to its input, so a copy goes to tmp_path first)"""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    src = tmp_path / "lib.so"
    shutil.copy(lib_path, src)
    subprocess.run([objdump, "--offloading", str(src)], check=True, cwd=tmp_path,
                   capture_output=True)
    cos = [p for p in tmp_path.iterdir() if "gfx950" in p.name]
    assert cos, "no gfx950 code object in the library"
    return "".join(subprocess.run([objdump, "-d", "--mcpu=gfx950", str(p)], check=True,
                                  capture_output=True, text=True).stdout for p in cos)


def test_no_packed_fp32_instructions(tmp_path):
    """No kernel of the product uses packed-FP32 VALU instructions: on MI355X their LO half can
    read back stale while other waves of the CU issue int8 / bf16 MFMAs (the
    round-4 overlapped-streams nondeterminism; scripts/dev/pk_synth.py measures it).  The build
    drops the target feature (_build.NO_PACKED_FP32); this guards against a source or flag
    change bringing them back."""
    from erp_match_eightpoint_test_amd import _build
    _build.build()
    isa = _device_isa(_build.LIB_PATH, tmp_path)
    assert "v_mfma_i32_32x32x32_i8" in isa and "v_mfma_f32_32x32x16_bf16" in isa
    packed = sorted(set(re.findall(r"\bv_pk_(?:add|mul|fma|mov)_(?:f32|b32)\b", isa)))
    assert packed == [], packed


@pytest.mark.parametrize("seed,offset,m,n", [(1, 0, 300, 7), (1, 80, 4000, 7), (7, 3, 9, 5),
                                             (1, 0, 1, 1), (1, 0, 20, 0), (3, 12345, 2, 2)])
def test_random_shuffle_prefix_matches_glibc(lib, oracle, seed, offset, m, n):
    """epipolar_tool's constructor choice (src/epipolar_tool.cpp:13-16): host-only entry point,
    against the oracle's glibc rand() + std::random_shuffle (pinned to the real libc)"""
    import numpy as np
    out = np.full(max(n, 1), -1, np.int32)
    assert lib.erp_random_shuffle_prefix(seed, offset, m, n, out.ctypes.data) == 0
    assert (out[:n] == oracle.GlibcRand(seed, offset).random_array(m)[:n]).all()
    assert lib.erp_random_shuffle_prefix(seed, offset, m, m + 1, out.ctypes.data) == 1
