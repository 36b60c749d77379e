"""Build the in-tree gfx950 library (hipcc, no cmake): lib/liberp_match.so.

The library holds the HIP kernels, the C ABI (include/erp_match.h) and the C++ class API
(include/erp/*.hpp).  It is built in-tree so it travels to the GPU box with the repository
snapshot; nothing is installed into site-packages.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB_PATH = os.path.join(LIB_DIR, "liberp_match.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ERP_OFFLOAD_ARCH", "gfx950")

SOURCES = ["kernels.hip", "matcher.hip", "capi.hip", "remap.hip", "remap_api.hip", "surf.hip", "surf_api.hip", "viz.hip",
           "host_api.cpp"]
HEADERS = ["erp_device.hpp", "erp_kernels.hpp", "erp_remap.hpp", "erp_surf.hpp", "erp_launch.hpp"]
PUBLIC_HEADERS = ["erp_match.h", os.path.join("erp", "feature_matcher.hpp"),
                  os.path.join("erp", "eight_point.hpp")]

# -ffp-contract=off: the matcher's flann::L2 order, the ratio test and the consensus
# distances must round exactly like the reference's x86-64 code (no FMA contraction).
# Never add -ffast-math / -fno-hip-fp32-correctly-rounded-divide-sqrt: sqrtf must be
# correctly rounded for bit-exact DMatch.distance.
# No packed-FP32 instructions in any kernel (v_pk_add/mul/fma_f32, v_pk_mov_b32): on MI355X a
# packed-FP32 result read one or two instructions later by another VALU op can come back with
# a stale LO half while other waves on the CU issue int8 / bf16 MFMAs (the Gram and matcher
# kernels of the other streams) -- measured by scripts/dev/pk_synth.py: ~3e7 wrong lo halves
# per 10 ms beside v_mfma_i32_32x32x32_i8, none alone.  That was the
# round-4 overlap nondeterminism.  The device cc1 drops the feature; the host cc1 ignores it
# (its "not a recognized feature" warning is filtered below).
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
            "-Wno-unused-function", f"--offload-arch={ARCH}", *NO_PACKED_FP32]
_HOST_FEATURE_WARNING = "'-packed-fp32-ops' is not a recognized feature for this target"


def _run_filtered(cmd):
    """run a hipcc command, dropping the host cc1's warning about the device-only feature"""
    r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
    err = "".join(line for line in r.stderr.splitlines(True) if _HOST_FEATURE_WARNING not in line)
    if err:
        sys.stderr.write(err)
    if r.returncode != 0:
        raise subprocess.CalledProcessError(r.returncode, cmd)
# per-source extras: the matcher's MFMA accumulators in VGPRs (the filter's bounds read them
# directly; the default AGPR form costs one v_accvgpr_read per element) and no NaN quieting in
# its min trees (finite descriptors; matcher.hip header)
EXTRA_FLAGS = {"matcher.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-honor-nans"]}


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files += [os.path.join(ROOT, "include", h) for h in PUBLIC_HEADERS]
    files.append(os.path.abspath(__file__))
    return files


def up_to_date() -> bool:
    if not os.path.exists(LIB_PATH):
        return False
    t = os.path.getmtime(LIB_PATH)
    return all(os.path.getmtime(f) <= t for f in _inputs() if os.path.exists(f))


def build(force: bool = False, verbose: bool = False, lib_path: str = LIB_PATH,
          src_override: dict | None = None, defines: list | None = None) -> str:
    """src_override / lib_path / defines: development variants (a source file replaced by
    another path, extra -D flags, built into another library; see capi.lib_path's
    ERP_LIB_PATH)."""
    if not force and lib_path == LIB_PATH and up_to_date():
        return LIB_PATH
    lib_dir = os.path.dirname(lib_path)
    os.makedirs(lib_dir, exist_ok=True)
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(lib_dir, os.path.splitext(src)[0] + ".o")
        path = (src_override or {}).get(src, os.path.join(CSRC, src))
        cmds.append([HIPCC, *CXXFLAGS, *EXTRA_FLAGS.get(src, []), *[f"-D{d}" for d in defines or []],
                     "-I", os.path.join(ROOT, "include"),
                     "-I", CSRC, "-c", path, "-o", obj])
        objs.append(obj)
    # one hipcc per source, in parallel (kernels.hip dominates; the rest overlap it)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0") or 0) or os.cpu_count() or 1))
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run_filtered(cmd)
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(run, c) for c in cmds]:
            f.result()
    tmp = lib_path + ".tmp"
    _run_filtered([HIPCC, *CXXFLAGS, "-shared", "-o", tmp, *objs])
    os.replace(tmp, lib_path)
    for o in objs:
        os.remove(o)
    return lib_path


DRIVER_SRC = os.path.join(ROOT, "tests", "cpp", "class_api_driver.cpp")
DRIVER_BIN = os.path.join(ROOT, "tests", "cpp", "class_api_driver")


def build_driver(force: bool = False) -> str:
    """the C++ class-API driver (tests/cpp): host code only, g++ against liberp_match.so -- the
    link a reference maintainer would do."""
    if (not force and os.path.exists(DRIVER_BIN)
            and os.path.getmtime(DRIVER_BIN) >= max(os.path.getmtime(DRIVER_SRC),
                                                    os.path.getmtime(LIB_PATH))):
        return DRIVER_BIN
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), DRIVER_SRC,
                    "-o", DRIVER_BIN, "-L", LIB_DIR, "-lerp_match", f"-Wl,-rpath,{LIB_DIR}",
                    "-Wl,-rpath,$ORIGIN/../../erp_match_eightpoint_test_amd/lib",
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return DRIVER_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
