"""Builds librt_amd.so (HIP kernels for gfx950 + the C ABI) in-tree.

Plain hipcc invocations, no cmake: every source is compiled for
--offload-arch=gfx950. The ref-precision kernel TU is compiled with
-ffp-contract=off so no multiply-add is fused (the reference's JS arithmetic
never fuses); the fp32 fast-mode TU may fuse.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR.parent / "csrc"
INCLUDE = PKG_DIR.parent.parent / "include"
LIB_DIR = PKG_DIR / "lib"
LIB_PATH = LIB_DIR / "librt_amd.so"
OBJ_DIR = PKG_DIR.parent / "build"

ARCH = "gfx950"

_COMMON = ["-std=c++17", "-O3", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
           f"-I{CSRC}", f"-I{INCLUDE}"]

# (source, extra flags, is_hip)
# -fno-slp-vectorize on the kernel units: the SLP vectoriser packs pairs of fp32
# ray/box operations into v_pk_* instructions, which need their operands in
# register pairs of every pairing used and so keep several copies of the ray
# live through the traversal loops. Without it the Cornell chunk kernel drops
# from 128 VGPRs + 8 spilled (scratch reloads inside the pre-filter loop) to
# 111 VGPRs and no spills: Cornell 7071 -> 7647, spheres-500 4878 -> 5096,
# rain 19821 -> 20212 Msamples/s (profiles/r01/noslp/).
_KERNEL_FLAGS = ["-fno-slp-vectorize"]
_UNITS = [
    ("pt_ref.hip", ["-ffp-contract=off", *_KERNEL_FLAGS], True),
    ("pt_fp32.hip", ["-ffp-contract=fast", *_KERNEL_FLAGS], True),
    ("rt_api.cpp", ["-ffp-contract=off", "-x", "hip"], True),
    ("scene.cpp", ["-ffp-contract=off"], False),
]
_HEADERS = ["json.hpp", "rt_math.hpp", "scene.hpp", "pt_kernel.hpp", "launch.hpp"]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build librt_amd.so")


def _newest_input() -> float:
    paths = [CSRC / u[0] for u in _UNITS] + [CSRC / h for h in _HEADERS] + [INCLUDE / "rt_amd.h", Path(__file__)]
    return max(p.stat().st_mtime for p in paths)


def build_native(force: bool = False, verbose: bool = False, variant: str = "", defines=(), flags=()) -> Path:
    """Compile (if stale) and return the path of librt_amd.so. `variant` + `defines`
    (+ extra compiler `flags`) build an experimental lib/librt_amd_<variant>.so
    (loaded with RT_AMD_VARIANT)."""
    lib_path = LIB_PATH.with_name(f"librt_amd_{variant}.so") if variant else LIB_PATH
    if not force and lib_path.exists() and lib_path.stat().st_mtime >= _newest_input():
        return lib_path
    cc = hipcc()
    obj_dir = OBJ_DIR / variant if variant else OBJ_DIR
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    for src, uflags, is_hip in _UNITS:
        obj = obj_dir / (src.replace(".", "_") + ".o")
        cmd = [cc, *_COMMON, *uflags, *flags, *[f"-D{d}" for d in defines]]
        if is_hip:
            cmd.append(f"--offload-arch={ARCH}")
        cmd += ["-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [cc, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib_path)
    return lib_path


ADDON_SRC = PKG_DIR.parent / "native" / "rt_addon.c"
ADDON_PATH = LIB_DIR / "rt_addon.node"
NODE_INCLUDE = Path("/usr/include/node")


def build_addon(force: bool = False, verbose: bool = False):
    """The N-API addon: C against Node's node_api.h, linked to
    librt_amd.so next to it. Returns its path, or None when Node's headers are
    not installed (the addon is then simply not built)."""
    if not (NODE_INCLUDE / "node_api.h").exists():
        return None
    lib = build_native()
    if not force and ADDON_PATH.exists() and ADDON_PATH.stat().st_mtime >= max(
            ADDON_SRC.stat().st_mtime, lib.stat().st_mtime, (INCLUDE / "rt_amd.h").stat().st_mtime):
        return ADDON_PATH
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        raise RuntimeError("no C compiler for the N-API addon")
    tmp = ADDON_PATH.with_suffix(".node.tmp")
    cmd = [cc, "-O2", "-fPIC", "-shared", "-Wall", "-DNODE_GYP_MODULE_NAME=rt_addon", f"-I{NODE_INCLUDE}",
           f"-I{INCLUDE}", str(ADDON_SRC), "-o", str(tmp), f"-L{LIB_DIR}", "-lrt_amd", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, ADDON_PATH)
    return ADDON_PATH


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    print(build_native(force=True, verbose=True, variant=a.variant, defines=a.defines))
