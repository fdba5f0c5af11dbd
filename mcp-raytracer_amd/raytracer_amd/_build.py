"""Builds librt_amd.so (HIP kernels for gfx950 + the C ABI) in-tree.

Plain hipcc invocations, no cmake: every source is compiled for
--offload-arch=gfx950. The ref-precision kernel TU is compiled with
-ffp-contract=off so no multiply-add is fused (the reference's JS arithmetic
never fuses); the fp32 fast-mode TU may fuse.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
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
# -disable-machine-licm on the kernel units (round 5): the machine-code loop-invariant motion
# hoisted the fp64 polynomial constants of ocml's sincos (and a few other constants) out of the
# path loops into VGPR pairs it then spilled to scratch, reloading them after every cosine-PDF
# sincos: 84-104 B of scratch per lane in the BVH chunk kernels, 40 B in the pool kernel, all
# at the 128-VGPR cap. Without it the constants are rematerialised where they are used: no
# scratch, 97-126 VGPRs; Cornell 13.97 -> 13.72 ms, spheres-500 5.70 -> 5.64, rain spp128
# 10.97 -> 10.82, spheres-100k 2048^2 spp16 30.06 -> 29.15 ms path kernel, bit-exact
# (profiles/r05/nolicm/).
_KERNEL_FLAGS = ["-fno-slp-vectorize", "-mllvm", "-disable-machine-licm"]
_UNITS = [
    ("pt_ref.hip", ["-ffp-contract=off", *_KERNEL_FLAGS], True),
    ("pt_fp32.hip", ["-ffp-contract=fast", *_KERNEL_FLAGS], True),
    ("frame.hip", [], True),
    ("png.hip", [], True),
    ("rt_api.cpp", ["-ffp-contract=off", "-x", "hip"], True),
    ("scene.cpp", ["-ffp-contract=off"], False),
    ("image.cpp", [], False),
]
_HEADERS = ["json.hpp", "rt_math.hpp", "scene.hpp", "pt_kernel.hpp", "launch.hpp", "png_deflate.hpp"]
_LIBS = ["-lz"]


def source_hash(defines=(), flags=()) -> str:
    """Build id: sha256 of every source and header the library is compiled from
    plus the compiler flags (16 hex digits). Embedded in librt_amd.so
    (rt_build_id) and written next to it, so a stale binary is never reused."""
    h = hashlib.sha256()
    for name in [u[0] for u in _UNITS] + _HEADERS:
        h.update(name.encode() + b"\0" + (CSRC / name).read_bytes())
    h.update((INCLUDE / "rt_amd.h").read_bytes())
    h.update(repr((ARCH, _COMMON[:3], [(u[0], u[1]) for u in _UNITS], _LIBS, list(defines), list(flags))).encode())
    return h.hexdigest()[:16]


def id_path(lib_path: Path) -> Path:
    return lib_path.with_name(lib_path.name + ".id")


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build librt_amd.so")


def build_native(force: bool = False, verbose: bool = False, variant: str = "", defines=(), flags=()) -> Path:
    """Compile (if stale) and return the path of librt_amd.so. `variant` + `defines`
    (+ extra compiler `flags`) build an experimental lib/librt_amd_<variant>.so
    (loaded with RT_AMD_VARIANT)."""
    lib_path = LIB_PATH.with_name(f"librt_amd_{variant}.so") if variant else LIB_PATH
    bid = source_hash(defines, flags)
    idp = id_path(lib_path)
    if not force and lib_path.exists() and idp.exists() and idp.read_text().strip() == bid:
        return lib_path
    cc = hipcc()
    obj_dir = OBJ_DIR / variant if variant else OBJ_DIR
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    cmds, objs = [], []
    for src, uflags, is_hip in _UNITS:
        obj = obj_dir / (src.replace(".", "_") + ".o")
        cmd = [cc, *_COMMON, *uflags, *flags, *[f"-D{d}" for d in defines], f'-DRT_BUILD_ID="{bid}"']
        if is_hip:
            cmd.append(f"--offload-arch={ARCH}")
        cmd += ["-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(str(obj))
    # the units compile independently: in parallel (the kernel units dominate)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in [ex.submit(subprocess.run, c, check=True) for c in cmds]:
            f.result()
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [cc, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *objs, *_LIBS]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib_path)
    idp.write_text(bid + "\n")
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
