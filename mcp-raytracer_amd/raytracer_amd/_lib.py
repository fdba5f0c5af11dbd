"""ctypes binding of librt_amd.so (include/rt_amd.h).

The library is loaded from this package's lib/ directory only; if it is
missing or does not export the ABI, import fails loudly - there is no CPU
fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from pathlib import Path

from ._build import LIB_PATH, id_path, source_hash

# Public header, parsed by tests to check that every declared symbol is exported.
HEADER = Path(__file__).resolve().parents[2] / "include" / "rt_amd.h"

RT_OK, RT_ERR_INVALID, RT_ERR_DEVICE, RT_ERR_RENDER = 0, 1, 2, 3
PRECISION = {"ref": 0, "fp32": 1}
TRAVERSAL = {"fast": 0, "reference": 1, "brute": 2, "auto": 3}

CT_NAMES = ["node", "sphere", "quad", "plane", "material", "light_quad", "light_sphere",
            "bounces", "diffuse", "samples", "rays", "exact", "exact_wave", "cand0", "cand2", "exact2"]
PR_NAMES = ["newpath", "rr", "hit", "miss", "hitrec", "scatter", "sample", "pdf", "acc", "tile", "node", "leaf",
            "wnode", "wleaf", "loop", "trips"]
COUNTER_WORDS = 64
STATS_WORDS = 8  # RT_STATS_WORDS: pixels, samples, smin, smax, bounces, bmin, bmax, error


class RtRegion(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class RtRenderStats(C.Structure):
    _fields_ = [("pixels", C.c_double),
                ("samples_total", C.c_double), ("samples_min", C.c_double),
                ("samples_max", C.c_double), ("samples_avg", C.c_double),
                ("bounces_total", C.c_double), ("bounces_min", C.c_double),
                ("bounces_max", C.c_double), ("bounces_avg", C.c_double)]


class RtCameraInfo(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("channels", C.c_int32),
                ("n_objects", C.c_int32), ("n_nodes", C.c_int32), ("n_lights", C.c_int32),
                ("n_materials", C.c_int32), ("bvh_depth", C.c_int32),
                ("samples_loop", C.c_int32), ("depth", C.c_int32), ("roulette", C.c_int32),
                ("roulette_depth", C.c_int32), ("mode", C.c_int32), ("adaptive", C.c_int32),
                ("precision", C.c_int32), ("traversal", C.c_int32), ("seed", C.c_uint32),
                ("samples", C.c_double), ("aperture", C.c_double),
                ("a_tolerance", C.c_double), ("a_batch", C.c_double)]


class RtLaunch(C.Structure):
    _fields_ = [("region", RtRegion), ("tile_group", C.c_int32), ("tile_groups", C.c_int32),
                ("precision", C.c_int32), ("traversal", C.c_int32), ("count_work", C.c_int32),
                ("rgb", C.c_void_p), ("radiance", C.c_void_p),
                ("px_samples", C.c_void_p), ("px_bounces", C.c_void_p),
                ("stream", C.c_void_p), ("synchronize", C.c_int32), ("packed_tiles", C.c_int32)]


MAX_DEVICES = 16  # RT_MAX_DEVICES
GATHER = {0: "rccl", 1: "peer"}  # RT_GATHER_*


class RtMultiPlan(C.Structure):
    _fields_ = [("region", RtRegion), ("n_devices", C.c_int32), ("slab_tiles", C.c_int32), ("tiles", C.c_int64),
                ("slab_bytes_rgb", C.c_int64), ("slab_bytes_radiance", C.c_int64), ("stats_offset", C.c_int64),
                ("group_tiles", C.c_int32 * MAX_DEVICES)]


class RtMultiInfo(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("transport", C.c_int32), ("devices", C.c_int32 * MAX_DEVICES),
                ("path_ms", C.c_float * MAX_DEVICES), ("accum_ms", C.c_float * MAX_DEVICES),
                ("gather_ms", C.c_float), ("plan", RtMultiPlan)]


class RtError(RuntimeError):
    """An error returned through the C ABI (the reference would throw an Error)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


_SIGS = {
    "rt_version": (C.c_int, []),
    "rt_last_error": (C.c_char_p, []),
    "rt_free": (None, [C.c_void_p]),
    "rt_generate_scene_data": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "rt_camera_create": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "rt_camera_destroy": (None, [C.c_void_p]),
    "rt_camera_get_info": (C.c_int, [C.c_void_p, C.POINTER(RtCameraInfo)]),
    "rt_camera_set_precision": (C.c_int, [C.c_void_p, C.c_int32]),
    "rt_camera_render_region": (C.c_int, [C.c_void_p, C.POINTER(RtRegion), C.c_void_p, C.c_void_p,
                                          C.POINTER(RtRenderStats)]),
    "rt_camera_render": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(RtRenderStats)]),
    "rt_camera_render_device": (C.c_int, [C.c_void_p, C.POINTER(RtLaunch), C.POINTER(RtRenderStats),
                                          C.POINTER(C.c_uint64)]),
    "rt_camera_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p]),
    "rt_debug_world_hit": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_debug_pass_plan": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                     C.POINTER(C.c_int64)]),
    "rt_debug_rng": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32, C.c_void_p]),
    "rt_debug_math": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_debug_fp64": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "rt_camera_kernel_times": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "rt_camera_adaptive_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]),
    "rt_camera_stats_words": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_camera_pass_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "rt_camera_last_kernel": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "rt_camera_release_device": (C.c_int, [C.c_void_p]),
    "rt_build_id": (C.c_char_p, []),
    "rt_tiles_unpack": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(RtRegion), C.c_int32, C.c_int32,
                                  C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_encode_png": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p),
                                C.POINTER(C.c_size_t)]),
    "rt_encode_ppm": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "rt_encode_png_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_size_t)]),
    "rt_debug_png_host": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_size_t)]),
    "rt_camera_render_png": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(RtRenderStats), C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_size_t)]),
    "rt_multi_plan_region": (C.c_int, [C.POINTER(RtRegion), C.c_int32, C.c_int32, C.c_int32,
                                       C.POINTER(RtMultiPlan)]),
    "rt_camera_render_multi": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.POINTER(RtRegion),
                                         C.c_void_p, C.c_void_p, C.POINTER(RtRenderStats)]),
    "rt_camera_render_png_multi": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.POINTER(RtRenderStats),
                                             C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "rt_camera_multi_info": (C.c_int, [C.c_void_p, C.POINTER(RtMultiInfo)]),
}

_lib = None


def load() -> C.CDLL:
    """Load librt_amd.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    path = LIB_PATH
    variant = os.environ.get("RT_AMD_VARIANT")  # experiments: lib/librt_amd_<variant>.so (same package dir)
    if variant:
        if not variant.isidentifier():
            raise ImportError(f"bad RT_AMD_VARIANT {variant!r}")
        path = LIB_PATH.with_name(f"librt_amd_{variant}.so")
    if not path.exists():
        raise ImportError(f"{path.name} not found at {path}; run __graft_entry__.build() "
                          "(hipcc --offload-arch=gfx950) first - there is no CPU fallback")
    # PyTorch-ROCm ships its own libamdhip64.so.7 (same soname as /opt/rocm's).
    # Whichever loads first serves the whole process, and torch cannot run on a
    # newer runtime, so let torch's copy load first when torch is installed; the
    # library then shares torch's HIP runtime (device memory, streams).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(os.fspath(path))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the binary must have been built from these sources (no stale .so under test)
    built = lib.rt_build_id().decode()
    want = source_hash() if not variant else (id_path(path).read_text().strip() if id_path(path).exists() else "")
    if built != want:
        raise ImportError(f"{path.name} was built from sources {built}, the tree has {want}: "
                          "rebuild with __graft_entry__.build()")
    _lib = lib
    return lib


def build_id() -> str:
    """Source hash librt_amd.so was built from (rt_build_id)."""
    return load().rt_build_id().decode()


def check(code: int) -> None:
    if code != RT_OK:
        msg = load().rt_last_error()
        raise RtError(code, msg.decode("utf-8", "replace") if msg else f"rt error {code}")


def to_json(obj) -> bytes:
    """Serialise like JSON.stringify, keeping Infinity/NaN (accepted by the C parser)."""
    return json.dumps(obj, allow_nan=True, separators=(",", ":")).encode()


def multi_plan(region, width: int, height: int, n_devices: int) -> dict:
    """rt_multi_plan_region: the split of a region over n devices (host only)."""
    p = RtMultiPlan()
    reg = RtRegion(*[int(v) for v in region])
    check(load().rt_multi_plan_region(C.byref(reg), int(width), int(height), int(n_devices), C.byref(p)))
    return {"region": (p.region.x, p.region.y, p.region.width, p.region.height), "n_devices": p.n_devices,
            "slab_tiles": p.slab_tiles, "tiles": p.tiles, "slab_bytes_rgb": p.slab_bytes_rgb,
            "slab_bytes_radiance": p.slab_bytes_radiance, "stats_offset": p.stats_offset,
            "group_tiles": list(p.group_tiles)[:p.n_devices]}


def device_count() -> int:
    n = C.c_int32(0)
    check(load().rt_device_count(C.byref(n)))
    return int(n.value)
