"""Camera: the reference's Camera surface over the HIP path tracer.

Mirrors src/camera.ts (RenderOptions 42-52, RenderRegion 54-59,
renderRegion 388-431, render 439-446) and RenderStats
(src/render-utils/renderStats.ts:6-64). A Camera is created by
create_camera_from_scene_data (scenes.py), exactly like the reference.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Iterable, Optional, Sequence

from . import _lib

RENDER_MODES = ("default", "bounces", "samples")


def _mm(total=0.0, mn=math.inf, mx=0.0, avg=0.0):
    return {"total": total, "min": mn, "max": mx, "avg": avg}


@dataclass
class RenderStats:
    """RenderStats (src/render-utils/renderStats.ts:6-64)."""

    pixels: float = 0
    samples: dict = field(default_factory=_mm)
    bounces: dict = field(default_factory=_mm)

    @classmethod
    def _from_c(cls, s: _lib.RtRenderStats) -> "RenderStats":
        return cls(pixels=s.pixels,
                   samples=_mm(s.samples_total, s.samples_min, s.samples_max, s.samples_avg),
                   bounces=_mm(s.bounces_total, s.bounces_min, s.bounces_max, s.bounces_avg))

    @staticmethod
    def merge(stats: Iterable["RenderStats"]) -> "RenderStats":
        """RenderStats.merge (renderStats.ts:42-64)."""
        m = RenderStats()
        for st in stats:
            m.pixels += st.pixels
            m.samples["total"] += st.samples["total"]
            m.samples["min"] = min(m.samples["min"], st.samples["min"])
            m.samples["max"] = max(m.samples["max"], st.samples["max"])
            m.bounces["total"] += st.bounces["total"]
            m.bounces["min"] = min(m.bounces["min"], st.bounces["min"])
            m.bounces["max"] = max(m.bounces["max"], st.bounces["max"])
        if m.pixels > 0:
            m.samples["avg"] = m.samples["total"] / m.pixels
        if m.samples["total"] > 0:
            m.bounces["avg"] = m.bounces["total"] / m.samples["total"]
        return m


def _region(region) -> _lib.RtRegion:
    if isinstance(region, dict):
        return _lib.RtRegion(int(region["x"]), int(region["y"]), int(region["width"]), int(region["height"]))
    x, y, w, h = region
    return _lib.RtRegion(int(x), int(y), int(w), int(h))


def _host_ptr(buf, nbytes: int, what: str):
    """Writable host pointer for a caller-owned buffer (bytearray / numpy / ctypes)."""
    if buf is None:
        return None, None
    try:
        import numpy as np  # noqa: F401
        if hasattr(buf, "__array_interface__"):
            arr = buf
            if not arr.flags["C_CONTIGUOUS"] or not arr.flags["WRITEABLE"]:
                raise ValueError(f"{what} must be a writable C-contiguous array")
            if arr.nbytes < nbytes:
                raise ValueError(f"{what} is too small: {arr.nbytes} < {nbytes} bytes")
            return C.c_void_p(arr.ctypes.data), arr
    except ImportError:  # pragma: no cover
        pass
    mv = memoryview(buf)
    if mv.readonly or mv.nbytes < nbytes:
        raise ValueError(f"{what} must be writable and hold at least {nbytes} bytes")
    cbuf = (C.c_char * mv.nbytes).from_buffer(buf)
    return C.cast(cbuf, C.c_void_p), cbuf


class Camera:
    """The reference Camera (src/camera.ts:61-472), rendering on MI355X."""

    channels = 3

    def __init__(self, scene_json: bytes, render_options_json: Optional[bytes]):
        lib = _lib.load()
        h = C.c_void_p()
        _lib.check(lib.rt_camera_create(scene_json, render_options_json, C.byref(h)))
        self._h = h
        self._lib = lib
        info = _lib.RtCameraInfo()
        _lib.check(lib.rt_camera_get_info(self._h, C.byref(info)))
        self._info = info

    # -- properties named as in the reference -------------------------------
    @property
    def image_width(self) -> int:
        return self._info.width

    @property
    def image_height(self) -> int:
        return self._info.height

    imageWidth = image_width
    imageHeight = image_height

    @property
    def info(self) -> dict:
        i = self._info
        return {f: getattr(i, f) for f, _ in _lib.RtCameraInfo._fields_}

    @property
    def precision(self) -> str:
        return "fp32" if self._info.precision == 1 else "ref"

    def set_precision(self, precision: str) -> None:
        _lib.check(self._lib.rt_camera_set_precision(self._h, _lib.PRECISION[precision]))
        self._info.precision = _lib.PRECISION[precision]

    @property
    def byte_length(self) -> int:
        return self.image_width * self.image_height * self.channels

    # -- rendering -----------------------------------------------------------
    def render_region(self, buffer, region, radiance=None) -> RenderStats:
        """Camera.renderRegion(buffer, region): writes the region's pixels of
        the full-frame RGB buffer (W*H*3 bytes) and returns RenderStats.
        `radiance` (optional float32 W*H*3) receives the final pixel colours."""
        ptr, _keep = _host_ptr(buffer, self.byte_length, "buffer")
        rptr, _keep2 = _host_ptr(radiance, self.byte_length * 4, "radiance")
        st = _lib.RtRenderStats()
        reg = _region(region)
        _lib.check(self._lib.rt_camera_render_region(self._h, C.byref(reg), ptr, rptr, C.byref(st)))
        return RenderStats._from_c(st)

    def render(self, buffer, radiance=None) -> RenderStats:
        """Camera.render(pixelData) (src/camera.ts:439-446)."""
        return self.render_region(buffer, (0, 0, self.image_width, self.image_height), radiance)

    renderRegion = render_region

    def render_png(self, bands: int = 1):
        """generateImageBuffer's core on the device (rt_camera_render_png): the frame
        rendered in one launch (`bands`, the reference's worker count, changes neither
        the image nor the merged stats), PNG encoded on the GPU -> (png bytes, RenderStats)."""
        out, n = C.c_void_p(), C.c_size_t()
        st = _lib.RtRenderStats()
        _lib.check(self._lib.rt_camera_render_png(self._h, int(bands), C.byref(st), C.byref(out), C.byref(n)))
        try:
            return C.string_at(out, n.value), RenderStats._from_c(st)
        finally:
            self._lib.rt_free(out)

    def render_region_multi(self, buffer, region, devices, radiance=None) -> RenderStats:
        """Camera.renderRegion over several GPUs from this one process (rt_camera_render_multi):
        the region's 8x8 tiles dealt round-robin over `devices` (HIP ordinals; one may repeat
        to rehearse the split on fewer GPUs), gathered on devices[0] over RCCL, stats merged as
        RenderStats.merge. Same buffers and result as render_region, bit for bit."""
        ptr, _keep = _host_ptr(buffer, self.byte_length, "buffer")
        rptr, _keep2 = _host_ptr(radiance, self.byte_length * 4, "radiance")
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        st = _lib.RtRenderStats()
        reg = _region(region)
        _lib.check(self._lib.rt_camera_render_multi(self._h, devs, len(devices), C.byref(reg), ptr, rptr, C.byref(st)))
        return RenderStats._from_c(st)

    def render_multi(self, buffer, devices, radiance=None) -> RenderStats:
        """Camera.render over several GPUs (render_region_multi of the whole image)."""
        return self.render_region_multi(buffer, (0, 0, self.image_width, self.image_height), devices, radiance)

    renderRegionMulti = render_region_multi

    def render_png_multi(self, devices):
        """generateImageBuffer over several GPUs (rt_camera_render_png_multi): the frame gathered on
        devices[0], PNG encoded there -> (png bytes, merged RenderStats)."""
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        out, n = C.c_void_p(), C.c_size_t()
        st = _lib.RtRenderStats()
        _lib.check(self._lib.rt_camera_render_png_multi(self._h, devs, len(devices), C.byref(st), C.byref(out),
                                                        C.byref(n)))
        try:
            return C.string_at(out, n.value), RenderStats._from_c(st)
        finally:
            self._lib.rt_free(out)

    def multi_info(self) -> dict:
        """The last multi-GPU render (rt_camera_multi_info): devices, transport, per-device
        path / accumulate ms and the root's gather ms (waits for their events)."""
        i = _lib.RtMultiInfo()
        _lib.check(self._lib.rt_camera_multi_info(self._h, C.byref(i)))
        n = i.n_devices
        return {"n_devices": n, "transport": _lib.GATHER.get(i.transport, "none") if n else "none",
                "devices": list(i.devices)[:n], "path_ms": list(i.path_ms)[:n], "accum_ms": list(i.accum_ms)[:n],
                "gather_ms": float(i.gather_ms), "slab_tiles": i.plan.slab_tiles, "tiles": i.plan.tiles}

    def render_device(self, *, rgb_ptr=None, radiance_ptr=None, region=None, tile_group=0, tile_groups=1,
                      precision: Optional[str] = None, stream=None, synchronize=False, count_work=False,
                      px_samples_ptr=None, px_bounces_ptr=None, traversal: Optional[str] = None,
                      packed: bool = False):
        """Device-resident render into caller-owned device buffers (full-frame
        layout, or with `packed` the tile-packed slab layout of rt_launch).
        Returns (RenderStats|None, work_counters|None)."""
        if region is None:
            region = (0, 0, self.image_width, self.image_height)
        L = _lib.RtLaunch()
        L.region = _region(region)
        L.tile_group, L.tile_groups = int(tile_group), int(tile_groups)
        L.precision = -1 if precision is None else _lib.PRECISION[precision]
        L.traversal = -1 if traversal is None else _lib.TRAVERSAL[traversal]
        # count_work: False/True (work counters) or "profile" (section timing, diagnostic)
        L.count_work = 2 if count_work == "profile" else (1 if count_work else 0)
        L.rgb = rgb_ptr
        L.radiance = radiance_ptr
        L.px_samples = px_samples_ptr
        L.px_bounces = px_bounces_ptr
        L.stream = stream
        L.synchronize = 1 if synchronize else 0
        L.packed_tiles = 1 if packed else 0
        st = _lib.RtRenderStats()
        cnt = (C.c_uint64 * _lib.COUNTER_WORDS)()
        _lib.check(self._lib.rt_camera_render_device(self._h, C.byref(L), C.byref(st), cnt))
        if not synchronize:
            return None, None
        if count_work == "profile":
            base = len(_lib.CT_NAMES)
            counters = {k: int(cnt[base + i]) for i, k in enumerate(_lib.PR_NAMES)}
            nl = _lib.PR_NAMES.index("loop")
            lb = base + len(_lib.PR_NAMES)
            for i, k in enumerate(_lib.PR_NAMES[:nl]):
                counters[f"lanes_{k}"] = int(cnt[lb + i])
                counters[f"execs_{k}"] = int(cnt[lb + nl + i])
        else:
            counters = dict(zip(_lib.CT_NAMES, [int(v) for v in cnt])) if count_work else None
        return RenderStats._from_c(st), counters

    def kernel_times(self):
        """(path_ms, accum_ms) of the last render call, from HIP events on its stream."""
        a, b = C.c_float(), C.c_float()
        _lib.check(self._lib.rt_camera_kernel_times(self._h, C.byref(a), C.byref(b)))
        return float(a.value), float(b.value)

    def stats_words(self, dst_ptr: int, stream=None) -> None:
        """Queue a copy of the last render's 8 RenderStats words (u64) to the
        device address `dst_ptr` on `stream` (rt_camera_stats_words)."""
        _lib.check(self._lib.rt_camera_stats_words(self._h, C.c_void_p(dst_ptr), C.c_void_p(stream)))

    def adaptive_info(self):
        """(rounds, samples rendered) of the last render's adaptive rounds
        (rt_camera_adaptive_info); (0, 0) when it was not adaptive or ran sequentially."""
        r, n = C.c_int32(), C.c_uint64()
        _lib.check(self._lib.rt_camera_adaptive_info(self._h, C.byref(r), C.byref(n)))
        return int(r.value), int(n.value)

    def pass_count(self) -> int:
        """Chunked-kernel passes of the last render (rt_camera_pass_count)."""
        n = C.c_int32()
        _lib.check(self._lib.rt_camera_pass_count(self._h, C.byref(n)))
        return int(n.value)

    KERNELS = ("none", "sequential", "chunked", "pool")

    def last_kernel(self) -> str:
        """Path kernel of the last render (rt_camera_last_kernel): 'sequential',
        'chunked' or 'pool' ('none' before any)."""
        n = C.c_int32()
        _lib.check(self._lib.rt_camera_last_kernel(self._h, C.byref(n)))
        return self.KERNELS[int(n.value)]

    def release_device(self) -> None:
        """Free the device copies; the next render re-creates them (rt_camera_release_device)."""
        _lib.check(self._lib.rt_camera_release_device(self._h))

    # -- introspection (tests) -----------------------------------------------
    def export(self):
        """Host copies of the flattened scene as numpy structured arrays."""
        import numpy as np
        i = self._info
        nodes = np.zeros(i.n_nodes, dtype=NODE_DTYPE)
        prims = np.zeros(i.n_objects, dtype=PRIM_DTYPE)
        mats = np.zeros(i.n_materials, dtype=MAT_DTYPE)
        lights = np.zeros(i.n_lights, dtype=LIGHT_DTYPE)
        prim_object = np.zeros(i.n_objects, dtype=np.int32)
        _lib.check(self._lib.rt_camera_export(self._h, nodes.ctypes.data, prims.ctypes.data, mats.ctypes.data,
                                              lights.ctypes.data if i.n_lights else None,
                                              prim_object.ctypes.data))
        return {"nodes": nodes, "prims": prims, "materials": mats, "lights": lights, "prim_object": prim_object}

    def debug_world_hit(self, origins, directions, traversal: Optional[str] = None):
        """Closest hit of rays through the device BVH (ref precision)."""
        import numpy as np
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
        out = np.zeros((o.shape[0], 10), dtype=np.float64)
        tr = -1 if traversal is None else _lib.TRAVERSAL[traversal]
        _lib.check(self._lib.rt_debug_world_hit(self._h, tr, o.shape[0], o.ctypes.data, d.ctypes.data,
                                                out.ctypes.data))
        return out

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.rt_camera_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _dtypes():
    import numpy as np
    node = np.dtype([("bmin", "<f4", 3), ("a", "<i4"), ("bmax", "<f4", 3), ("b", "<i4")])
    prim = np.dtype([("type", "<i4"), ("mat", "<i4"), ("s0", "<f8"), ("g0", "<f4", 4), ("g1", "<f4", 4),
                     ("g2", "<f4", 4), ("g3", "<f4", 4), ("g4", "<f4", 4)])
    mat = np.dtype([("type", "<i4"), ("c0", "<i4"), ("c1", "<i4"), ("pad0", "<i4"), ("color", "<f4", 4),
                    ("emitted", "<f4", 4), ("p0", "<f8"), ("pad1", "<f8")])
    light = np.dtype([("prim", "<i4"), ("type", "<i4"), ("area", "<f8")])
    assert node.itemsize == 32 and prim.itemsize == 96 and mat.itemsize == 64 and light.itemsize == 16
    return node, prim, mat, light


try:
    NODE_DTYPE, PRIM_DTYPE, MAT_DTYPE, LIGHT_DTYPE = _dtypes()
except ImportError:  # pragma: no cover
    NODE_DTYPE = PRIM_DTYPE = MAT_DTYPE = LIGHT_DTYPE = None


def rng_stream(seed: int, pixel: int, sample: int, n: int) -> Sequence[int]:
    """The path RNG stream (seeded Math.random replacement), host evaluation."""
    out = (C.c_uint32 * n)()
    _lib.check(_lib.load().rt_debug_rng(seed, pixel, sample, n, out))
    return list(out)
