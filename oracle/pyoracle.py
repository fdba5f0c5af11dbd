"""ORACLE (test infrastructure only) - ctypes wrapper of liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module. It is the checker, never the product path.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

COUNTER_NAMES = ["node", "sphere", "quad", "plane", "material", "light_quad", "light_sphere",
                 "bounces", "diffuse", "samples", "rays"]


def build(force: bool = False) -> Path:
    src = HERE / "oracle.cpp"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE), "liboracle.so"], check=True)
    return LIB


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(os.fspath(LIB))
        D = C.POINTER(C.c_double)
        lib.or_last_error.restype = C.c_char_p
        lib.or_render.restype = C.c_int
        lib.or_render.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p]
        lib.or_world_hit.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                     C.c_void_p]
        for name in ["or_sphere_hit"]:
            getattr(lib, name).argtypes = [D, C.c_double, D, D, C.c_double, C.c_double, D]
        lib.or_quad_hit.argtypes = [D, D, D, D, D, C.c_double, C.c_double, D]
        lib.or_plane_intersect.argtypes = [D, D, D, D, D, C.c_double, C.c_double, D]
        lib.or_prim_box.argtypes = [C.c_int, D, D, D, C.c_double, D]
        lib.or_aabb_hit.argtypes = [D, D, D, D, C.c_double, C.c_double]
        for name in ["or_quad_pdf_value"]:
            getattr(lib, name).argtypes = [D, D, D, D, D]
            getattr(lib, name).restype = C.c_double
        lib.or_quad_area.argtypes = [D, D]
        lib.or_quad_area.restype = C.c_double
        lib.or_sphere_pdf_value.argtypes = [D, C.c_double, D, D]
        lib.or_sphere_pdf_value.restype = C.c_double
        lib.or_cosine_pdf_value.argtypes = [D, D]
        lib.or_cosine_pdf_value.restype = C.c_double
        lib.or_schlick.argtypes = [C.c_double, C.c_double]
        lib.or_schlick.restype = C.c_double
        lib.or_reflect.argtypes = [D, D, D]
        lib.or_refract.argtypes = [D, D, C.c_double, D]
        lib.or_unit.argtypes = [D, D]
        lib.or_length.argtypes = [D]
        lib.or_length.restype = C.c_double
        lib.or_onb.argtypes = [D, D, D]
        lib.or_get_ray.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, D]
        lib.or_material_probe.argtypes = [C.c_char_p, D, D, C.c_int, C.c_uint32, C.c_int, C.c_void_p]
        lib.or_onb.restype = None
        lib.or_mixture_value.argtypes = [C.c_int, D, D]
        lib.or_mixture_value.restype = C.c_double
        lib.or_rng_stream.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p]
        lib.or_camera_info.argtypes = [C.c_char_p, C.c_char_p, D]
        lib.or_math_probe.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
        lib.or_math_probe.restype = None
        _lib = lib
    return _lib


def _d(v):
    a = (C.c_double * len(v))(*[float(x) for x in v])
    return a


def _err():
    return RuntimeError(load().or_last_error().decode())


def dims(scene: dict, render: dict | None = None):
    d = (C.c_int * 4)()
    rc = load().or_render(json.dumps(scene).encode(), json.dumps(render).encode() if render else None,
                          0, 0, 0, 0, 1, 1, 0, None, None, None, None, None, None, d)
    if rc:
        raise _err()
    return {"width": d[0], "height": d[1], "bvh_depth": d[2], "n_lights": d[3]}


def render(scene: dict, render_opts: dict | None = None, region=None, precision: str = "ref", row_step: int = 1,
           threads: int = 1, counters: bool = False):
    """Render with the oracle. Returns dict(radiance, rgb, px_samples, px_bounces, stats, counters, width, height)."""
    lib = load()
    dm = dims(scene, render_opts)
    W, H = dm["width"], dm["height"]
    if region is None:
        region = (0, 0, W, H)
    rad = np.zeros((H, W, 3), dtype=np.float32)
    rgb = np.zeros((H, W, 3), dtype=np.uint8)
    pxs = np.zeros((H, W), dtype=np.int32)
    pxb = np.zeros((H, W), dtype=np.int32)
    st = np.zeros(7, dtype=np.float64)
    ct = np.zeros(11, dtype=np.float64)
    d = (C.c_int * 4)()
    rc = lib.or_render(json.dumps(scene).encode(), json.dumps(render_opts).encode() if render_opts else None,
                       int(region[0]), int(region[1]), int(region[2]), int(region[3]), int(row_step), int(threads),
                       1 if precision == "fp32" else 0, rad.ctypes.data, rgb.ctypes.data, pxs.ctypes.data,
                       pxb.ctypes.data, st.ctypes.data, ct.ctypes.data if counters else None, d)
    if rc:
        raise _err()
    stats = {"pixels": st[0], "samples": {"total": st[1], "min": st[2], "max": st[3]},
             "bounces": {"total": st[4], "min": st[5], "max": st[6]}}
    out = {"radiance": rad, "rgb": rgb, "px_samples": pxs, "px_bounces": pxb, "stats": stats,
           "width": W, "height": H}
    if counters:
        out["counters"] = dict(zip(COUNTER_NAMES, ct.tolist()))
    return out


def world_hit(scene: dict, origins, directions, tmin=0.001, tmax=float("inf")):
    o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
    dr = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
    out = np.zeros((o.shape[0], 10), dtype=np.float64)
    if load().or_world_hit(json.dumps(scene).encode(), o.shape[0], o.ctypes.data, dr.ctypes.data, tmin, tmax,
                           out.ctypes.data):
        raise _err()
    return out


def sphere_hit(c, r, o, d, tmin, tmax):
    out = (C.c_double * 9)()
    load().or_sphere_hit(_d(c), r, _d(o), _d(d), tmin, tmax, out)
    return {"hit": bool(out[0]), "t": out[1], "p": list(out[2:5]), "normal": list(out[5:8]), "front": bool(out[8])}


def quad_hit(q, u, v, o, d, tmin, tmax):
    out = (C.c_double * 9)()
    load().or_quad_hit(_d(q), _d(u), _d(v), _d(o), _d(d), tmin, tmax, out)
    return {"hit": bool(out[0]), "t": out[1], "p": list(out[2:5]), "normal": list(out[5:8]), "front": bool(out[8])}


def plane_intersect(q, u, v, o, d, tmin, tmax):
    out = (C.c_double * 4)()
    load().or_plane_intersect(_d(q), _d(u), _d(v), _d(o), _d(d), tmin, tmax, out)
    return {"hit": bool(out[0]), "t": out[1], "alpha": out[2], "beta": out[3]}


def prim_box(kind, a, b=(0, 0, 0), c=(0, 0, 0), r=0.0):
    out = (C.c_double * 6)()
    load().or_prim_box({"sphere": 0, "quad": 1, "plane": 2}[kind], _d(a), _d(b), _d(c), r, out)
    return list(out[:3]), list(out[3:])


def aabb_hit(mn, mx, o, d, tmin, tmax):
    return bool(load().or_aabb_hit(_d(mn), _d(mx), _d(o), _d(d), tmin, tmax))


def quad_pdf_value(q, u, v, origin, direction):
    return load().or_quad_pdf_value(_d(q), _d(u), _d(v), _d(origin), _d(direction))


def quad_area(u, v):
    return load().or_quad_area(_d(u), _d(v))


def sphere_pdf_value(c, r, origin, direction):
    return load().or_sphere_pdf_value(_d(c), r, _d(origin), _d(direction))


def cosine_pdf_value(n, direction):
    return load().or_cosine_pdf_value(_d(n), _d(direction))


def schlick(cosine, ratio):
    return load().or_schlick(cosine, ratio)


def reflect(v, n):
    out = (C.c_double * 3)()
    load().or_reflect(_d(v), _d(n), out)
    return list(out)


def refract(v, n, eta):
    out = (C.c_double * 3)()
    load().or_refract(_d(v), _d(n), eta, out)
    return list(out)


def unit(v):
    out = (C.c_double * 3)()
    load().or_unit(_d(v), out)
    return list(out)


def length(v):
    return load().or_length(_d(v))


def onb(n, a=(0, 0, 0)):
    """ONBasis(n): (u, v, w, local(a)) - src/geometry/onbasis.ts:18-51."""
    out = (C.c_double * 12)()
    load().or_onb(_d(n), _d(a), out)
    return list(out[0:3]), list(out[3:6]), list(out[6:9]), list(out[9:12])


def material_probe(material: dict, din, normal, front=True, seed=1, n=1):
    """n trials of Material.scatter + emitted (src/materials/*.ts) at a hit at the
    origin: array (n, 12) = valid, hasScattered, reflected, attenuation.xyz,
    direction.xyz (scattered ray or pdf.generate()), emitted.xyz."""
    out = np.zeros((n, 12), dtype=np.float64)
    if load().or_material_probe(json.dumps(material).encode(), _d(din), _d(normal), int(bool(front)), seed, n,
                                out.ctypes.data):
        raise _err()
    return out


def mixture_value(values, weights):
    return load().or_mixture_value(len(values), _d(values), _d(weights))


def rng_stream(seed, pixel, sample, n):
    out = (C.c_uint32 * n)()
    load().or_rng_stream(seed, pixel, sample, n, out)
    return list(out)


def get_ray(scene: dict, render_opts: dict | None, i: int, j: int, n: int = 0):
    """Camera.getRay(i, j) of sample n (src/camera.ts), RNG keyed as in a render: (origin, direction)."""
    out = (C.c_double * 6)()
    if load().or_get_ray(json.dumps(scene).encode(), json.dumps(render_opts).encode() if render_opts else b"", i, j, n,
                         out):
        raise _err()
    return list(out[0:3]), list(out[3:6])


def camera_info(scene: dict, render_opts: dict | None = None):
    out = (C.c_double * 14)()
    if load().or_camera_info(json.dumps(scene).encode(), json.dumps(render_opts).encode() if render_opts else None,
                             out):
        raise _err()
    return {"width": int(out[0]), "height": int(out[1]), "pixel00": list(out[2:5]), "du": list(out[5:8]),
            "dv": list(out[8:11]), "center": list(out[11:14])}


def math_probe(u):
    """The oracle's (cos(phi), sin(phi), pow(xi, 5)) for xi = u / 2^32, phi = 2 pi xi."""
    u = np.ascontiguousarray(u, dtype=np.uint32)
    out = np.zeros((u.size, 3), dtype=np.float64)
    load().or_math_probe(int(u.size), u.ctypes.data, out.ctypes.data)
    return out
