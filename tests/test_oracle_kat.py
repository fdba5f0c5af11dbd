"""Pin the oracle's building blocks to the reference's own known-answer tests.

Each case cites the jest test it transcribes (paths under the reference's
tests/). jest's toBeCloseTo(x) default precision 2 means |d| < 0.005;
toBeCloseTo(x, p) means |d| < 10**-p / 2.
"""
import math

import numpy as np

import pytest


def close(a, b, p=2):
    return abs(a - b) < 10 ** (-p) / 2


# ---- tests/entities/sphere.test.ts:16-90 -----------------------------------
def test_sphere_hit_kats(oracle):
    c, r = (0, 0, -1), 0.5
    h = oracle.sphere_hit(c, r, (0, 0, 0), (0, 0, -1), 0, math.inf)
    assert h["hit"] and close(h["t"], 0.5)
    assert all(close(a, b) for a, b in zip(h["p"], (0, 0, -0.5)))
    assert all(close(a, b) for a, b in zip(h["normal"], (0, 0, 1)))  # outward
    assert h["front"] is True
    assert not oracle.sphere_hit(c, r, (0, 1, 0), (0, 0, -1), 0, math.inf)["hit"]
    h = oracle.sphere_hit(c, r, (0, 0, -1), (0, 0, -1), 0.001, math.inf)  # from inside
    assert h["hit"] and close(h["t"], 0.5) and all(close(a, b) for a, b in zip(h["p"], (0, 0, -1.5)))
    assert all(close(a, b) for a, b in zip(h["normal"], (0, 0, 1)))  # -(outward (0,0,-1))
    assert h["front"] is False
    h = oracle.sphere_hit(c, r, (0, 0.5, 0), (0, 0, -1), 0, math.inf)  # grazing
    assert h["hit"] and close(h["t"], 1.0) and h["front"] is True
    assert not oracle.sphere_hit(c, r, (0, 0, 0), (0, 0, -1), 0.6, 1.0)["hit"]
    assert not oracle.sphere_hit(c, r, (0, 0, 0), (0, 0, -1), 0.0, 0.4)["hit"]


# ---- tests/entities/sphere.test.ts:99-152 ----------------------------------
def test_sphere_pdf_kats(oracle):
    c, r = (0, 0, -1), 0.5
    assert oracle.sphere_pdf_value(c, r, (0, 0, 0), (0, 1, 0)) == 0
    v = oracle.sphere_pdf_value(c, r, (0, 0, 0), (0, 0, -1))
    expected = 1 / (2 * math.pi * (1 - math.sqrt(1 - 0.25)))
    assert close(v, expected, 5)
    assert oracle.sphere_pdf_value(c, r, (0, 0, 5), (0, 0, -1)) > v


# ---- tests/entities/quad.test.ts:17-203,240-261 ----------------------------
def test_quad_kats(oracle):
    assert close(oracle.quad_area((1, 0, 0), (0, 1, 0)), 1)
    assert close(oracle.quad_area((2, 0, 0), (0, 3, 0)), 6)
    q, u, v = (0, 0, 5), (1, 0, 0), (0, 1, 0)
    h = oracle.quad_hit(q, u, v, (0.5, 0.5, 0), (0, 0, 1), 0, math.inf)
    assert h["hit"] and close(h["t"], 5) and all(close(a, b) for a, b in zip(h["p"], (0.5, 0.5, 5)))
    assert not oracle.quad_hit(q, u, v, (1.5, 0.5, 0), (0, 0, 1), 0, math.inf)["hit"]
    for corner in [(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0)]:  # corners are inclusive
        h = oracle.quad_hit(q, u, v, corner, (0, 0, 1), 0, math.inf)
        assert h["hit"] and close(h["t"], 5)
    assert not oracle.quad_hit(q, u, v, (0, 0, 0), (1, 1, 0), 0, math.inf)["hit"]  # parallel
    f = oracle.quad_hit(q, u, v, (0.5, 0.5, 0), (0, 0, 1), 0, math.inf)
    assert f["front"] is False and close(f["normal"][2], -1)
    b = oracle.quad_hit(q, u, v, (0.5, 0.5, 10), (0, 0, -1), 0, math.inf)
    assert b["front"] is True and close(b["normal"][2], 1)
    mn, mx = oracle.prim_box("quad", (1, 2, 5), (3, 0, 0), (0, 4, 0))
    for a, e in zip(mn + mx, [1 - 1e-4, 2 - 1e-4, 5 - 1e-4, 4 + 1e-4, 6 + 1e-4, 5 + 1e-4]):
        assert close(a, e)
    mn, mx = oracle.prim_box("quad", (0, 0, 0), (1, 1, 0), (0, 1, 1))
    for a, e in zip(mn + mx, [-1e-4, -1e-4, -1e-4, 1 + 1e-4, 2 + 1e-4, 1 + 1e-4]):
        assert close(a, e)
    # pdfValue: miss -> 0; hit -> dist^2 / (area * |cos|)
    assert oracle.quad_pdf_value(q, u, v, (0, 0, 0), (0, 1, 0)) == 0
    d = oracle.unit((0.5, 0.5, 5))
    pv = oracle.quad_pdf_value(q, u, v, (0, 0, 0), d)
    dist2 = 0.5 ** 2 + 0.5 ** 2 + 25
    expected = dist2 / (1 * abs(d[2]))
    assert pv > 0 and close(pv, expected, 5 - 3)  # fp32-stored direction: compare to 1e-3 relative scale
    assert abs(pv - expected) / expected < 1e-6


# ---- tests/entities/quad.test.ts:356-370 (just outside the edge) ----------
def test_quad_barely_misses(oracle):
    assert not oracle.quad_hit((0, 0, 5), (1, 0, 0), (0, 1, 0), (1.0001, 0.5, 0), (0, 0, 1), 0, math.inf)["hit"]


# ---- tests/entities/plane.test.ts:100-136,211-287 --------------------------
def test_plane_kats(oracle):
    r = oracle.plane_intersect((0, 0, 0), (2, 0, 0), (0, 3, 0), (1, 1.5, -1), (0, 0, 1), 0, math.inf)
    assert r["hit"] and close(r["t"], 1) and close(r["alpha"], 0.5) and close(r["beta"], 0.5)
    assert not oracle.plane_intersect((0, 0, 5), (1, 0, 0), (0, 1, 0), (0, 0, 0), (0, 0, 1), 0, 4)["hit"]
    inf = math.inf
    mn, mx = oracle.prim_box("plane", (0, 0, 5), (1, 0, 0), (0, 1, 0))
    assert mn[:2] == [-inf, -inf] and mx[:2] == [inf, inf] and close(mn[2], 5 - 1e-4) and close(mx[2], 5 + 1e-4)
    mn, mx = oracle.prim_box("plane", (0, 3, 0), (1, 0, 0), (0, 0, 1))
    assert mn[0] == -inf and mn[2] == -inf and close(mn[1], 3 - 1e-4) and close(mx[1], 3 + 1e-4)
    mn, mx = oracle.prim_box("plane", (-2, 0, 0), (0, 1, 0), (0, 0, 1))
    assert close(mn[0], -2 - 1e-4) and close(mx[0], -2 + 1e-4) and mn[1] == -inf and mx[2] == inf
    mn, mx = oracle.prim_box("plane", (0, 0, 0), (1, 1, 0), (0, 1, 1))
    assert mn == [-inf] * 3 and mx == [inf] * 3


# ---- tests/geometry/aabb.test.ts:6-66 --------------------------------------
def test_aabb_kats(oracle):
    box = ((-1, -1, -1), (1, 1, 1))
    assert oracle.aabb_hit(*box, (0, 0, -5), (0, 0, 1), 0.1, 100)
    assert not oracle.aabb_hit(*box, (5, 0, 0), (0, 0, 1), 0.1, 100)
    assert not oracle.aabb_hit(*box, (0, 0, -5), (0, 0, 1), 0.1, 3)


def test_aabb_weak_per_axis_test_is_reference_behaviour(oracle):
    """AABB.hit clips each axis against the ORIGINAL interval (aabb.ts:49-54),
    so a ray that passes each slab at different times still 'hits'."""
    # Ray along +x+y: x-slab at t in [4,6], y-slab at t in [-1,1] (the intervals don't overlap).
    box = ((4, -1, -1), (6, 1, 1))
    assert oracle.aabb_hit(*box, (0, 0, 0), (1, 1, 0.0001), 0.001, math.inf)


# ---- tests/geometry/pdf.test.ts:55-77,126-156 ------------------------------
def test_cosine_pdf_kats(oracle):
    n = (0, 1, 0)
    assert close(oracle.cosine_pdf_value(n, (0, 1, 0)), 1 / math.pi)
    assert close(oracle.cosine_pdf_value(n, oracle.unit((1, 1, 0))), 0.7071 / math.pi, 4)
    assert close(oracle.cosine_pdf_value(n, (1, 0, 0)), 0)
    assert oracle.cosine_pdf_value(n, (0, -1, 0)) == 0


def test_mixture_pdf_kats(oracle):
    assert close(oracle.mixture_value([1, 1], [0.5, 0.5]), 1.0)
    assert close(oracle.mixture_value([1, 3], [0.5, 0.5]), 2)
    assert close(oracle.mixture_value([1, 3], [1, 3]), 2.5)


# ---- tests/materials/dielectric.test.ts:109-135 ----------------------------
def test_schlick_kats(oracle):
    perp = oracle.schlick(1.0, 1 / 1.5)
    graz = oracle.schlick(0.1, 1 / 1.5)
    assert graz > perp
    assert close(perp, 0.04, 1)
    assert graz > 0.5


# ---- tests/materials/metal.test.ts:30-73 -----------------------------------
def test_metal_reflect_kat(oracle):
    d = oracle.unit((1, -1, 0))
    r = oracle.reflect(d, (0, 1, 0))
    e = oracle.unit((1, 1, 0))
    assert all(close(a, b, 5) for a, b in zip(r, e))


# ---- tests/geometry/vec3.test.ts (gl-matrix boundary) ----------------------
def test_vec3_boundary(oracle):
    assert oracle.length((3, 4, 0)) == 5.0
    assert oracle.unit((0, 0, 0)) == [0, 0, 0]  # len 0: normalize leaves zeros
    u = oracle.unit((1, 2, 2))
    assert all(close(a, b, 6) for a, b in zip(u, (1 / 3, 2 / 3, 2 / 3)))
    # fp32 storage: components are exactly representable floats
    assert all(np.float32(a) == a for a in u)
    r = oracle.refract((0, -1, 0), (0, 1, 0), 1 / 1.5)  # normal incidence passes straight through
    assert all(close(a, b, 6) for a, b in zip(r, (0, -1, 0)))


# ---- tests/camera.test.ts:161-174 (dimensions) -----------------------------
def test_camera_dimensions(oracle):
    scene = {"camera": {"vfov": 90, "from": [0, 0, 0], "at": [0, 0, -1], "up": [0, 1, 0],
                        "background": {"type": "gradient", "top": [1, 1, 1], "bottom": [0.5, 0.7, 1]}},
             "objects": [{"type": "sphere", "pos": [0, 0, -1], "r": 0.5, "material": {"type": "lambert",
                                                                                     "color": [0.5, 0.5, 0.5]}}]}
    d = oracle.camera_info(scene)
    assert (d["width"], d["height"]) == (400, 225)
    d = oracle.camera_info(scene, {"width": 100, "aspect": 1.0})
    assert (d["width"], d["height"]) == (100, 100)


# ---- tests/camera.test.ts:725-816 (background lerp) ------------------------
@pytest.mark.parametrize("look,expect", [((0, 1, 0), "bottom"), ((0, -1, 0), "top")])
def test_background_gradient(oracle, look, expect):
    top, bottom = [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]
    scene = {"camera": {"vfov": 1, "from": [0, 0, 0], "at": list(look), "up": [1, 0, 0], "focus": 1,
                        "background": {"type": "gradient", "top": top, "bottom": bottom}},
             "objects": [{"type": "sphere", "pos": [100, 100, 100], "r": 0.1,
                          "material": {"type": "lambert", "color": [1, 1, 1]}}]}
    out = oracle.render(scene, {"width": 4, "aspect": 1, "samples": 1, "aTolerance": 0})
    c = out["radiance"][2, 2]
    want = bottom if expect == "bottom" else top
    assert all(close(a, b, 2) for a, b in zip(c, want))


# ---- tests/camera.test.ts:331-396 (render stats) ---------------------------
def test_render_stats_kats(oracle):
    scene = {"camera": {"vfov": 90, "from": [0, 0, 0], "at": [0, 0, -1], "up": [0, 1, 0], "aperture": 0,
                        "background": {"type": "gradient", "top": [1, 1, 1], "bottom": [0.5, 0.7, 1]}},
             "objects": [{"type": "sphere", "pos": [0, 0, -1], "r": 0.5, "material": {"type": "lambert",
                                                                                     "color": [0.5, 0.5, 0.5]}}]}
    out = oracle.render(scene, {"width": 10, "aspect": 1.0, "samples": 1})
    st = out["stats"]
    assert st["samples"]["total"] == 100 and st["pixels"] == 100
    assert st["samples"]["min"] == 1 and st["samples"]["max"] == 1
    assert st["bounces"]["min"] >= 0
    out = oracle.render(scene, {"width": 20, "aspect": 1.0, "samples": 1}, region=(5, 5, 10, 10))
    assert out["stats"]["pixels"] == 100 and out["stats"]["samples"]["total"] == 100


def test_rng_stream_product_matches_oracle(oracle, rt):
    """The seeded Math.random replacement: product (host) and oracle streams agree bit-for-bit."""
    for key in [(0x5EED, 0, 0), (1, 12345, 7), (0xFFFFFFFF, 4096 * 4096 - 1, 1023)]:
        assert rt.rng_stream(*key, 64) == oracle.rng_stream(*key, 64)


# ---- tests/geometry/vec3.test.ts:81-110 ------------------------------------
def test_vec3_length_and_unit_kats(oracle):
    assert oracle.length((3, 4, 0)) == 5 and oracle.length((0, 0, 0)) == 0
    assert close(oracle.length((1, 1, 1)), math.sqrt(3))
    u = oracle.unit((3, 4, 0))
    assert close(u[0], 3 / 5) and close(u[1], 4 / 5) and close(u[2], 0) and close(oracle.length(u), 1)


# ---- tests/geometry/onbasis.test.ts:7-86 -----------------------------------
def _dot(a, b):
    return sum(x * y for x, y in zip(a, b))


@pytest.mark.parametrize("n", [(0, 1, 0), (1, 0, 0), (0, 0, 1), (1, 1, 1), (-1, 2, 3)])
def test_onbasis_kats(oracle, n):
    n = oracle.unit(n)
    u, v, w, _ = oracle.onb(n)
    assert close(_dot(w, n), 1)
    for a in (u, v, w):
        assert close(oracle.length(a), 1)
    assert close(_dot(u, v), 0) and close(_dot(u, w), 0) and close(_dot(v, w), 0)


def test_onbasis_local_kats(oracle):
    n = (0, 1, 0)
    u, v, w, z = oracle.onb(n, (0, 0, 1))
    assert close(_dot(z, n), 1)
    x = oracle.onb(n, (1, 0, 0))[3]
    y = oracle.onb(n, (0, 1, 0))[3]
    assert close(_dot(x, n), 0) and close(_dot(y, n), 0) and close(_dot(y, x), 0)
    c = oracle.onb(n, (1, 2, 3))[3]
    want = [a + 2 * b + 3 * e for a, b, e in zip(u, v, w)]
    assert all(close(a, b) for a, b in zip(c, want))


# ---- tests/geometry/interval.test.ts:55-70 + src/entities/sphere.ts:60-62 --
def test_hit_interval_is_open(oracle):
    """Primitive hits use Interval.surrounds (strict): a root exactly at tmin
    or tmax is rejected, so the far root is taken or the ray misses."""
    c, r, o, d = (0, 0, -1), 0.5, (0, 0, 0), (0, 0, -1)
    h = oracle.sphere_hit(c, r, o, d, 0.5, math.inf)
    assert h["hit"] and h["t"] == 1.5
    assert not oracle.sphere_hit(c, r, o, d, 0.001, 0.5)["hit"]
    assert oracle.sphere_hit(c, r, o, d, 0.001, 0.5000001)["t"] == 0.5


# ---- tests/geometry/hittableList.test.ts + tests/geometry/bvh.test.ts ------
def _world(spheres):
    return {"camera": {"vfov": 90, "from": [0, 0, 0], "at": [0, 0, -1], "up": [0, 1, 0],
                       "background": {"type": "gradient", "top": [1, 1, 1], "bottom": [0.5, 0.7, 1]}},
            "objects": [{"type": "sphere", "pos": list(c), "r": r, "material": {"type": "lambert",
                                                                                "color": [0.8, 0.8, 0.8]}}
                        for c, r in spheres]}


def _hit(oracle, spheres, o, d, tmin, tmax):
    row = oracle.world_hit(_world(spheres), [o], [d], tmin, tmax)[0]
    return {"hit": bool(row[0]), "t": row[1], "p": row[2:5], "obj": int(row[9])}


def _brute(oracle, spheres, o, d, tmin, tmax):
    """HittableList.hit (src/geometry/hittableList.ts:40-60): closest-so-far over the list."""
    best = None
    for i, (c, r) in enumerate(spheres):
        h = oracle.sphere_hit(c, r, o, d, tmin, best["t"] if best else tmax)
        if h["hit"]:
            best = dict(h, obj=i)
    return best


S1, S2 = ((0, 0, -1), 0.5), ((0, 0, -3), 0.5)  # hittableList.test.ts:49-50


def test_hittable_list_kats(oracle):
    o, d = (0, 0, 0), (0, 0, -1)
    far = ((0, 100, -5), 10)  # hittableList.test.ts:12-14
    assert _hit(oracle, [S1], o, d, 0.001, math.inf)["hit"]
    assert not _hit(oracle, [S1], (0, 100, 0), d, 0.001, math.inf)["hit"]
    assert _hit(oracle, [S1, far], (0, 100, 0), d, 0.001, math.inf)["hit"]
    assert not _hit(oracle, [S1], (5, 5, 0), d, 0.001, math.inf)["hit"]
    h = _hit(oracle, [S1, S2], o, d, 0.001, math.inf)
    assert close(h["t"], 0.5) and close(h["p"][2], -0.5) and h["obj"] == 0
    h = _hit(oracle, [S2, S1], o, d, 0.001, math.inf)  # add order does not matter
    assert close(h["t"], 0.5) and close(h["p"][2], -0.5) and h["obj"] == 1
    assert close(_hit(oracle, [S1, S2], o, d, 0.001, 1.0)["t"], 0.5)
    h = _hit(oracle, [S1, S2], o, d, 1.0, math.inf)  # sphere1's far root beats sphere2
    assert close(h["t"], 1.5) and close(h["p"][2], -1.5)
    assert not _hit(oracle, [S1, S2], o, d, 1.6, 2.4)["hit"]


BVH_SPHERES = [((0, 0, -1), 0.5), ((-1, 0, -1), 0.5), ((1, 0, -1), 0.5), ((0, -100.5, -1), 100)]  # bvh.test.ts:15-20
SMALL_SPHERES = [((i - 5, 0, -5), 0.3) for i in range(10)]  # bvh.test.ts:23-28


def test_bvh_box_kat(oracle):
    boxes = [oracle.prim_box("sphere", c, r=r) for c, r in BVH_SPHERES]
    mn = [min(b[0][a] for b in boxes) for a in range(3)]
    mx = [max(b[1][a] for b in boxes) for a in range(3)]
    assert mn[0] <= -1.5 and mx[0] >= 1.5 and mn[1] <= -100.5 - 100


def test_bvh_hit_kats(oracle):
    h = _hit(oracle, BVH_SPHERES, (0, 0, 0), (0, 0, -1), 0.1, 100)
    assert h["hit"] and close(h["t"], 0.5)
    assert not _hit(oracle, BVH_SPHERES, (0, 5, 0), (0, 1, 0), 0.1, 100)["hit"]
    assert _hit(oracle, SMALL_SPHERES, (0, 0, 0), (0, 0, -1), 0.1, 100)["hit"]


@pytest.mark.parametrize("spheres", [BVH_SPHERES, SMALL_SPHERES], ids=["four", "leaf"])
def test_bvh_matches_list(oracle, spheres):
    """bvh.test.ts:89-158 - BVH and list agree (t bit-exact, same object), on the
    test's rays plus a seeded fan of float32 rays."""
    rng = np.random.default_rng(11)
    dirs = [oracle.unit((0.5, -0.5, -1)), (0, 0, -1)] + [list(v) for v in rng.normal(size=(200, 3))]
    o = (0, 0, 0)
    sd = _world(spheres)
    D = np.asarray(dirs, dtype=np.float32)
    rows = oracle.world_hit(sd, np.zeros_like(D), D, 0.1, 100)
    for d, row in zip(D.astype(np.float64), rows):
        b = _brute(oracle, spheres, o, d, 0.1, 100)
        assert bool(row[0]) == (b is not None)
        if b is not None:
            assert row[1] == b["t"] and int(row[9]) == b["obj"]


# ---- tests/materials/*.test.ts: Material.scatter / emitted ------------------
# material_probe rows: valid, hasScattered, reflected, attenuation.xyz, dir.xyz, emitted.xyz
RED = {"type": "lambert", "color": [0.8, 0.2, 0.2]}
SILVER = {"type": "metal", "color": [0.9, 0.9, 0.9], "fuzz": 0.1}
GLASS = {"type": "glass", "ior": 1.5}


def test_diffuse_light_kats(oracle):
    """diffuseLight.test.ts:7-59 - emits its colour, never scatters."""
    r = oracle.material_probe({"type": "light", "emit": [3, 2, 1]}, (0, 1, 0), (0, 1, 0), n=4)
    assert (r[:, 0] == 0).all() and (r[:, 9:12] == [3, 2, 1]).all()


def test_non_emitting_materials_emit_black(oracle):
    """defaultMaterial.test.ts:26-40 / layeredMaterial.test.ts:188-201 /
    mixedMaterial.test.ts:242-253: only lights emit."""
    for m in [RED, SILVER, GLASS, {"type": "mixed", "diff": RED, "spec": SILVER, "weight": 0.5},
              {"type": "layered", "outer": GLASS, "inner": RED}]:
        assert (oracle.material_probe(m, (0, -1, 0), (0, 1, 0))[:, 9:12] == 0).all(), m["type"]


def test_lambertian_kats(oracle):
    """lambertian.test.ts:9-125 - albedo attenuation, cosine-PDF directions in the normal's hemisphere."""
    r = oracle.material_probe({"type": "lambert", "color": [0.5, 0.7, 0.3]}, (0, 1, 0), (0, 1, 0), n=200)
    assert (r[:, 0] == 1).all() and (r[:, 1] == 0).all()
    assert np.allclose(r[:, 3:6], np.float32([0.5, 0.7, 0.3]))
    assert (r[:, 7] > 0).all() and np.allclose(np.linalg.norm(r[:, 6:9], axis=1), 1, atol=0.05)


def test_metal_fuzz_kats(oracle):
    """metal.test.ts:77-125 - fuzz perturbs the mirror direction, which stays outward."""
    r = oracle.material_probe({"type": "metal", "color": [0.8, 0.6, 0.2], "fuzz": 0.5}, (0, -1, 0), (0, 1, 0), n=100)
    ok = r[:, 0] == 1
    assert ok.all() and (r[:, 7] > 0).all()
    perfect = (np.abs(r[:, 6]) < 1e-3) & (np.abs(r[:, 7] - 1) < 1e-3) & (np.abs(r[:, 8]) < 1e-3)
    assert perfect.sum() < 10


def test_metal_absorbs_below_surface(oracle):
    """metal.test.ts:127-160 - a grazing ray with heavy fuzz is absorbed
    (null) whenever the fuzzed reflection points below the surface."""
    d = oracle.unit((1, -0.01, 0))
    r = oracle.material_probe({"type": "metal", "color": [0.8, 0.6, 0.2], "fuzz": 0.8}, d, (0, 1, 0), n=400)
    assert 0 < (r[:, 0] == 0).sum() < 400  # some absorbed, some not
    assert (r[r[:, 0] == 1, 7] > 0).all()


def test_dielectric_scatter_kats(oracle):
    """dielectric.test.ts:16-107 - always a scattered ray, entering and exiting; white attenuation."""
    g = {"type": "glass", "ior": 1.5}
    for din, front in [((0, 0, -1), True), ((0, 0, 1), False)]:
        r = oracle.material_probe(g, din, (0, 0, 1), front, n=50)
        assert (r[:, 0] == 1).all() and (r[:, 1] == 1).all() and (r[:, 3:6] == 1).all()
        assert (np.linalg.norm(r[:, 6:9], axis=1) > 0).all()
    r = oracle.material_probe({"type": "glass", "ior": 2.4}, oracle.unit((0.9, 0.1, 0)), (-1, 0, 0), False, n=50)
    assert (r[:, 0] == 1).all() and (np.linalg.norm(r[:, 6:9], axis=1) > 0).all()
    # ratio * sin(theta) > 1: total internal reflection on every trial
    r = oracle.material_probe({"type": "glass", "ior": 2.4}, oracle.unit((1, -0.3, 0)), (0, 1, 0), False, n=50)
    assert (r[:, 2] == 1).all()


def test_mixed_material_kats(oracle):
    """mixedMaterial.test.ts:49-130,214-240 - weight clamps to [0,1]; weight 1 is
    always material1 (PDF), 0 always material2 (scattered ray); 0.3 splits ~30/70;
    emission is the weighted sum."""
    mix = lambda w: {"type": "mixed", "diff": RED, "spec": SILVER, "weight": w}
    for w, want_pdf in [(1.0, True), (1.5, True), (0.0, False), (-0.5, False)]:
        r = oracle.material_probe(mix(w), (1, -1, 0), (0, 1, 0), n=20)
        valid = r[:, 0] == 1
        assert valid.all()
        assert ((r[:, 1] == 0) == want_pdf).all(), w
    r = oracle.material_probe(mix(0.3), (1, -1, 0), (0, 1, 0), n=2000)
    assert abs((r[:, 1] == 0).mean() - 0.3) < 0.05
    e = oracle.material_probe({"type": "mixed", "weight": 0.3, "diff": {"type": "light", "emit": [1, 1, 0]},
                               "spec": {"type": "light", "emit": [0, 1, 1]}}, (0, -1, 0), (0, 1, 0))[0, 9:12]
    assert all(close(a, b, 5) for a, b in zip(e, (0.3, 1.0, 0.7)))


def test_layered_material_kats(oracle):
    """layeredMaterial.test.ts:57-260 - a dielectric reflection returns white
    attenuation and a ray; a transmission hands the refracted ray to the
    inner material (Lambertian: its albedo + PDF; Metal: its albedo + ray)."""
    lay = {"type": "layered", "outer": GLASS, "inner": RED}
    r = oracle.material_probe(lay, (1, 0, 0), (-1, 0, 0), n=1000)
    refl = (r[:, 1] == 1) & (r[:, 3:6] == 1).all(axis=1)
    paint = (r[:, 1] == 0) & np.isclose(r[:, 3:6], np.float32([0.8, 0.2, 0.2])).all(axis=1)
    assert refl.sum() > 0 and paint.sum() > 0 and refl.sum() + paint.sum() == 1000
    metal = {"type": "metal", "color": [0.8, 0.8, 0.9], "fuzz": 0.1}
    r = oracle.material_probe({"type": "layered", "outer": GLASS, "inner": metal}, (1, -1, 0), (0, 1, 0), n=1000)
    glass = (r[:, 1] == 1) & (r[:, 3:6] == 1).all(axis=1)
    through = (r[:, 1] == 1) & np.isclose(r[:, 3:6], np.float32([0.8, 0.8, 0.9])).all(axis=1)
    assert glass.sum() > 0 and through.sum() > 0


# ---- tests/camera.test.ts: getRay, defocus, orientations, roulette ---------
def _cam_scene(**cam):
    """createTestSceneData (camera.test.ts:99-131): one grey Lambertian sphere at (0, 0, -1)."""
    c = {"vfov": 90, "from": [0, 0, 0], "at": [0, 0, -1], "up": [0, 1, 0],
         "background": {"type": "gradient", "top": [1, 1, 1], "bottom": [0.5, 0.7, 1.0]}}
    c.update(cam)
    return {"camera": c, "materials": [{"id": "test-material", "material": {"type": "lambert", "color": [0.5] * 3}}],
            "objects": [{"type": "sphere", "pos": [0, 0, -1], "r": 0.5, "material": "test-material"}]}


RD = {"width": 100, "aspect": 1.0, "samples": 1}  # camera.test.ts:153-157


def _add(a, b):
    return [x + y for x, y in zip(a, b)]


def test_get_ray_aperture_zero_is_deterministic(oracle):
    """camera.test.ts:202-222 - aperture 0, samples 1: every sample's ray is the same."""
    sd = _cam_scene(aperture=0)
    r0 = oracle.get_ray(sd, RD, 50, 50, 0)
    assert all(oracle.get_ray(sd, RD, 50, 50, n) == r0 for n in range(1, 8))


def test_get_ray_defocus_varies_origins_and_keeps_focus(oracle):
    """camera.test.ts:176-276 - aperture > 0 moves ray origins over the lens; every ray
    of a pixel still passes through the same point of the focus plane (samples 1: no
    jitter), which sits |from - at| away unless `focus` is given."""
    sd = _cam_scene(aperture=2.0, focus=1.0)
    rays = [oracle.get_ray(sd, {**RD, "samples": 10}, 50, 50, n) for n in range(10)]
    assert len({tuple(o) for o, _ in rays}) > 1
    for from_, at, focus, plane_z in [([0, 0, 3], [0, 0, 0], None, 0.0), ([0, 0, 3], [0, 0, 0], 5.0, -2.0)]:
        sd = _cam_scene(**{"from": from_, "at": at, "aperture": 1.0, **({"focus": focus} if focus else {})})
        pts = [_add(*oracle.get_ray(sd, RD, 50, 50, n)) for n in range(6)]
        assert len({tuple(o) for o, _ in (oracle.get_ray(sd, RD, 50, 50, n) for n in range(6))}) > 1
        for p in pts:
            assert all(close(a, b, 6) for a, b in zip(p, pts[0]))
            assert close(p[2], plane_z, 6)


@pytest.mark.parametrize("aperture", [0.001, 10.0])
def test_get_ray_aperture_edge_cases(oracle, aperture):
    """camera.test.ts:278-300."""
    o, d = oracle.get_ray(_cam_scene(aperture=aperture, focus=1.0), RD, 50, 50, 3)
    assert all(math.isfinite(x) for x in o + d) and oracle.length(d) > 0


def test_get_ray_image_bounds_and_distinct_pixels(oracle):
    """camera.test.ts:304-330 - corner pixels give finite non-zero directions; pixels differ."""
    sd = _cam_scene()
    ds = [tuple(oracle.get_ray(sd, RD, i, j)[1]) for i, j in [(0, 0), (99, 0), (0, 99), (99, 99), (50, 50)]]
    assert all(oracle.length(d) > 0 for d in ds) and len(set(ds)) == 5
    assert ds[0][0] < 0 < ds[1][0] and ds[0][1] > 0 > ds[2][1]  # row 0 is the top of the image


@pytest.mark.parametrize("from_,at", [([0, 0, 1], [0, 0, 0]), ([1, 1, 1], [0, 0, 0]), ([-1, 0, 0], [1, 0, 0]),
                                      ([0, 5, 0], [0, 0, 0])])
def test_get_ray_orientations(oracle, from_, at):
    """camera.test.ts:417-439 - the centre pixel looks along at - from."""
    o, d = oracle.get_ray(_cam_scene(**{"from": from_, "at": at}), {**RD, "width": 101}, 50, 50)
    look = oracle.unit([b - a for a, b in zip(from_, at)])
    assert all(close(a, b, 6) for a, b in zip(oracle.unit(d), look)) and o == [float(x) for x in from_]


def test_roulette_reduces_bounces(oracle):
    """camera.test.ts:592-654 - Russian roulette keeps every pixel and does not add bounces."""
    sd = _cam_scene()
    for spp, rdepth, tol in [(100, 3, 1.2), (50, 2, 1.1)]:
        off = oracle.render(sd, {"width": 10, "aspect": 1.0, "samples": spp, "roulette": False, "aTolerance": 0})
        on = oracle.render(sd, {"width": 10, "aspect": 1.0, "samples": spp, "roulette": True, "rouletteDepth": rdepth,
                                "aTolerance": 0})
        assert off["stats"]["pixels"] == on["stats"]["pixels"] == 100
        assert on["stats"]["bounces"]["total"] <= off["stats"]["bounces"]["total"] * tol


@pytest.mark.parametrize("albedo", [0.0, 2.0])
def test_roulette_zero_and_high_attenuation(oracle, albedo):
    """camera.test.ts:658-698 - zero and >1 attenuation render finite radiance (continuation
    probability capped at 0.95)."""
    sd = _cam_scene()
    sd["materials"][0]["material"]["color"] = [albedo] * 3
    out = oracle.render(sd, {"width": 10, "aspect": 1.0, "samples": 8, "roulette": True, "rouletteDepth": 1,
                             "aTolerance": 0})
    assert np.isfinite(out["radiance"]).all() and (out["radiance"] >= 0).all()
