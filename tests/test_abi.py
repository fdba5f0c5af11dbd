"""The C ABI boundary (include/rt_amd.h): exports, host-side behaviour and the
reference's error behaviour. No GPU needed (no render calls)."""
import ctypes
import re

import pytest


def test_library_exports_every_declared_symbol(rt):
    from raytracer_amd import _lib
    lib = _lib.load()
    text = _lib.HEADER.read_text()
    names = set(re.findall(r"^\s*(?:int|void|const char\*)\s+\**(rt_\w+)\s*\(", text, re.M))
    assert len(names) >= 20
    for n in sorted(names):
        assert hasattr(lib, n), f"{n} declared in rt_amd.h but not exported"
    assert lib.rt_version() == 3


def test_build_id_matches_sources(rt):
    """The loaded librt_amd.so was compiled from this tree's sources and flags."""
    from raytracer_amd import _build
    assert rt.build_id() == _build.source_hash()
    assert len(rt.build_id()) == 16


def test_library_is_gfx950_code_object(rt):
    from raytracer_amd import _lib
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data
    assert b"pt_render_kernel" in data


def test_product_kernels_do_not_spill_to_scratch(rt):
    """Every kernel a product render launches keeps its state in registers: a scratch reload
    inside the path loop misses L2 behind the record stream (round 5: the fp64 sincos constants
    MachineLICM hoisted and spilled cost 1-3 % and doubled the record write traffic; DESIGN.md
    §4). Instrumented (INSTR > 0) and emission-stack (EMIT) variants are diagnostic or keep the
    stack in scratch by design."""
    import sys
    from pathlib import Path
    from raytracer_amd import _lib
    pytest.importorskip("msgpack", reason="the AMDGPU metadata note is msgpack (tools/kernel_resources.py)")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import kernel_resources
    ks = kernel_resources.resources(_lib.LIB_PATH)
    assert len(ks) > 40, f"only {len(ks)} kernels found in the gfx950 code objects"
    # pt_pool_kernel<Real, TRAV, LDSS>; pt_chunk_kernel / pt_render_kernel<Real, EMIT=false, INSTR=0, ...>
    product = re.compile(r"pt_pool_kernel|pt_(chunk|render)_kernelI[df]Lb0ELi0E|pt_accum_kernel|pt_adapt_kernel")
    checked = [k for k in ks if product.search(k["name"])]
    assert len(checked) >= 20
    spills = [(k["name"], k["scratch"]) for k in checked if k["scratch"] != 0]
    assert not spills, spills
    # the persistent 1024-thread workgroups run 4 waves per SIMD: <= 128 VGPRs
    assert max(k["vgpr"] for k in checked if re.search(r"pt_(pool|chunk)_kernel", k["name"])) <= 128


def test_pool_kernel_trip_loop_waits_on_no_stores(rt, tmp_path):
    """The LDS-resident pool kernels (the headline's) keep their `s_waitcnt vmcnt(0)` count at the
    prologue's and the work hand-out's few: a vmcnt(0) in the trip loop also waits for the sample
    records stored just before it. Round 6 found 17 such waits, inserted before writes of a register
    the wait-count pass kept pending from the adaptive active-list load on the paths around its
    branch (pt_kernel.hpp slot_pixel; Cornell +0.4 %, fp32 +1.3 %, adaptive +4 %)."""
    import shutil
    import subprocess
    import sys
    from pathlib import Path
    from raytracer_amd import _lib
    objdump = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")
    if not objdump.exists():
        objdump = Path(shutil.which("llvm-objdump") or "/nonexistent")
    if not objdump.exists():
        pytest.skip("llvm-objdump not found")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import kernel_resources
    counts = {}
    for i, code in enumerate(kernel_resources.code_objects(_lib.LIB_PATH)):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(code)
        text = subprocess.run([str(objdump), "-d", "--no-show-raw-insn", str(f)], check=True,
                              capture_output=True, text=True).stdout
        name = None
        for line in text.splitlines():
            # pt_pool_kernel<Real, TRAV_BRUTE, LDSS 2> (the LDSS-0 instances read the scene from
            # global memory: their vmcnt waits are the scene loads)
            m = re.match(r"^[0-9a-f]+ <(_ZN2rt14pt_pool_kernelI[df]Li2ELi2E[^>]*)>:", line)
            if m:
                name = m.group(1)
                counts[name] = 0
            elif re.match(r"^[0-9a-f]+ <", line):
                name = None
            elif name and "s_waitcnt vmcnt(0)" in line:
                counts[name] += 1
    assert len(counts) == 2, counts  # ref and fp32
    assert max(counts.values()) <= 8, counts


def test_camera_info_defaults_and_merge_order(rt):
    sd = rt.generate_scene_data({"type": "cornell"})
    cam = rt.create_camera_from_scene_data(sd)  # render defaults + scene render {aspect 1, rouletteDepth 5}
    i = cam.info
    assert (i["width"], i["height"]) == (400, 400)
    assert i["samples"] == 100 and i["depth"] == 100 and i["roulette_depth"] == 5 and i["adaptive"] == 1
    assert i["a_tolerance"] == 0.05 and i["a_batch"] == 10
    # provided render options win over the scene's (scenes.ts:97-100)
    cam = rt.create_camera_from_scene_data(sd, {"width": 50, "aspect": 2, "rouletteDepth": 2, "aTolerance": 0})
    i = cam.info
    assert (i["width"], i["height"], i["roulette_depth"], i["adaptive"]) == (50, 25, 2, 0)
    d = rt.create_camera_from_scene_data(rt.generate_scene_data({"type": "rain", "options": {"seed": 1}}))
    assert (d.image_width, d.image_height) == (400, 225)  # 16:9 default (camera.test.ts:161-166)


def test_precision_option(rt):
    sd = rt.generate_scene_data({"type": "cornell"})
    assert rt.create_camera_from_scene_data(sd).precision == "ref"
    assert rt.create_camera_from_scene_data(sd, {"precision": "fp32"}).precision == "fp32"
    with pytest.raises(rt.RtError):
        rt.create_camera_from_scene_data(sd, {"precision": "half"})


@pytest.mark.parametrize("mutate,msg", [
    (lambda s: s["objects"][0].__setitem__("material", "nope"), "Material not found: nope"),
    (lambda s: s["objects"][0].__setitem__("type", "cone"), "Unknown object type: cone"),
    (lambda s: s["materials"][0]["material"].__setitem__("type", "plastic"), "Unknown material type: plastic"),
    (lambda s: s.__setitem__("objects", []), "reading 'maximum'"),
    (lambda s: s["objects"][0].__setitem__("material", {"type": "layered", "outer": {"type": "lambert",
                                                        "color": [1, 1, 1]}, "inner": "red"}),
     "Material is not a dielectric"),
])
def test_reference_errors(rt, mutate, msg):
    sd = rt.generate_scene_data({"type": "cornell"})
    mutate(sd)
    with pytest.raises(rt.RtError, match=re.escape(msg)):
        rt.create_camera_from_scene_data(sd)


def test_missing_vfov_gives_nan_camera_not_error(rt):
    """{...defaults, ...{vfov: undefined}} overrides the default with undefined
    (scenes.ts:83-94 -> camera.ts:115): the camera is built, its frame is NaN."""
    sd = rt.generate_scene_data({"type": "cornell"})
    del sd["camera"]["vfov"]
    cam = rt.create_camera_from_scene_data(sd, {"width": 8})
    assert cam.image_width == 8


def test_unknown_scene_type(rt):
    with pytest.raises(rt.RtError):
        rt.generate_scene_data({"type": "teapot"})


def test_metal_fuzz_and_mixed_weight_clamps(rt):
    sd = {"camera": {"vfov": 40, "from": [0, 0, 1], "at": [0, 0, 0], "up": [0, 1, 0],
                     "background": {"type": "gradient", "top": [1, 1, 1], "bottom": [1, 1, 1]}},
          "objects": [
              {"type": "sphere", "pos": [0, 0, 0], "r": 1, "material": {"type": "metal", "color": [1, 1, 1],
                                                                         "fuzz": 3}},
              {"type": "sphere", "pos": [0, 0, 0], "r": 1, "material": {"type": "metal", "color": [1, 1, 1]}},
              {"type": "sphere", "pos": [0, 0, 0], "r": 1, "material": {"type": "mixed", "weight": -2,
                                                                         "diff": {"type": "lambert", "color": [1, 1, 1]},
                                                                         "spec": {"type": "light", "emit": [2, 2, 2]}}},
          ]}
    mats = rt.create_camera_from_scene_data(sd, {"width": 4}).export()["materials"]
    metals = mats[mats["type"] == 1]
    assert sorted(metals["p0"].tolist()) == [0.0, 1.0]  # fuzz 3 -> 1; missing -> 0
    mixed = mats[mats["type"] == 4]
    assert mixed["p0"][0] == 0.0  # weight clamped into [0, 1]
    assert list(mixed["emitted"][0][:3]) == [2.0, 2.0, 2.0]  # E1*0 + E2*(1-0)


def test_png_encoder_roundtrip(rt):
    """rt_encode_png (librt_amd.so): 8-bit RGB, filter 0, zlib; CRCs checked by the decoder."""
    from raytracer_amd.png import decode_png_rgb, encode_png
    import numpy as np
    px = (np.arange(5 * 3 * 3) % 251).astype(np.uint8)
    for level in (0, 6, 9):
        w, h, out = decode_png_rgb(encode_png(px.tobytes(), 5, 3, level=level))
        assert (w, h) == (5, 3) and out == px.tobytes()
    big = np.random.default_rng(0).integers(0, 256, (300, 211, 3), dtype=np.uint8)
    w, h, out = decode_png_rgb(encode_png(big.tobytes(), 211, 300))
    assert (w, h) == (211, 300) and out == big.tobytes()
    with pytest.raises(ValueError):
        encode_png(b"\0" * 10, 5, 3)
    with pytest.raises(rt.RtError):
        encode_png(px.tobytes(), 5, 3, level=11)


def test_ppm_encoder(rt):
    from raytracer_amd.png import encode_ppm
    import numpy as np
    px = (np.arange(4 * 2 * 3) % 251).astype(np.uint8)
    out = encode_ppm(px.tobytes(), 4, 2)
    assert out == b"P6\n4 2\n255\n" + px.tobytes()


def test_divide_into_regions_matches_reference(rt):
    regs = rt.divide_into_regions(10, 7, 3)
    assert [(r["y"], r["height"]) for r in regs] == [(0, 3), (3, 3), (6, 1)]
    assert len(rt.divide_into_regions(10, 2, 8)) == 2


def test_fast_traversal_only_where_exact(rt):
    """Scenes whose primitives can be hit outside their reference box (negative
    radius sphere in the default scene) fall back to the reference traversal."""
    cornell = rt.generate_scene_data({"type": "cornell"})  # 8 primitives: AUTO -> brute force
    assert rt.create_camera_from_scene_data(cornell).info["traversal"] == 2
    assert rt.create_camera_from_scene_data(cornell, {"traversal": "fast"}).info["traversal"] == 0
    assert rt.create_camera_from_scene_data(rt.generate_scene_data({"type": "default"})).info["traversal"] == 1
    assert rt.create_camera_from_scene_data(rt.generate_scene_data({"type": "default"}),
                                            {"traversal": "brute"}).info["traversal"] == 1
    sd = rt.generate_scene_data({"type": "rain", "options": {"seed": 1}})  # 21 primitives: AUTO -> fast
    assert rt.create_camera_from_scene_data(sd).info["traversal"] == 0
    assert rt.create_camera_from_scene_data(sd, {"traversal": "reference"}).info["traversal"] == 1
    with pytest.raises(rt.RtError):
        rt.create_camera_from_scene_data(sd, {"traversal": "sideways"})


def _png_frames():
    import numpy as np
    rng = np.random.default_rng(7)
    yield "1x1", rng.integers(0, 256, (1, 1, 3), dtype=np.uint8)
    yield "noise", rng.integers(0, 256, (37, 211, 3), dtype=np.uint8)
    yield "flat", np.full((64, 300, 3), 17, np.uint8)
    yy, xx = np.mgrid[0:120, 0:173]
    grad = np.stack([xx * 255 // 172, yy * 255 // 119, (xx + yy) % 256], -1).astype(np.uint8)
    yield "gradient", grad
    noisy = np.clip(grad.astype(int) + rng.integers(-3, 4, grad.shape), 0, 255).astype(np.uint8)
    yield "gradient_noise", noisy
    yield "tall", rng.integers(0, 4, (1500, 3, 3), dtype=np.uint8)  # segments span many rows


def test_device_png_encoder_algorithm_on_host(rt):
    """The device PNG encoder's algorithm (png_deflate.hpp, run on the host by
    rt_debug_png_host): valid PNG (chunk CRCs, zlib Adler-32, deflate stream) for
    frames that exercise every filter type, runs, stored and dynamic blocks and
    segments spanning rows; decodes to the frame exactly."""
    import zlib
    from raytracer_amd.png import debug_png_host, decode_png_rgb
    sizes = {}
    for name, px in _png_frames():
        h, w, _ = px.shape
        png = debug_png_host(px.tobytes(), w, h)
        assert decode_png_rgb(png) == (w, h, px.tobytes()), name
        assert debug_png_host(px.tobytes(), w, h) == png  # deterministic
        sizes[name] = (len(png), px.size)
    # flat regions collapse to runs; noise falls back to stored blocks (<= 0.3 % over raw)
    assert sizes["flat"][0] < sizes["flat"][1] / 50
    assert sizes["gradient"][0] < sizes["gradient"][1] / 4
    assert sizes["noise"][0] < sizes["noise"][1] * 1.003 + 100
    import numpy as np
    with pytest.raises(rt.RtError):
        debug_png_host(np.zeros(12, np.uint8).tobytes(), 0, 4)


def test_device_png_encoder_filters_and_blocks(rt):
    """The encoder's row filters follow libpng's min-sum choice and its blocks
    are the kinds the design says (a gradient picks Sub/Up/Paeth, a flat frame
    is one run per segment)."""
    import struct
    import zlib
    from raytracer_amd.png import debug_png_host
    for name, px in _png_frames():
        h, w, _ = px.shape
        png = debug_png_host(px.tobytes(), w, h)
        pos, idat = 8, b""
        while pos < len(png):
            (n,) = struct.unpack(">I", png[pos:pos + 4])
            if png[pos + 4:pos + 8] == b"IDAT":
                idat += png[pos + 8:pos + 8 + n]
            pos += 12 + n
        assert idat[:2] == b"\x78\x01"
        raw = zlib.decompress(idat)
        ftypes = {raw[y * (3 * w + 1)] for y in range(h)}
        assert ftypes <= {0, 1, 2, 3, 4}
        if name == "gradient":
            assert ftypes - {0}, "a gradient should pick a predicting filter"


def test_pass_plan_caps_items_at_the_counter_headroom(rt):
    """a record budget past the int32 hand-out counter's headroom gives more,
    bounded passes instead of the 'chunked pass too large' error (rt_api.cpp pass_units).
    Config 5 (4096^2, spp 1024: 262,144 tiles; a 1-sample-chunk schedule numbers up to 1,024
    items per slot) at the 32 GB budget that failed in round 4 (profiles/r04/sbuf/)."""
    from raytracer_amd import _lib
    lib = _lib.load()
    cap = (1 << 31) - (1 << 22)

    def plan(units, slots, chunks, rec, budget):
        out = ctypes.c_int64(0)
        _lib.check(lib.rt_debug_pass_plan(units, slots, chunks, rec, budget, ctypes.byref(out)))
        return out.value

    tiles, spp = 4096 * 4096 // 64, 1024
    rec_tile = 64 * spp * 12
    for chunks in (spp, 600, 64):
        for budget_mb in (8192, 32768, 1 << 20):
            per = plan(tiles, 64, chunks, rec_tile, budget_mb << 20)
            assert 1 <= per <= tiles
            assert per * 64 * chunks < cap                      # every pass fits the counter
            assert per <= max(1, (budget_mb << 20) // rec_tile)  # and the record budget
            passes = -(-tiles // per)
            assert passes * per >= tiles
    # the budget that fit in round 4 still gives the same pass (8 GB: 10,922 tiles, 25 passes)
    assert plan(tiles, 64, spp, rec_tile, 8192 << 20) == (8192 << 20) // rec_tile
    # past the headroom the counter, not the budget, sizes the pass
    big = plan(tiles, 64, spp, rec_tile, 32768 << 20)
    assert big == (cap - 1) // (64 * spp) < (32768 << 20) // rec_tile
    # a small launch takes one pass; a budget below one unit still makes progress
    assert plan(10, 64, 16, 1000, 1 << 30) == 10
    assert plan(10, 64, 16, 1 << 20, 1) == 1
    with pytest.raises(_lib.RtError):
        plan(10, 0, 16, 1000, 1 << 30)
