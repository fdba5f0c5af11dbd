"""Single-process multi-GPU entry of the C ABI (rt_camera_render_multi / _png_multi).

The reference's parallel render is one process driving N workers over row bands of one
buffer, merging their RenderStats (src/raytracer.ts:60-90,185-205,
src/render-utils/renderWorker.ts:17-35, src/render-utils/renderStats.ts:42-64). The C ABI's
counterpart renders tile groups on N devices from one call and gathers them on devices[0]
(RCCL for distinct devices, device-to-device copies when a device is listed more than once).
The path RNG is keyed by (pixel, sample), so every split must equal one single-device launch
bit for bit, and that launch equals the oracle (test_gpu_parity.py); the n = 1 case is also
checked against the oracle directly. On the 1-GPU test box, lists that repeat device 0 rehearse
the N-way split (peer transport); on a multi-GPU node the all-devices case takes RCCL.
"""
import numpy as np
import pytest

from test_gpu_parity import NOADAPT, _cfgs, _mixed_scene, assert_identical

pytestmark = pytest.mark.gpu


def _single(rt, sd, ro, region=None):
    cam = rt.create_camera_from_scene_data(sd, ro)
    W, H = cam.image_width, cam.image_height
    rgb = np.zeros((H, W, 3), np.uint8)
    rad = np.zeros((H, W, 3), np.float32)
    st = cam.render_region(rgb, region or (0, 0, W, H), radiance=rad)
    return rgb, rad, st


def _multi(rt, sd, ro, devices, region=None, radiance=True):
    cam = rt.create_camera_from_scene_data(sd, ro)
    W, H = cam.image_width, cam.image_height
    rgb = np.zeros((H, W, 3), np.uint8)
    rad = np.zeros((H, W, 3), np.float32) if radiance else None
    st = cam.render_region_multi(rgb, region or (0, 0, W, H), devices, radiance=rad)
    return cam, rgb, rad, st


def _stats_equal(a, b):
    assert a.pixels == b.pixels
    assert a.samples == b.samples and a.bounces == b.bounces


def test_render_multi_one_device_matches_oracle_and_single_launch(rt, oracle, gpu):
    """n = 1 through the whole multi path (slab render, stats words in the spare tile, RCCL
    send / recv to itself on a one-rank communicator, unpack, merge) against the oracle."""
    sd = rt.generate_scene_data({"type": "cornell"})
    ro = {"width": 40, "samples": 12, "depth": 16, **NOADAPT}
    cam, rgb, rad, st = _multi(rt, sd, ro, [0])
    orc = oracle.render(sd, ro)
    assert_identical(rad, rgb, orc["radiance"], orc["rgb"], "multi [0] vs oracle")
    assert st.pixels == orc["stats"]["pixels"]
    for k in ("total", "min", "max"):
        assert st.samples[k] == orc["stats"]["samples"][k] and st.bounces[k] == orc["stats"]["bounces"][k]
    info = cam.multi_info()
    assert info["n_devices"] == 1 and info["devices"] == [0] and info["transport"] == "rccl"
    assert info["path_ms"][0] > 0 and info["gather_ms"] > 0
    rgb1, rad1, st1 = _single(rt, sd, ro)
    assert_identical(rad, rgb, rad1, rgb1, "multi [0] vs single launch")
    _stats_equal(st, st1)


@pytest.mark.parametrize("name", ["cornell", "spheres", "rain", "default", "mixed"])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_render_multi_split_equals_single_launch(rt, gpu, name, n):
    """The N-way split rehearsed on device 0 (listed n times: n contexts, n streams, n host
    threads, peer gather) equals one launch for every scene class - brute force (pool kernel),
    LDS-resident BVH, tiny BVH, the default scene (plane, layered, sphere light, aperture) and
    a custom mixed / layered / emissive-mixed scene."""
    if name == "mixed":
        sd, ro = _mixed_scene(), {"width": 40, "samples": 8, "depth": 12, **NOADAPT}
    else:
        cfg, ro = _cfgs()[name]
        sd = rt.generate_scene_data(cfg)
    cam, rgb, rad, st = _multi(rt, sd, ro, [0] * n)
    rgb1, rad1, st1 = _single(rt, sd, ro)
    assert_identical(rad, rgb, rad1, rgb1, f"{name} multi x{n} vs single")
    _stats_equal(st, st1)
    info = cam.multi_info()
    assert info["n_devices"] == n and info["transport"] == "peer"
    assert sum(1 for t in info["path_ms"] if t > 0) >= 1


def test_render_multi_regions_and_buffers(rt, gpu):
    """A region (only its pixels written, the rest of the caller's buffer untouched), no
    radiance buffer, more devices than tiles (empty tile groups) and a region off the image."""
    sd = rt.generate_scene_data({"type": "cornell"})
    ro = {"width": 48, "samples": 6, "depth": 8, **NOADAPT}
    region = (5, 9, 27, 30)
    cam = rt.create_camera_from_scene_data(sd, ro)
    W, H = cam.image_width, cam.image_height
    rgb = np.full((H, W, 3), 7, np.uint8)
    st = cam.render_region_multi(rgb, region, [0, 0, 0])
    rgb1 = np.full((H, W, 3), 7, np.uint8)
    rad1 = np.zeros((H, W, 3), np.float32)
    st1 = cam.render_region(rgb1, region, radiance=rad1)
    assert np.array_equal(rgb, rgb1)
    _stats_equal(st, st1)
    outside = np.ones((H, W), bool)
    outside[9:39, 5:32] = False
    assert (rgb[outside] == 7).all()
    # a 1-tile region over 5 devices: four render nothing (stats of no pixels merge away)
    rgb2 = np.zeros((H, W, 3), np.uint8)
    st2 = cam.render_region_multi(rgb2, (8, 8, 8, 8), [0] * 5)
    rgb3 = np.zeros((H, W, 3), np.uint8)
    st3 = cam.render_region(rgb3, (8, 8, 8, 8))
    assert np.array_equal(rgb2, rgb3)
    _stats_equal(st2, st3)
    # a region entirely off the image: nothing rendered, nothing written
    rgb4 = np.zeros((H, W, 3), np.uint8)
    st4 = cam.render_region_multi(rgb4, (W + 4, 0, 8, 8), [0, 0])
    assert st4.pixels == 0 and not rgb4.any()


def test_render_multi_adaptive_and_fp32(rt, gpu):
    """Adaptive sampling (the reference default: rounds that wait on the host, one thread per
    device) and fp32 precision through the split."""
    sd = rt.generate_scene_data({"type": "cornell"})
    for ro in ({"width": 40, "samples": 40, "depth": 16},  # adaptive defaults
               {"width": 40, "samples": 16, "depth": 16, "precision": "fp32", **NOADAPT}):
        cam, rgb, rad, st = _multi(rt, sd, ro, [0, 0, 0, 0])
        rgb1, rad1, st1 = _single(rt, sd, ro)
        assert_identical(rad, rgb, rad1, rgb1, f"multi x4 {ro}")
        _stats_equal(st, st1)


def test_render_multi_all_visible_devices(rt, gpu):
    """Every visible GPU once (RCCL over xGMI on a multi-GPU node; one rank here)."""
    sd = rt.generate_scene_data({"type": "spheres", "options": {"count": 500, "seed": 42}})
    ro = {"width": 96, "aspect": 1, "samples": 8, "depth": 8, **NOADAPT}
    devs = list(range(gpu))
    cam, rgb, rad, st = _multi(rt, sd, ro, devs)
    rgb1, rad1, st1 = _single(rt, sd, ro)
    assert_identical(rad, rgb, rad1, rgb1, f"multi {devs}")
    _stats_equal(st, st1)
    assert cam.multi_info()["transport"] == "rccl"
    # repeated renders reuse every device's scene, stream and slabs
    st2 = cam.render_region_multi(rgb, (0, 0, cam.image_width, cam.image_height), devs, radiance=rad)
    assert_identical(rad, rgb, rad1, rgb1, f"multi {devs} again")
    _stats_equal(st2, st1)


def test_render_png_multi_equals_single_device_png(rt, gpu):
    """generateImageBuffer over N devices: the same frame, so the same PNG bytes and stats."""
    sd = rt.generate_scene_data({"type": "cornell"})
    ro = {"width": 64, "samples": 8, "depth": 8, **NOADAPT}
    cam = rt.create_camera_from_scene_data(sd, ro)
    png1, st1 = cam.render_png(1)
    png, st = cam.render_png_multi([0, 0])
    assert png == png1
    _stats_equal(st, st1)
    png2, _ = cam.render_png_multi(list(range(gpu)))
    assert png2 == png1


def test_render_multi_errors(rt, gpu, monkeypatch):
    sd = rt.generate_scene_data({"type": "cornell"})
    cam = rt.create_camera_from_scene_data(sd, {"width": 16, "samples": 2, "depth": 4, **NOADAPT})
    buf = np.zeros((16, 16, 3), np.uint8)
    with pytest.raises(rt.RtError, match="not visible"):
        cam.render_multi(buf, [gpu])
    with pytest.raises(rt.RtError):
        cam.render_multi(buf, [])
    monkeypatch.setenv("RT_AMD_GATHER", "rccl")
    with pytest.raises(rt.RtError, match="distinct"):
        cam.render_multi(buf, [0, 0])
    monkeypatch.delenv("RT_AMD_GATHER")
    # the reference's render error (a miss without a background) surfaces from any device
    del sd["camera"]["background"]
    cam2 = rt.create_camera_from_scene_data(sd, {"width": 16, "samples": 2, "depth": 4, **NOADAPT})
    with pytest.raises(rt.RtError, match="reading 'top'"):
        cam2.render_multi(buf, [0, 0])
    # and the camera stays usable: single-device renders after a multi one
    st = cam.render(buf)
    assert st.pixels == 256 and cam.multi_info()["n_devices"] == 0
