"""Golden fixtures (tests/golden/, made by make_golden.py from the oracle).

CPU: the oracle and the generators reproduce their committed outputs.
GPU: the HIP path reproduces the committed oracle images.
"""
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
IMAGES = sorted(p.stem for p in GOLDEN.glob("*.npz") if p.stem != "v8_math")
SCENES = sorted(p.stem for p in GOLDEN.glob("scene_*.json"))


def _load(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    return z, json.loads(str(z["scene"])), json.loads(str(z["render"]))


def test_golden_fixtures_present():
    assert len(IMAGES) >= 6 and len(SCENES) >= 4


@pytest.mark.parametrize("name", IMAGES)
def test_oracle_reproduces_golden(oracle, name):
    z, sd, ro = _load(name)
    out = oracle.render(sd, ro)
    assert np.array_equal(out["radiance"], z["radiance"], equal_nan=True)
    assert np.array_equal(out["rgb"], z["rgb"])


@pytest.mark.parametrize("name", SCENES)
def test_generator_reproduces_golden_scene(rt, name):
    d = json.loads((GOLDEN / f"{name}.json").read_text())
    assert rt.generate_scene_data(d["config"]) == d["scene"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", IMAGES)
def test_gpu_reproduces_golden(rt, gpu, name):
    z, sd, ro = _load(name)
    cam = rt.create_camera_from_scene_data(sd, ro)
    H, W = z["rgb"].shape[:2]
    rgb = np.zeros((H, W, 3), np.uint8)
    rad = np.zeros((H, W, 3), np.float32)
    cam.render(rgb, radiance=rad)
    # bit-identity: every pixel, u8 and fp32 radiance
    n_rgb = int((rgb != z["rgb"]).any(axis=-1).sum())
    n_rad = int((~((rad == z["radiance"]) | (np.isnan(rad) & np.isnan(z["radiance"])))).any(axis=-1).sum())
    print(f"{name}: pixels differing rgb {n_rgb}, radiance {n_rad}")
    assert n_rgb == 0 and n_rad == 0, (name, n_rgb, n_rad)
