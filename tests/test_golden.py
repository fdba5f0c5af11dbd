"""Golden fixtures (tests/golden/, made by make_golden.py from the oracle).

CPU: the oracle and the generators reproduce their committed outputs.
GPU: the HIP path reproduces the committed oracle images.
"""
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
IMAGES = sorted(p.stem for p in GOLDEN.glob("*.npz"))
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
    eq = float((rgb == z["rgb"]).all(axis=-1).mean())
    close = float(np.isclose(rad, z["radiance"], rtol=1e-6, atol=1e-6, equal_nan=True).all(axis=-1).mean())
    print(f"{name}: rgb equal {eq:.5f} radiance equal {close:.5f}")
    assert eq >= 0.995 and close >= 0.995
