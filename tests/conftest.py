import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def rt():
    from raytracer_amd import _build
    _build.build_native()
    import raytracer_amd
    return raytracer_amd


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def gpu(rt):
    n = rt.device_count()
    if n < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    return n
