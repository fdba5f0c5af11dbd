"""Scene construction: SceneConfig -> SceneData -> Camera.

Mirrors src/scenes/scenes.ts: SceneConfig (29-34), generateSceneData (42-50),
generateScene (52-55) and createCameraFromSceneData (60-104). The generators
themselves (spheres / rain / cornell / default) run in the native library so
the benchmark inputs are produced by the same code on every host.
"""
from __future__ import annotations

import ctypes as C
import json
from typing import Optional

from . import _lib
from .camera import Camera

SCENE_TYPES = ("default", "spheres", "rain", "cornell", "custom")


def generate_scene_data(scene_config: dict) -> dict:
    """generateSceneData(sceneConfig) (src/scenes/scenes.ts:42-50)."""
    t = scene_config.get("type", "default")
    if t == "custom":
        return scene_config["data"]
    if t not in SCENE_TYPES:
        raise _lib.RtError(_lib.RT_ERR_INVALID, f"Unknown scene type: {t}")
    opts = scene_config.get("options")
    out = C.c_void_p()
    lib = _lib.load()
    _lib.check(lib.rt_generate_scene_data(t.encode(), _lib.to_json(opts) if opts is not None else None,
                                          C.byref(out)))
    try:
        text = C.string_at(out).decode()
    finally:
        lib.rt_free(out)
    return json.loads(text, parse_constant=lambda c: float(c.replace("Infinity", "inf")))


def create_camera_from_scene_data(scene_data: dict, render_options: Optional[dict] = None) -> Camera:
    """createCameraFromSceneData(sceneData, renderOptions) (src/scenes/scenes.ts:60-104)."""
    ro = None
    if render_options is not None:
        ro = _lib.to_json({k: v for k, v in render_options.items() if v is not None})
    return Camera(_lib.to_json(scene_data), ro)


def generate_scene(scene_config: dict) -> Camera:
    """generateScene(sceneConfig) (src/scenes/scenes.ts:52-55)."""
    return create_camera_from_scene_data(generate_scene_data(scene_config), scene_config.get("render"))


# Reference spellings
generateSceneData = generate_scene_data
createCameraFromSceneData = create_camera_from_scene_data
generateScene = generate_scene
