#!/usr/bin/env python3
"""Diagnostic: one rank's share (tile group 0 of N) of a bench scene under
different runtime knobs (env), to expose the critical-path tail of small
per-rank workloads. usage: tail_probe.py scene N [N ...]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import raytracer_amd as rt  # noqa: E402
from bench import SCENES  # noqa: E402

RO = {"cornell": {"width": 800, "samples": 256, "depth": 16}, "spheres": {"width": 800, "samples": 64, "depth": 8},
      "rain": {"width": 1920, "samples": 512, "depth": 16}}
scene = sys.argv[1]
cfg, ex, _ = SCENES[scene]
sd = rt.generate_scene_data(cfg)
cam = rt.create_camera_from_scene_data(sd, {**RO[scene], **ex, "aTolerance": 0})
H, W = cam.image_height, cam.image_width
f = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
for n in [int(x) for x in sys.argv[2:]]:
    for _ in range(2):
        cam.render_device(rgb_ptr=f.data_ptr(), tile_group=0, tile_groups=n, synchronize=True)
    t0 = time.perf_counter()
    for _ in range(5):
        cam.render_device(rgb_ptr=f.data_ptr(), tile_group=0, tile_groups=n, synchronize=True)
    ms = (time.perf_counter() - t0) / 5 * 1e3
    print(json.dumps({"scene": scene, "n": n, "ms": round(ms, 3), "kt": [round(x, 3) for x in cam.kernel_times()]}),
          flush=True)
