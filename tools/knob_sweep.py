#!/usr/bin/env python3
"""Runtime-knob sweep of one rank's share (tile group 0 of N) of a bench scene:
path-kernel ms from HIP events (median of 5 after 2 warm-up renders) per arm.
Arms come from $ARMS, one per line: "<name> [KEY=VALUE ...]" (env knobs read at
each launch, e.g. RT_AMD_READY, RT_AMD_POOL, RT_AMD_CHUNK, RT_AMD_REFILL).
usage: ARMS=... SWEEP_N="1 8" [SWEEP_SPP=32] python tools/knob_sweep.py <scene>"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))

RO = {"cornell": {"width": 800, "samples": 256, "depth": 16}, "spheres": {"width": 800, "samples": 64, "depth": 8},
      "rain": {"width": 1920, "samples": 512, "depth": 16},
      "spheres100k": {"width": 4096, "samples": 16, "depth": 100}}


def main():
    import numpy as np
    import torch
    import raytracer_amd as rt
    from bench import SCENES
    scene = sys.argv[1]
    cfg, ex, _ = SCENES[scene]
    ro = dict(RO[scene])
    if os.environ.get("SWEEP_SPP"):  # e.g. 32: one pass of config 5 (spp 1024 in passes of 32)
        ro["samples"] = int(os.environ["SWEEP_SPP"])
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**ro, **ex, "aTolerance": 0})
    frame = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    arms = [ln.split() for ln in os.environ.get("ARMS", "base").splitlines() if ln.strip()]
    knobs = sorted({kv.split("=")[0] for arm in arms for kv in arm[1:]})
    for n in [int(x) for x in os.environ.get("SWEEP_N", "1 8").split()]:
        for arm in arms:
            for k in knobs:
                os.environ.pop(k, None)
            for kv in arm[1:]:
                k, v = kv.split("=", 1)
                os.environ[k] = v
            kt = []
            for r in range(7):
                cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=n, stream=s)
                if r >= 2:
                    kt.append(cam.kernel_times()[0])
            print(json.dumps({"scene": scene, "n": n, "arm": arm[0], "path_ms": round(float(np.median(kt)), 4),
                              "min_ms": round(float(min(kt)), 4), "kernel": cam.last_kernel()}), flush=True)


if __name__ == "__main__":
    main()
