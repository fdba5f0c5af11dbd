#!/usr/bin/env python3
"""Schedule-knob sweep for the chunked path kernel: a bench scene rendered under every
combination of environment overrides, path-kernel ms from HIP events (median of 4).

    SWEEP_VARS="RT_AMD_READY=32,48,56 RT_AMD_REFILL=1,4" python tools/env_sweep.py spheres100k

SWEEP_TG=N renders rank 0's share (tile group 0 of N) instead of the whole frame.
"""
import itertools
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch
    import raytracer_amd as rt
    from bench import SCENES
    scene = sys.argv[1] if len(sys.argv) > 1 else "spheres100k"
    spp = int(os.environ.get("SWEEP_SPP", "64"))
    extra = {"cornell": {"width": 800, "samples": 256, "depth": 16},
             "spheres": {"width": 800, "samples": 64, "depth": 8},
             "rain": {"width": 1920, "samples": 512, "depth": 16},
             "spheres100k": {"width": int(os.environ.get("SWEEP_W", "4096")), "samples": spp, "depth": 100}}[scene]
    cfg, ex, _ = SCENES[scene]
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**extra, **ex, "aTolerance": 0})
    frame = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    axes = []
    for spec in os.environ.get("SWEEP_VARS", "RT_AMD_READY=48").split():
        k, vals = spec.split("=", 1)
        axes.append([(k, v) for v in vals.split(",")])
    tg = int(os.environ.get("SWEEP_TG", "1"))
    ref = None
    for combo in itertools.product(*axes):
        for k, v in combo:
            if v == "auto":
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        kt = []
        for r in range(6):
            cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=tg, stream=s)
            if r >= 2:
                kt.append(sum(cam.kernel_times()))
        torch.cuda.synchronize()
        img = frame.cpu().numpy()
        ref = img if ref is None else ref
        print(json.dumps({"scene": scene, "tile_groups": tg, **dict(combo), "ms": round(float(np.median(kt)), 3),
                          "same_image": bool((img == ref).all()), "kernel": cam.last_kernel()}), flush=True)


if __name__ == "__main__":
    main()
