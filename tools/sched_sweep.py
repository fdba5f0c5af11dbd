#!/usr/bin/env python3
"""Hand-out sweep for the path kernel: rank 0's share (tile group 0 of N) of a bench
scene under RT_AMD_POOL (tile-chunks per atomic) x RT_AMD_CHUNK (first-phase chunk)
overrides, path-kernel ms from HIP events (median of 4)."""
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
    scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
    extra = {"cornell": {"width": 800, "samples": 256, "depth": 16},
             "spheres": {"width": 800, "samples": 64, "depth": 8},
             "rain": {"width": 1920, "samples": 512, "depth": 16},
             "spheres100k": {"width": int(os.environ.get("SWEEP_W", "2048")), "samples": 64, "depth": 100}}[scene]
    cfg, ex, _ = SCENES[scene]
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**extra, **ex, "aTolerance": 0})
    frame = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    pools = os.environ.get("SWEEP_POOL", "auto 1 2 4").split()
    chunks = os.environ.get("SWEEP_CHUNK", "auto 8 16 32").split()
    for n in [int(x) for x in os.environ.get("SWEEP_N", "1 2 8").split()]:
        for pool, chunk in itertools.product(pools, chunks):
            for k, v in (("RT_AMD_POOL", pool), ("RT_AMD_CHUNK", chunk)):
                if v == "auto":
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            kt = []
            for r in range(6):
                cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=n, stream=s)
                if r >= 2:
                    kt.append(cam.kernel_times()[0])
            print(json.dumps({"scene": scene, "n": n, "pool": pool, "chunk": chunk,
                              "path_ms": round(float(np.median(kt)), 4), "kernel": cam.last_kernel()}), flush=True)


if __name__ == "__main__":
    main()
