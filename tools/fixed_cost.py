#!/usr/bin/env python3
"""Per-launch fixed cost of the chunked/pool path kernel: rank 0's share of the
headline render for N = 1 .. 256 tile groups (path kernel ms from HIP events),
plus spp sweeps of a single tile (minimal launches). Fits T(N) = a + b / N."""
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
             "spheres": {"width": 800, "samples": 64, "depth": 8}}[scene]
    cfg, ex, _ = SCENES[scene]
    sd = rt.generate_scene_data(cfg)
    cam = rt.create_camera_from_scene_data(sd, {**extra, **ex, "aTolerance": 0})
    H, W = cam.image_height, cam.image_width
    frame = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ns, ts = [], []
    for n in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        kt = []
        for r in range(6):
            cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=n, stream=s)
            if r >= 2:
                kt.append(cam.kernel_times()[0])
        t = float(np.median(kt))
        ns.append(n)
        ts.append(t)
        print(json.dumps({"scene": scene, "n": n, "path_ms": round(t, 4), "kernel": cam.last_kernel()}), flush=True)
    A = np.stack([np.ones(len(ns)), 1.0 / np.array(ns)], 1)
    (a, b), *_ = np.linalg.lstsq(A[3:], np.array(ts[3:]), rcond=None)
    print(json.dumps({"fit_n_ge_8": {"a_ms": round(float(a), 4), "b_ms": round(float(b), 3)}}), flush=True)
    for spp in (1, 4, 16, 64):
        c1 = rt.create_camera_from_scene_data(sd, {**extra, **ex, "aTolerance": 0, "samples": spp})
        kt = []
        for r in range(6):
            c1.render_device(rgb_ptr=frame.data_ptr(), region=(400, 400, 8, 8), stream=s)
            if r >= 2:
                kt.append(c1.kernel_times()[0])
        print(json.dumps({"scene": scene, "one_tile_spp": spp, "path_ms": round(float(np.median(kt)), 4),
                          "kernel": c1.last_kernel()}), flush=True)


if __name__ == "__main__":
    main()
