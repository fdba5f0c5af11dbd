#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: time one rank's share of the headline
render (tile_group 0 of N, exactly what rank 0 runs under bench.py --gpus N,
minus the RCCL reduce) for N = 1, 2, 4, 8. Prints per-N ms and the implied
efficiency T(1) / (N * T(N)) of the render part."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import raytracer_amd as rt
    from bench import SCENES
    scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
    extra = {"cornell": {"width": 800, "samples": 256, "depth": 16},
             "spheres": {"width": 800, "samples": 64, "depth": 8},
             "rain": {"width": 1920, "samples": 512, "depth": 16}}[scene]
    cfg, ex, _ = SCENES[scene]
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**extra, **ex, "aTolerance": 0})
    H, W = cam.image_height, cam.image_width
    frame = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    base = None
    for n in (1, 2, 4, 8):
        def step():
            frame.zero_()
            cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=n, stream=s)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        base = base or ms
        step()
        kt = cam.kernel_times()
        print(json.dumps({"scene": scene, "n": n, "rank0_ms": round(ms, 3), "path_kernel_ms": round(kt[0], 3),
                          "accum_kernel_ms": round(kt[1], 3),
                          "efficiency_vs_n1": round(base / (n * ms), 4)}), flush=True)


if __name__ == "__main__":
    main()
