#!/usr/bin/env python3
"""Adaptive-sampling round schedule sweep (RT_AMD_ADAPT_FIRST / RT_AMD_ADAPT_GROW):
frame time, rounds and speculative samples per scene, plus the sequential kernel."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from bench import SCENES
    import raytracer_amd as rt

    cfgs = [("cornell", 800, 256, 16), ("spheres", 800, 64, 8), ("rain", 1920, 128, 16), ("default", 800, 64, 16)]
    arms = [("seq", {"RT_AMD_ADAPT_ROUNDS": "0"})] + [
        (f"f{f}g{g}", {"RT_AMD_ADAPT_FIRST": str(f), "RT_AMD_ADAPT_GROW": str(g)})
        for f in (10, 20, 40) for g in (2, 3)]
    if len(sys.argv) > 1:
        cfgs = [c for c in cfgs if c[0] in sys.argv[1:]]
    for scene, width, spp, depth in cfgs:
        cfg, extra, _ = SCENES[scene]
        sd = rt.generate_scene_data(cfg)
        for name, env in arms:
            for k in ("RT_AMD_ADAPT_ROUNDS", "RT_AMD_ADAPT_FIRST", "RT_AMD_ADAPT_GROW"):
                os.environ.pop(k, None)
            os.environ.update(env)
            cam = rt.create_camera_from_scene_data(sd, {"width": width, "samples": spp, "depth": depth, **extra})
            W, H = cam.image_width, cam.image_height
            buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
            st, _ = cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True)
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True)
                ts.append(time.perf_counter() - t0)
            rounds, rendered = cam.adaptive_info()
            ms = sorted(ts)[1] * 1e3
            kept = st.samples["total"]
            print(json.dumps({"scene": scene, "arm": name, "ms": round(ms, 3), "kernel": cam.last_kernel(),
                              "rounds": rounds, "kept": int(kept), "rendered": rendered,
                              "msamples_per_s": round(kept / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
