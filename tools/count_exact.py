#!/usr/bin/env python3
"""Diagnostic: work counters of the fast/brute strategies (exact-test counts per ray, per wave-trip)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from bench import SCENES
    import raytracer_amd as rt
    cfgs = [("cornell", 800, 64, 16, "brute"), ("cornell", 800, 64, 16, "fast"),
            ("spheres", 800, 16, 8, "fast"), ("rain", 1920, 16, 16, "fast"), ("spheres100k", 1024, 4, 100, "fast")]
    if len(sys.argv) > 1:
        cfgs = [c for c in cfgs if c[0] in sys.argv[1:]]
    for scene, width, spp, depth, trav in cfgs:
        cfg, extra, _ = SCENES[scene]
        cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {
            "width": width, "samples": spp, "depth": depth, "aTolerance": 0, "traversal": trav, **extra})
        buf = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
        _, c = cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True, count_work=True)
        rays = max(c["rays"], 1)
        print(json.dumps({"cfg": f"{scene} {trav}", "per_ray": {k: round(v / rays, 3) for k, v in c.items()},
                          "exact_wave_per_ray_x64": round(64 * c["exact_wave"] / rays, 3)}), flush=True)


if __name__ == "__main__":
    main()
