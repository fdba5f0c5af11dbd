#!/usr/bin/env python3
"""Diagnostic: wave-cycle breakdown of the path loop by section (count_work="profile").

Runs the section-timing build (INSTR == 2) once per configuration and prints each
section's share of the summed wave-cycles, plus wall time of the product build.
"""
import os
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from bench import SCENES
    from raytracer_amd import _build
    _build.build_native()
    import raytracer_amd as rt

    cfgs = [("cornell", 800, 256, 16, "ref", "auto"), ("cornell", 800, 256, 16, "ref", "fast"),
            ("cornell", 800, 256, 16, "fp32", "auto"), ("spheres", 800, 64, 8, "ref", "auto"),
            ("rain", 1920, 64, 16, "ref", "auto"), ("spheres100k", 1024, 4, 100, "ref", "auto")]
    if len(sys.argv) > 1:
        cfgs = [c for c in cfgs if c[0] in sys.argv[1:]]
    if os.environ.get("RT_SECTIONS_ONLY"):  # e.g. "ref auto": only the configs of that precision / traversal
        prec, trav = os.environ["RT_SECTIONS_ONLY"].split()
        cfgs = [c for c in cfgs if c[4] == prec and c[5] == trav]
    for scene, width, spp, depth, prec, trav in cfgs:
        cfg, extra, _ = SCENES[scene]
        sd = rt.generate_scene_data(cfg)
        cam = rt.create_camera_from_scene_data(sd, {"width": width, "samples": spp, "depth": depth, "aTolerance": 0,
                                                    "precision": prec, "traversal": trav, **extra})
        W, H = cam.image_width, cam.image_height
        buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
        cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True)
        wall = time.perf_counter() - t0
        _, sec = cam.render_device(rgb_ptr=buf.data_ptr(), synchronize=True, count_work="profile")
        parts = {k: v for k, v in sec.items() if k not in ("loop", "trips") and not k.startswith(("lanes_", "execs_"))}
        life = sec["loop"]  # summed wave lifetimes (wave-view profiler: sections sum to it)
        lanes = {k[6:]: round(v / max(sec["execs_" + k[6:]], 1), 1) for k, v in sec.items() if k.startswith("lanes_")}
        execs = {k[6:]: round(v * 64 / (W * H * spp), 3) for k, v in sec.items() if k.startswith("execs_")}
        tot = sum(parts.values())
        line = {"cfg": f"{scene} {W}x{H} spp{spp} d{depth} {prec} {trav}", "wall_ms": round(wall * 1e3, 2),
                "trips_per_sample": round(sec["trips"] * 64 / (W * H * spp), 3),
                "share": {k: round(v / tot, 4) for k, v in parts.items()},
                "sections_vs_lifetime": round(tot / max(life, 1), 4),
                "active_lanes_per_exec": lanes, "wave_execs_per_64_samples": execs}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
