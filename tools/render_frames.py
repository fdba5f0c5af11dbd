#!/usr/bin/env python3
"""A few device-resident frames of one bench configuration, nothing else (no oracle, no counters):
the program rocprofv3's PC sampling / counter passes run, so the profile holds only the path kernel
and its accumulate pass.  usage: python tools/render_frames.py [--scene cornell] [--width 800]
[--spp 256] [--depth 16] [--frames 3] [--adaptive]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=16)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--adaptive", action="store_true")
    a = ap.parse_args()
    import torch
    from bench import SCENES
    import raytracer_amd as rt
    cfg, extra, _ = SCENES[a.scene]
    ro = {"width": a.width, "samples": a.spp, "depth": a.depth,
          **({"aTolerance": 0.05, "aBatch": 10} if a.adaptive else {"aTolerance": 0}), **extra}
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), ro)
    frame = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
    for f in range(a.frames):
        cam.render_device(rgb_ptr=frame.data_ptr(), synchronize=True)
        print(f"frame {f}: path / accumulate ms {cam.kernel_times()}", flush=True)


if __name__ == "__main__":
    main()
