#!/usr/bin/env python3
"""Where a launch's tail goes: per-wave start / hand-out-dry / end times of one render.

Needs the diagnostic variant library built from a tree with tools/wave_probe.patch applied
(the probe is not in the product kernel) and RT_WAVE_PROBE=1 (run with
RT_AMD_VARIANT=<its name>): every wave of a chunked / pool launch records the 100 MHz real-time
clock at its start, when the item hand-out ran dry for it, and at its end, plus its item count
and hardware ids (pt_kernel.hpp WaveProbe). For each scene and tile-group count N it renders
tile group 0 of N (rank 0's share under bench.py --gpus N, as tools/rank_share.py) and prints
the launch span, the percentiles of the waves' dry and end times, the drain (end - dry) and the
last waves.

usage: RT_AMD_VARIANT=wprobe python tools/wave_probe.py [cornell|spheres|rain ...]
"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))

EXTRA = {"cornell": {"width": 800, "samples": 256, "depth": 16},
         "spheres": {"width": 800, "samples": 64, "depth": 8},
         "rain": {"width": 1920, "samples": 512, "depth": 16}}
SLOTS = 8192  # pt_kernel.hpp kWaveProbeSlots
TICK_US = 0.01  # s_memrealtime: 100 MHz


def probe(lib, fn):
    lib.rt_debug_wave_probe(None, 0, 1)
    fn()
    buf = (ctypes.c_ulonglong * (SLOTS * 4))()
    if lib.rt_debug_wave_probe(buf, SLOTS * 4, 0) != 0:
        raise SystemExit("rt_debug_wave_probe failed (is RT_AMD_VARIANT a RT_WAVE_PROBE=1 build?)")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(SLOTS, 4)
    a = a[a[:, 0] != 0]
    t0 = a[:, 0].astype(np.int64)
    base = t0.min()
    start = (t0 - base) * TICK_US
    dry = (a[:, 1].astype(np.int64) - base) * TICK_US
    end = (a[:, 2].astype(np.int64) - base) * TICK_US
    items = (a[:, 3] >> np.uint64(32)).astype(np.int64)
    xcc = ((a[:, 3] >> np.uint64(28)) & np.uint64(0xF)).astype(np.int64)
    hw = (a[:, 3] & np.uint64(0x0FFFFFFF)).astype(np.int64)
    return start, dry, end, items, xcc, hw


def pct(x):
    return {p: round(float(np.percentile(x, p)), 1) for p in (0, 10, 50, 90, 99, 100)}


def main():
    import torch
    import raytracer_amd as rt
    from raytracer_amd import _lib
    from bench import SCENES
    lib = _lib.load()
    lib.rt_debug_wave_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.rt_debug_wave_probe.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    for scene in sys.argv[1:] or ["cornell", "spheres"]:
        cfg, ex, _ = SCENES[scene]
        cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**EXTRA[scene], **ex, "aTolerance": 0})
        H, W = cam.image_height, cam.image_width
        frame = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
        for n in (1, 8):
            def render():
                cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=0, tile_groups=n, synchronize=True)
            render()
            render()
            start, dry, end, items, xcc, hw = probe(lib, render)
            kt = cam.kernel_times()
            span = float(end.max())
            drain = end - dry
            order = np.argsort(end)[::-1][:8]
            print(json.dumps({
                "scene": scene, "n": n, "waves": int(len(end)), "path_kernel_ms": round(kt[0], 4),
                "span_us": round(span, 1), "start_us": pct(start), "dry_us": pct(dry), "end_us": pct(end),
                "drain_us": pct(drain), "items": pct(items),
                "busy_frac": round(float((end - start).sum() / (len(end) * span)), 4),
                "last_waves": [{"end": round(float(end[i]), 1), "dry": round(float(dry[i]), 1),
                                "items": int(items[i]), "xcc": int(xcc[i]), "cu": int((hw[i] >> 8) & 0xF),
                                "se": int((hw[i] >> 13) & 0x7)} for i in order],
                "end_by_xcc_max": {int(x): round(float(end[xcc == x].max()), 1) for x in np.unique(xcc)},
            }), flush=True)
        cam.close()


if __name__ == "__main__":
    main()
