"""Debug: adaptive rounds vs the sequential kernel on the golden adaptive case."""
import os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
import numpy as np
import torch
import raytracer_amd as rt

sd = rt.generate_scene_data({"type": "cornell"})
for ro in [{"width": 24, "samples": 40, "depth": 8}, {"width": 24, "samples": 40, "depth": 8, "aTolerance": 0.5}]:
    res = {}
    for env in [("seq", {"RT_AMD_ADAPT_ROUNDS": "0"}), ("pool", {}), ("chunked", {"RT_AMD_POOL_KERNEL": "0"}),
                ("first40", {"RT_AMD_ADAPT_FIRST": "40"}), ("first10", {"RT_AMD_ADAPT_FIRST": "10"})]:
        for k in ("RT_AMD_ADAPT_ROUNDS", "RT_AMD_POOL_KERNEL", "RT_AMD_ADAPT_FIRST"):
            os.environ.pop(k, None)
        os.environ.update(env[1])
        cam = rt.create_camera_from_scene_data(sd, ro)
        W, H = cam.image_width, cam.image_height
        rgb = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
        rad = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
        pxs = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        pxb = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        st, _ = cam.render_device(rgb_ptr=rgb.data_ptr(), radiance_ptr=rad.data_ptr(), px_samples_ptr=pxs.data_ptr(),
                                  px_bounces_ptr=pxb.data_ptr(), synchronize=True)
        res[env[0]] = (rad.cpu().numpy(), pxs.cpu().numpy(), pxb.cpu().numpy(), cam.last_kernel(), cam.pass_count(), st)
    base = res["seq"]
    print("ro", ro, "seq samples hist", np.unique(base[1], return_counts=True))
    for k, v in res.items():
        d = (v[0] != base[0]).any(-1)
        ds = v[1] != base[1]
        print(k, v[3], "passes", v[4], "rad diff px", int(d.sum()), "samples diff", int(ds.sum()),
              "bounce diff", int((v[2] != base[2]).sum()), "stats", v[5].samples, flush=True)
        if d.sum():
            ys, xs = np.nonzero(d)
            for y, x in list(zip(ys, xs))[:8]:
                print("   px", (x, y), "n seq", base[1][y, x], "n", v[1][y, x], "b seq", base[2][y, x], "b", v[2][y, x])
