"""RCCL leg of the multi-GPU frame path on a one-GPU box (run as a child process by
tests/test_gpu_parity.py::test_rccl_gather_of_tile_groups_assembles_the_frame).

RCCL refuses two ranks on one device, so the gather is exercised at world size 1 over
the "nccl" (= RCCL) backend: the frame is split into `groups` tile groups as
`groups` ranks would render them (tile-packed u8 slabs + their spare stats tile,
distributed.render_frame's layout), each slab travels through a real RCCL
dist.gather into its row of the stacked buffer, rt_tiles_unpack assembles the frame
and the stats words merge as RenderStats.merge does. bench.py's timing reduction
(all_reduce MAX of a float64 pair) runs over RCCL too. Prints one JSON line.
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))


def main():
    import torch
    import torch.distributed as dist

    groups = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    scene = sys.argv[2] if len(sys.argv) > 2 else "cornell"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"

    import raytracer_amd as rt
    from raytracer_amd import distributed as rtd

    cfg = {"cornell": {"type": "cornell"}, "spheres": {"type": "spheres", "options": {"count": 500, "seed": 42}}}[scene]
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg),
                                           {"width": 72, "aspect": 1, "samples": 8, "depth": 8, "aTolerance": 0})
    W, H = cam.image_width, cam.image_height
    region = (0, 0, W, H)
    s = torch.cuda.current_stream(dev).cuda_stream
    n_tiles = rtd.slab_tiles(region, groups)
    n_px = n_tiles * rtd.TILE_PIXELS
    slabs = torch.zeros((groups, rtd.slab_pixels(region, groups), 3), dtype=torch.uint8, device=dev)
    gathered = torch.full_like(slabs, 0xAB)
    for g in range(groups):
        slab = slabs[g]
        cam.render_device(rgb_ptr=slab.data_ptr(), region=region, tile_group=g, tile_groups=groups, stream=s,
                          packed=True)
        cam.stats_words(slab.data_ptr() + n_px * 3, s)
        torch.cuda.current_stream(dev).synchronize()
        dist.gather(slab, gather_list=[gathered[g]], dst=0)  # RCCL, world size 1
    frame = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
    rtd.unpack_tiles(gathered, region, W, H, frame, s, slab_tiles=n_tiles + 1)
    merged = rtd.stats_from_words(rtd.gathered_stats(gathered, n_px).cpu().tolist())
    single = torch.zeros_like(frame)
    st1, _ = cam.render_device(rgb_ptr=single.data_ptr(), stream=s, synchronize=True)
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    same_stats = (merged.pixels == st1.pixels
                  and all(merged.samples[k] == st1.samples[k] for k in ("total", "min", "max"))
                  and all(merged.bounces[k] == st1.bounces[k] for k in ("total", "min", "max")))
    out = {"backend": dist.get_backend(), "groups": groups, "scene": scene,
           "slabs_equal_gathered": bool(torch.equal(slabs, gathered)),
           "frame_equal": bool(torch.equal(frame, single)), "stats_equal": bool(same_stats),
           "all_reduce": [float(v) for v in t.cpu()], "pixels": float(merged.pixels)}
    dist.destroy_process_group()
    cam.close()
    print(json.dumps(out))
    return 0 if out["slabs_equal_gathered"] and out["frame_equal"] and out["stats_equal"] else 1


if __name__ == "__main__":
    sys.exit(main())
