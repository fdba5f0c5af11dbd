#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU (every tile group, not group 0 only).

For N = 1, 2, 4, 8, renders EVERY tile group g of N into its tile-packed slab exactly as rank g
runs it under `bench.py --gpus N` (distributed.render_frame: packed slab + spare stats tile) and
times each group; an N-GPU step lasts as long as the SLOWEST rank, so the projection is

    T(N) = max_g share(g) + gather(N slabs) + unpack(N slabs)

where `gather` is measured as N real `dist.gather` calls of one slab each over a world-size-1
"nccl" (= RCCL) group (RCCL refuses two ranks on one device). On the 8-GPU node the gather is ONE
call whose N - 1 remote slabs (frame / N bytes each: 240 KB for an 800^2 frame at N = 8, ~2 us on
one 150 GB/s xGMI link) arrive in parallel, so the N sequential calls - dominated by per-call
overhead - bound it from above; one world-1 collective over all N slabs is reported beside it
(`gather_one_call_ms`, `efficiency_one_call_gather`). `unpack` is
rt_tiles_unpack of the gathered [N, slab, 3] buffer into the frame. The reference's counterpart:
worker row bands, src/raytracer.ts:60-90,185-205. Prints one JSON line per N with the max / min
/ mean share, the projected step and its efficiency T(1) / (N T(N)).

usage: python tools/rank_share.py [cornell|spheres|rain ...]
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
sys.path.insert(0, str(ROOT))

EXTRA = {"cornell": {"width": 800, "samples": 256, "depth": 16},
         "spheres": {"width": 800, "samples": 64, "depth": 8},
         "rain": {"width": 1920, "samples": 512, "depth": 16}}


def _timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def run(scene, reps):
    import torch
    import torch.distributed as dist
    import raytracer_amd as rt
    from raytracer_amd import distributed as rtd
    from bench import SCENES
    cfg, ex, _ = SCENES[scene]
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data(cfg), {**EXTRA[scene], **ex, "aTolerance": 0})
    H, W = cam.image_height, cam.image_width
    region = (0, 0, W, H)
    dev = torch.device("cuda", 0)
    frame = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    t1 = _timed(lambda: cam.render_device(rgb_ptr=frame.data_ptr(), stream=s), reps)
    print(json.dumps({"scene": scene, "n": 1, "step_ms": round(t1, 3), "efficiency": 1.0}), flush=True)
    for n in (2, 4, 8):
        n_tiles = rtd.slab_tiles(region, n)
        n_px = n_tiles * rtd.TILE_PIXELS
        slabs = torch.zeros((n, rtd.slab_pixels(region, n), 3), dtype=torch.uint8, device=dev)
        gathered = torch.zeros_like(slabs)
        shares, kernels = [], []
        for g in range(n):
            def share():
                cam.render_device(rgb_ptr=slabs[g].data_ptr(), region=region, tile_group=g, tile_groups=n,
                                  stream=s, packed=True)
                cam.stats_words(slabs[g].data_ptr() + n_px * 3, s)
            shares.append(_timed(share, reps))
            kernels.append(cam.kernel_times())

        def gather():
            for g in range(n):
                dist.gather(slabs[g], gather_list=[gathered[g]], dst=0)
        t_gather = _timed(gather, reps)
        # one collective moving all N slabs (the real N-rank gather is ONE call: N - 1 slabs arrive
        # at rank 0 at once over separate xGMI links); the N sequential calls above bound it above
        flat = slabs.reshape(-1)
        flat_out = torch.empty_like(flat)
        t_gather1 = _timed(lambda: dist.all_gather_into_tensor(flat_out, flat), reps)
        t_unpack = _timed(lambda: rtd.unpack_tiles(gathered, region, W, H, frame, s, slab_tiles=n_tiles + 1), reps)
        # the assembled frame must be the single launch's (the rehearsal renders the real shares)
        single = torch.zeros_like(frame)
        cam.render_device(rgb_ptr=single.data_ptr(), stream=s, synchronize=True)
        ok = bool(torch.equal(frame, single))
        proj = max(shares) + t_gather + t_unpack
        print(json.dumps({
            "scene": scene, "n": n, "share_ms": {"max": round(max(shares), 3), "min": round(min(shares), 3),
                                               "mean": round(sum(shares) / n, 3),
                                               "slowest_group": shares.index(max(shares))},
            "path_kernel_ms_max": round(max(k[0] for k in kernels), 3),
            "gather_world1_ms": round(t_gather, 4), "gather_one_call_ms": round(t_gather1, 4),
            "unpack_ms": round(t_unpack, 4),
            "projected_step_ms": round(proj, 3), "efficiency": round(t1 / (n * proj), 4),
            "efficiency_one_call_gather": round(t1 / (n * (max(shares) + t_gather1 + t_unpack)), 4),
            "efficiency_share_only": round(t1 / (n * max(shares)), 4), "frame_equals_single": ok}), flush=True)
        if not ok:
            raise SystemExit(f"{scene} N={n}: assembled frame differs from the single launch")
    cam.close()


def main():
    import socket
    import torch
    import torch.distributed as dist
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    reps = int(os.environ.get("RANK_SHARE_REPS", "5"))
    for scene in sys.argv[1:] or ["cornell", "spheres"]:
        run(scene, reps)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
