"""Multi-rank partition and framebuffer assembly on CPU (gloo, world_size 2).

The GPU render of each rank's tiles is stood in for by the oracle's image
(no GPU here); what is under test is the product's tile ownership
(raytracer_amd.distributed.owner_mask, the kernel's tile walk) and the
reduce-to-rank-0 assembly (assemble_on_root), the same code bench.py runs
over RCCL.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("W,H,world", [(37, 21, 2), (64, 64, 3), (8, 9, 4), (800, 800, 8)])
def test_owner_masks_partition_the_image(W, H, world):
    from raytracer_amd.distributed import owner_mask
    cover = sum(owner_mask(W, H, (0, 0, W, H), r, world).astype(int) for r in range(world))
    assert cover.min() == 1 and cover.max() == 1
    # a sub-region partition covers exactly the region
    cover = sum(owner_mask(W, H, (3, 2, W - 5, H - 3), r, world).astype(int) for r in range(world))
    assert cover[2:H - 1, 3:W - 2].min() == 1 and cover.sum() == (W - 5) * (H - 3)


def _worker(rank, world, port, full_rgb, full_rad, q):
    import torch
    import torch.distributed as dist
    from raytracer_amd.distributed import assemble_on_root, owner_mask
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W = full_rgb.shape[:2]
    m = owner_mask(W, H, (0, 0, W, H), rank, world)
    frame = torch.zeros((H, W, 3), dtype=torch.uint8)
    rad = torch.zeros((H, W, 3), dtype=torch.float32)
    frame[torch.from_numpy(m)] = torch.from_numpy(full_rgb)[torch.from_numpy(m)]
    rad[torch.from_numpy(m)] = torch.from_numpy(full_rad)[torch.from_numpy(m)]
    assemble_on_root(frame)
    assemble_on_root(rad)
    if rank == 0:
        q.put((frame.numpy().copy(), rad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_assembly_equals_full_render(oracle, rt):
    import torch.multiprocessing as mp
    sd = rt.generate_scene_data({"type": "cornell"})
    full = oracle.render(sd, {"width": 40, "samples": 4, "depth": 6, "aTolerance": 0})
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, full["rgb"], full["radiance"], q)) for r in range(2)]
    for p in procs:
        p.start()
    rgb, rad = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(rgb, full["rgb"])
    assert np.array_equal(rad, full["radiance"])  # x + 0 == x: the reduce is exact
