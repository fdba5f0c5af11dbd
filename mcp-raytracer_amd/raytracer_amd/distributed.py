"""Multi-GPU image partition and framebuffer gather (one process per GPU).

The reference's only parallelism is worker threads rendering contiguous row
bands into one SharedArrayBuffer (src/raytracer.ts:60-90,185-205). Here the
region is split into 8x8-pixel tiles dealt round-robin to the ranks (tile t
goes to rank t % world), which spreads bright and dark areas of the frame over
every GPU. Each rank renders only its tiles, straight into a tile-packed slab
(rt_launch.packed_tiles: its k-th tile's 64 pixels at [k*64, k*64 + 64)), so a
rank moves frame/world bytes, not a full frame. One RCCL gather over xGMI
collects the equal-size slabs on rank 0, and rt_tiles_unpack (a HIP kernel)
scatters them into the caller's full-frame buffer. The path RNG is keyed by
(pixel, sample), so the partition never changes a pixel.
"""
from __future__ import annotations

import ctypes as C

TILE = 8
TILE_PIXELS = TILE * TILE


def tile_count(region, tile=TILE):
    x, y, w, h = region
    return (-(-w // tile)) * (-(-h // tile))


def owned_tiles(region, rank: int, world: int, tile=TILE):
    """Tile indices (row-major over the region) that `rank` renders."""
    return list(range(rank, tile_count(region, tile), world))


def slab_tiles(region, world: int) -> int:
    """Tiles per rank slab: the largest share (every slab is padded to it)."""
    return -(-tile_count(region) // world)


def clamp_region(region, width: int, height: int):
    x, y, w, h = region
    x0, y0 = max(x, 0), max(y, 0)
    x1, y1 = min(x + w, width), min(y + h, height)
    return (x0, y0, max(x1 - x0, 0), max(y1 - y0, 0))


def owner_mask(width: int, height: int, region, rank: int, world: int, tile=TILE):
    """Boolean HxW mask of the pixels `rank` writes (mirrors the kernel's tile walk)."""
    import numpy as np

    x, y, w, h = clamp_region(region, width, height)
    x1, y1 = x + w, y + h
    tiles_x = -(-w // tile)
    m = np.zeros((height, width), dtype=bool)
    for t in owned_tiles((x, y, w, h), rank, world, tile):
        tx, ty = t % tiles_x, t // tiles_x
        m[y + ty * tile:min(y + (ty + 1) * tile, y1), x + tx * tile:min(x + (tx + 1) * tile, x1)] = True
    return m


def gather_slabs(slab, world: int, out=None, group=None):
    """RCCL/gloo gather of every rank's slab to rank 0. Returns the stacked
    [world, *slab.shape] tensor on rank 0 (`out` if given), None elsewhere."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return slab.unsqueeze(0)
    if slab.is_cuda and dist.get_backend(group) == "gloo":
        # CPU-backend rehearsal (several ranks on one GPU): gloo gathers host tensors only
        g = gather_slabs(slab.cpu(), world, group=group)
        if g is None:
            return None
        if out is None:
            return g.to(slab.device)
        out.copy_(g)
        return out
    rank = dist.get_rank(group)
    if rank == 0:
        if out is None:
            out = torch.empty((world, *slab.shape), dtype=slab.dtype, device=slab.device)
        dist.gather(slab, gather_list=list(out.unbind(0)), dst=0, group=group)
        return out
    dist.gather(slab, dst=0, group=group)
    return None


def unpack_tiles(slabs, region, width: int, height: int, frame, stream=None):
    """rt_tiles_unpack: scatter [world, slab_tiles*64, 3] device slabs into the
    region of the device frame (HxWx3, uint8 or float32). No CPU fallback."""
    import torch

    from . import _lib

    if not (slabs.is_cuda and frame.is_cuda):
        raise RuntimeError("unpack_tiles needs device tensors (HIP kernel)")
    world, n_px = slabs.shape[0], slabs.shape[1]
    elem = {torch.uint8: 1, torch.float32: 4}[frame.dtype]
    if slabs.dtype != frame.dtype or not slabs.is_contiguous() or not frame.is_contiguous():
        raise ValueError("slabs and frame must be contiguous and of one dtype")
    reg = _lib.RtRegion(*[int(v) for v in region])
    st = stream if stream is not None else torch.cuda.current_stream(frame.device).cuda_stream
    _lib.check(_lib.load().rt_tiles_unpack(C.c_void_p(slabs.data_ptr()), world, n_px // TILE_PIXELS, C.byref(reg),
                                           width, height, 3, elem, C.c_void_p(frame.data_ptr()), C.c_void_p(st)))
    return frame


def render_frame(camera, frame, rank: int, world: int, stream=None, precision=None, radiance=None, region=None,
                 slab=None, rad_slab=None, gathered=None, rad_gathered=None):
    """Render this rank's tiles of `region` (default: the whole image) and
    assemble them in rank 0's `frame` (HxWx3 uint8 device tensor; `radiance`
    optionally HxWx3 float32). Slab buffers may be passed in to avoid
    reallocation. Returns rank 0's frame (None on the other ranks when world > 1)."""
    import torch

    W, H = camera.image_width, camera.image_height
    region = clamp_region(region or (0, 0, W, H), W, H)
    if world == 1:
        camera.render_device(rgb_ptr=frame.data_ptr(), radiance_ptr=radiance.data_ptr() if radiance is not None else None,
                             region=region, stream=stream, precision=precision)
        return frame
    n_px = slab_tiles(region, world) * TILE_PIXELS
    if slab is None:
        slab = torch.empty((n_px, 3), dtype=torch.uint8, device=frame.device)
    if radiance is not None and rad_slab is None:
        rad_slab = torch.empty((n_px, 3), dtype=torch.float32, device=frame.device)
    camera.render_device(rgb_ptr=slab.data_ptr(), radiance_ptr=rad_slab.data_ptr() if radiance is not None else None,
                         region=region, tile_group=rank, tile_groups=world, stream=stream, precision=precision,
                         packed=True)
    g = gather_slabs(slab, world, out=gathered)
    gr = gather_slabs(rad_slab, world, out=rad_gathered) if radiance is not None else None
    if rank != 0:
        return None
    unpack_tiles(g, region, W, H, frame, stream)
    if radiance is not None:
        unpack_tiles(gr, region, W, H, radiance, stream)
    return frame
