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

RenderStats ride in the same gather: every u8 slab carries one spare tile
whose first 64 bytes receive the rank's 8 stats words (rt_camera_stats_words,
a device-to-device copy queued after the render), and rank 0 merges them as
RenderStats.merge does for the reference's workers
(src/render-utils/renderStats.ts:42-64, src/raytracer.ts:86-89): no extra
collective and no host round trip in the frame path.
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


STATS_BYTES = 64  # RT_STATS_WORDS u64 words
I64_MAX = (1 << 63) - 1


def slab_pixels(region, world: int) -> int:
    """Pixels of a u8 slab: the largest share plus one spare tile for the stats
    words (rt_tiles_unpack never reads tile k = slab_tiles: its region index
    r + slab_tiles*world is past the last tile)."""
    return (slab_tiles(region, world) + 1) * TILE_PIXELS


def stats_from_words(w):
    """RenderStats from the 8 stats words (read_stats in rt_api.cpp)."""
    import math

    from .camera import RenderStats, _mm

    w = [int(v) & ((1 << 64) - 1) for v in w]
    if w[7] & 1:
        raise RuntimeError("Cannot read properties of undefined (reading 'top')")
    if w[7] & 2:
        raise RuntimeError("emission stack overflow: depth exceeds the emissive-scatter limit (128)")
    none = (1 << 64) - 1
    px, st, bt = float(w[0]), float(w[1]), float(w[4])
    return RenderStats(pixels=px,
                       samples=_mm(st, math.inf if w[2] == none else float(w[2]), float(w[3]),
                                   st / px if px > 0 else 0.0),
                       bounces=_mm(bt, math.inf if w[5] == none else float(w[5]), float(w[6]),
                                   bt / st if st > 0 else 0.0))


def merge_stats_words(words):
    """RenderStats.merge (renderStats.ts:42-64) over per-rank stats words, on
    whatever device `words` ([world, 8] int64 tensor, u64 bit patterns) lives:
    totals summed, minima / maxima over ranks (a rank without samples holds
    ~0 = -1 in its minima and is skipped), error flags or'ed. Returns [8] int64."""
    import torch

    w = words.reshape(-1, 8)
    big = torch.full_like(w[:, 2], I64_MAX)
    smin = torch.where(w[:, 2] == -1, big, w[:, 2]).amin()
    bmin = torch.where(w[:, 5] == -1, big, w[:, 5]).amin()
    smin = torch.where(smin == I64_MAX, torch.full_like(smin, -1), smin)
    bmin = torch.where(bmin == I64_MAX, torch.full_like(bmin, -1), bmin)
    err = w[0, 7]
    for r in range(1, w.shape[0]):
        err = torch.bitwise_or(err, w[r, 7])
    return torch.stack([w[:, 0].sum(), w[:, 1].sum(), smin, w[:, 3].amax(), w[:, 4].sum(), bmin,
                        w[:, 6].amax(), err])


def gathered_stats(gathered, n_px: int):
    """The merged stats words ([8] int64) of rank 0's gathered u8 slabs."""
    import torch

    g = gathered.reshape(gathered.shape[0], -1)[:, n_px * 3:n_px * 3 + STATS_BYTES]
    return merge_stats_words(g.contiguous().view(torch.int64))


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


def unpack_tiles(slabs, region, width: int, height: int, frame, stream=None, slab_tiles=None):
    """rt_tiles_unpack: scatter [world, slab_tiles*64, 3] device slabs into the
    region of the device frame (HxWx3, uint8 or float32). No CPU fallback.
    `slab_tiles` (default: from the slab shape) may count the spare stats tile."""
    import torch

    from . import _lib

    if not (slabs.is_cuda and frame.is_cuda):
        raise RuntimeError("unpack_tiles needs device tensors (HIP kernel)")
    world = slabs.shape[0]
    n_px = slabs[0].numel() // 3 if slab_tiles is None else int(slab_tiles) * TILE_PIXELS
    elem = {torch.uint8: 1, torch.float32: 4}[frame.dtype]
    if slabs.dtype != frame.dtype or not slabs.is_contiguous() or not frame.is_contiguous():
        raise ValueError("slabs and frame must be contiguous and of one dtype")
    reg = _lib.RtRegion(*[int(v) for v in region])
    st = stream if stream is not None else torch.cuda.current_stream(frame.device).cuda_stream
    _lib.check(_lib.load().rt_tiles_unpack(C.c_void_p(slabs.data_ptr()), world, n_px // TILE_PIXELS, C.byref(reg),
                                           width, height, 3, elem, C.c_void_p(frame.data_ptr()), C.c_void_p(st)))
    return frame


def render_frame(camera, frame, rank: int, world: int, stream=None, precision=None, radiance=None, region=None,
                 slab=None, rad_slab=None, gathered=None, rad_gathered=None, stats: bool = False):
    """Render this rank's tiles of `region` (default: the whole image) and
    assemble them in rank 0's `frame` (HxWx3 uint8 device tensor; `radiance`
    optionally HxWx3 float32). Slab buffers may be passed in to avoid
    reallocation (`slab` / `gathered`: slab_pixels(region, world) pixels, the
    spare tile holding the stats words). The render is queued on `stream`
    (default: torch's current stream of the frame's device); the gather and the
    unpack run on torch's current stream (collectives are issued there), and
    `stream` is then made to wait for them, so rank 0's frame is complete in
    order on both streams. Returns rank 0's frame (None on the other ranks when world > 1); with
    `stats`, (frame, merged RenderStats) on rank 0 - that waits for the stream."""
    import torch

    W, H = camera.image_width, camera.image_height
    region = clamp_region(region or (0, 0, W, H), W, H)
    if stream is None:
        stream = torch.cuda.current_stream(frame.device).cuda_stream
    if world == 1:
        camera.render_device(rgb_ptr=frame.data_ptr(), radiance_ptr=radiance.data_ptr() if radiance is not None else None,
                             region=region, stream=stream, precision=precision)
        if not stats:
            return frame
        w = torch.empty(8, dtype=torch.int64, device=frame.device)
        camera.stats_words(w.data_ptr(), stream)
        _sync(stream)
        return frame, stats_from_words(w.cpu().tolist())
    n_tiles = slab_tiles(region, world)
    n_px = n_tiles * TILE_PIXELS
    if slab is None:
        slab = torch.empty((n_px + TILE_PIXELS, 3), dtype=torch.uint8, device=frame.device)
    if slab.numel() < (n_px + TILE_PIXELS) * 3:
        raise ValueError("slab must hold slab_pixels(region, world) pixels (the spare tile carries the stats)")
    if radiance is not None and rad_slab is None:
        rad_slab = torch.empty((n_px, 3), dtype=torch.float32, device=frame.device)
    camera.render_device(rgb_ptr=slab.data_ptr(), radiance_ptr=rad_slab.data_ptr() if radiance is not None else None,
                         region=region, tile_group=rank, tile_groups=world, stream=stream, precision=precision,
                         packed=True)
    camera.stats_words(slab.data_ptr() + n_px * 3, stream)
    # the gather runs on torch's current stream: order it after the render's stream
    _wait(stream, frame.device)
    g = gather_slabs(slab, world, out=gathered)
    gr = gather_slabs(rad_slab, world, out=rad_gathered) if radiance is not None else None
    if rank != 0:
        # the gather still reads `slab` on torch's current stream: a next render queued on
        # `stream` must not overwrite it first
        _wait_for_current(stream, frame.device)
        return None
    cur = torch.cuda.current_stream(frame.device).cuda_stream
    unpack_tiles(g, region, W, H, frame, cur, slab_tiles=n_tiles + 1)
    if radiance is not None:
        unpack_tiles(gr, region, W, H, radiance, cur)
    _wait_for_current(stream, frame.device)
    if not stats:
        return frame
    w = gathered_stats(g, n_px)
    return frame, stats_from_words(w.cpu().tolist())


def _wait(stream, device):
    """Make torch's current stream wait for work queued on `stream` (a raw
    hipStream_t), so collectives issued by torch see the render."""
    import torch

    cur = torch.cuda.current_stream(device)
    if stream == cur.cuda_stream:
        return
    ext = torch.cuda.ExternalStream(stream, device=device)
    ev = torch.cuda.Event()
    ev.record(ext)
    cur.wait_event(ev)


def _wait_for_current(stream, device):
    """Make `stream` (a raw hipStream_t) wait for the work queued so far on
    torch's current stream (the gather and unpack)."""
    import torch

    cur = torch.cuda.current_stream(device)
    if stream == cur.cuda_stream:
        return
    ev = torch.cuda.Event()
    ev.record(cur)
    torch.cuda.ExternalStream(stream, device=device).wait_event(ev)


def _sync(stream):
    import torch

    torch.cuda.ExternalStream(stream).synchronize()
