"""Multi-GPU image partition and framebuffer assembly (one process per GPU).

The reference's only parallelism is worker threads rendering contiguous row
bands into a SharedArrayBuffer (src/raytracer.ts:60-90,185-205). Here the
image is split into 8x8-pixel tiles, dealt round-robin to the ranks (tile t of
the region goes to rank t % world), so bright and dark areas of the frame are
spread over every GPU. Each rank renders only its tiles into a zeroed
full-frame buffer; one RCCL reduce (SUM) over xGMI assembles the frame on
rank 0 - every pixel has exactly one non-zero writer, and x + 0 == x is exact
for both the u8 frame and the fp32 radiance. The path RNG is keyed by (pixel,
sample), so the partition never changes a pixel.
"""
from __future__ import annotations

TILE = 8


def tile_count(region, tile=TILE):
    x, y, w, h = region
    return (-(-w // tile)) * (-(-h // tile))


def owned_tiles(region, rank: int, world: int, tile=TILE):
    """Tile indices (row-major over the region) that `rank` renders."""
    return list(range(rank, tile_count(region, tile), world))


def owner_mask(width: int, height: int, region, rank: int, world: int, tile=TILE):
    """Boolean HxW mask of the pixels `rank` writes (mirrors the kernel's tile walk)."""
    import numpy as np

    x, y, w, h = region
    x1, y1 = min(x + w, width), min(y + h, height)
    tiles_x = -(-(x1 - x) // tile)
    m = np.zeros((height, width), dtype=bool)
    for t in owned_tiles((x, y, x1 - x, y1 - y), rank, world, tile):
        tx, ty = t % tiles_x, t // tiles_x
        m[y + ty * tile:min(y + (ty + 1) * tile, y1), x + tx * tile:min(x + (tx + 1) * tile, x1)] = True
    return m


def assemble_on_root(frame, group=None):
    """RCCL/gloo reduce (SUM) of the per-rank partial frames into rank 0's buffer."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM, group=group)
    return frame


def render_frame(camera, frame, rank: int, world: int, stream=None, precision=None, radiance=None):
    """Render this rank's tiles of the whole image into `frame` (a zeroed
    HxWx3 uint8 device tensor) and assemble the full image on rank 0."""
    frame.zero_()
    if radiance is not None:
        radiance.zero_()
    camera.render_device(rgb_ptr=frame.data_ptr(), radiance_ptr=radiance.data_ptr() if radiance is not None else None,
                         tile_group=rank, tile_groups=world, stream=stream, precision=precision)
    assemble_on_root(frame)
    if radiance is not None:
        assemble_on_root(radiance)
    return frame
