"""generateImageBuffer: the reference's render orchestration over the GPU core.

Mirrors src/raytracer.ts: RaytracerOptions (19-23), generateImageBuffer
(39-113) and divideIntoRegions (185-205). The reference's parallel mode fans
row bands out to worker threads that each rebuild the Camera and call
renderRegion; here each band is a renderRegion call on the GPU. Because the
path RNG is keyed by (pixel, sample), the image is identical for any band split.
"""
from __future__ import annotations

import os
import sys
from typing import Optional

from .scenes import generate_scene


def divide_into_regions(image_width: int, image_height: int, count: int):
    """divideIntoRegions (src/raytracer.ts:185-205): ceil(H/count)-row bands."""
    region_height = -(-image_height // count)
    regions = []
    for i in range(count):
        start_y = i * region_height
        height = min(region_height, image_height - start_y)
        if height <= 0:
            break
        regions.append({"x": 0, "y": start_y, "width": image_width, "height": height})
    return regions


def generate_image_buffer(scene_config: Optional[dict] = None, options: Optional[dict] = None,
                          return_stats: bool = False):
    """generateImageBuffer(sceneConfig, options) -> PNG bytes (src/raytracer.ts:39-113)."""
    scene_config = scene_config or {"type": "default"}
    options = options or {}
    parallel = bool(options.get("parallel", False))
    threads = options.get("threads")
    verbose = bool(options.get("verbose", False))

    camera = generate_scene(scene_config)
    w, h = camera.image_width, camera.image_height
    if w * h == 0:
        camera.close()
        raise RuntimeError("Generated pixelData buffer is empty before calling sharp.")
    # the reference's worker bands (parallel) or one region: rendered on the GPU into
    # the device frame, stats merged as RenderStats.merge, PNG encoded on the GPU
    bands = 1
    if parallel:
        bands = threads or max(1, (os.cpu_count() or 2) - 1)
        if verbose:
            print(f"Starting parallel render with {bands} worker threads", file=sys.stderr)
    png, stats = camera.render_png(bands)
    camera.close()
    if verbose:
        print(f"Adaptive sampling stats: avg={stats.samples['avg']:.2f}, min={stats.samples['min']}, "
              f"max={stats.samples['max']}", file=sys.stderr)
        print(f"Ray bounce stats: avg={stats.bounces['avg']:.2f}, min={stats.bounces['min']}, "
              f"max={stats.bounces['max']}", file=sys.stderr)
    return (png, stats) if return_stats else png


generateImageBuffer = generate_image_buffer
divideIntoRegions = divide_into_regions
