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

from .camera import RenderStats
from .png import encode_png
from .scenes import create_camera_from_scene_data, generate_scene, generate_scene_data


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
    w, h, ch = camera.image_width, camera.image_height, camera.channels
    pixel_data = bytearray(w * h * ch)
    if not parallel:
        stats = camera.render(pixel_data)
    else:
        thread_count = threads or max(1, (os.cpu_count() or 2) - 1)
        if verbose:
            print(f"Starting parallel render with {thread_count} worker threads", file=sys.stderr)
        scene_data = generate_scene_data(scene_config)
        regions = divide_into_regions(w, h, thread_count)
        results = []
        for region in regions:
            worker_cam = create_camera_from_scene_data(scene_data, scene_config.get("render"))
            results.append(worker_cam.render_region(pixel_data, region))
            worker_cam.close()
        stats = RenderStats.merge(results)
    camera.close()
    if verbose:
        print(f"Adaptive sampling stats: avg={stats.samples['avg']:.2f}, min={stats.samples['min']}, "
              f"max={stats.samples['max']}", file=sys.stderr)
        print(f"Ray bounce stats: avg={stats.bounces['avg']:.2f}, min={stats.bounces['min']}, "
              f"max={stats.bounces['max']}", file=sys.stderr)
    if len(pixel_data) == 0:
        raise RuntimeError("Generated pixelData buffer is empty before calling sharp.")
    png = encode_png(pixel_data, w, h, ch)
    return (png, stats) if return_stats else png


generateImageBuffer = generate_image_buffer
divideIntoRegions = divide_into_regions
