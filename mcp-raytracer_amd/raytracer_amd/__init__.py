"""raytracer_amd - MI355X-native path-tracing core for df07/mcp-raytracer.

The hot path (camera rays, BVH traversal, sphere/quad/plane hits, material
scatter with mixture-PDF light sampling, spp accumulation) runs as HIP
kernels for gfx950 in librt_amd.so, behind the C ABI in include/rt_amd.h.
This package is the host-side mirror of the reference's TypeScript surface:

    generate_scene_data / create_camera_from_scene_data / generate_scene  (src/scenes/scenes.ts)
    Camera.render_region / Camera.render -> RenderStats                  (src/camera.ts)
    generate_image_buffer                                                (src/raytracer.ts)
"""
from ._lib import RtError, build_id, device_count
from .camera import Camera, RenderStats, rng_stream
from .raytracer import divide_into_regions, divideIntoRegions, generate_image_buffer, generateImageBuffer
from .scenes import (create_camera_from_scene_data, createCameraFromSceneData, generate_scene,
                     generate_scene_data, generateScene, generateSceneData)

__all__ = [
    "Camera", "RenderStats", "RtError", "build_id", "device_count", "rng_stream",
    "generate_scene_data", "create_camera_from_scene_data", "generate_scene",
    "generate_image_buffer", "divide_into_regions",
    "generateSceneData", "createCameraFromSceneData", "generateScene", "generateImageBuffer",
    "divideIntoRegions",
]
