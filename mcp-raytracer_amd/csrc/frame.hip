// Framebuffer assembly of the multi-GPU split: rank r renders
// the region's 8x8 tiles r, r + N, r + 2N, ... into a tile-packed slab
// (RenderOut::packed); rank 0 receives every rank's slab (RCCL gather) and this
// kernel scatters the slabs back into the full-frame layout that
// Camera.renderRegion's caller owns (src/camera.ts:388-431, writeColorToBuffer
// 455-472: offset (j*W + i)*3). Pure data movement: one thread per packed pixel,
// coalesced reads of the slab, 8-pixel row runs of writes.
#include "launch.hpp"

namespace rt {

template <class T>
__global__ __launch_bounds__(256) void tiles_unpack_kernel(const T* __restrict__ slabs, int groups, int slab_tiles,
                                                           RtRegion reg, int tiles_x, int total_tiles, int width,
                                                           int channels, T* __restrict__ frame) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (slab r, tile k, lane l)
    const long n = (long)groups * slab_tiles * kWave;
    if (idx >= n) return;
    const int l = (int)(idx & (kWave - 1));
    const long rk = idx >> 6;
    const int r = (int)(rk / slab_tiles), k = (int)(rk - (long)r * slab_tiles);
    const long g = (long)r + (long)k * groups;  // the region's tile index
    if (g >= total_tiles) return;
    const int ty = (int)(g / tiles_x), tx = (int)(g - (long)ty * tiles_x);
    const int i = reg.x + tx * kTile + (l & (kTile - 1));
    const int j = reg.y + ty * kTile + l / kTile;
    if (i >= reg.x + reg.width || j >= reg.y + reg.height) return;
    const T* src = slabs + idx * channels;
    T* dst = frame + ((long)j * width + i) * channels;
    for (int c = 0; c < channels; ++c) dst[c] = src[c];
}

hipError_t launch_tiles_unpack(const void* slabs, int groups, int slab_tiles, const RtRegion& reg, int width,
                               int channels, int elem_bytes, void* frame, hipStream_t stream) {
    const int tiles_x = (reg.width + kTile - 1) / kTile, tiles_y = (reg.height + kTile - 1) / kTile;
    const long total = (long)tiles_x * tiles_y;
    const long n = (long)groups * slab_tiles * kWave;
    if (n == 0 || total == 0) return hipSuccess;
    const long grid = (n + 255) / 256;
    if (elem_bytes == 1)
        hipLaunchKernelGGL(tiles_unpack_kernel<uint8_t>, dim3((unsigned)grid), dim3(256), 0, stream,
                           (const uint8_t*)slabs, groups, slab_tiles, reg, tiles_x, (int)total, width, channels,
                           (uint8_t*)frame);
    else
        hipLaunchKernelGGL(tiles_unpack_kernel<float>, dim3((unsigned)grid), dim3(256), 0, stream,
                           (const float*)slabs, groups, slab_tiles, reg, tiles_x, (int)total, width, channels,
                           (float*)frame);
    return hipGetLastError();
}

}  // namespace rt
