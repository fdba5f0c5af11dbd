// Kernel launch entry points, one translation unit per scalar precision so the
// ref build can be compiled with -ffp-contract=off (no fused multiply-adds:
// the reference's JS arithmetic never fuses) while the fp32 build may fuse.
#pragma once

#include <hip/hip_runtime.h>

#include "pt_kernel.hpp"

namespace rt {

enum Precision : int32_t { PREC_REF = 0, PREC_FP32 = 1 };

struct LaunchGeom {
    int tiles_x;
    int my_tiles;
    int grid;
    size_t lds_bytes;
};

hipError_t launch_render_ref(bool emit, bool count, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, hipStream_t stream);
hipError_t launch_render_fp32(bool emit, bool count, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                              const LaunchGeom& g, hipStream_t stream);
// Resets the stats words / counters / tile counter before a render.
hipError_t launch_init_stats(unsigned long long* stats, unsigned long long* counters, unsigned int* tile_counter,
                             hipStream_t stream);
// Closest hit through the device traversal for a batch of rays (parity tests).
hipError_t launch_world_hit_ref(const DevScene& S, int n, const float* orig, const float* dir, double tmin,
                                double tmax, double* out, hipStream_t stream);

}  // namespace rt
