// Kernel launch entry points, one translation unit per scalar precision so the
// ref build can be compiled with -ffp-contract=off (no fused multiply-adds:
// the reference's JS arithmetic never fuses) while the fp32 build may fuse.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "pt_kernel.hpp"

namespace rt {

enum Precision : int32_t { PREC_REF = 0, PREC_FP32 = 1 };

struct LaunchGeom {
    int tiles_x;
    int my_tiles;
    int grid;
    size_t lds_bytes;  // traversal stack + the LDS-resident scene prefix
    int lds_level;     // LDS-resident scene: 0 none, 1 traversal data + prims, 2 also mats + lights
};

// LDS budget (stack + [tnodes][prims]) up to which the scene is copied into LDS.
constexpr int kLdsSceneMaxBytes = 152 * 1024;
// Static LDS of the chunked / pool kernels (the phase table), beside the dynamic allocation.
constexpr size_t kStaticLdsBytes = 512;
// ... plus the per-wave section timers of the diagnostic variants: every kernel of a
// count == 2 launch, and every pool kernel of an RT_POOL_PROF build.
inline size_t static_lds_bytes(int count, bool pool) {
    const bool prof = count == 2 || (pool && RT_POOL_PROF);
    return kStaticLdsBytes + (prof ? (size_t)kProfWaves * kProfSlot * sizeof(unsigned long long) : 0);
}

struct KernelVariant {
    bool emit;   // emission stack (a scattering material emits)
    int count;   // 0 product, 1 work counters, 2 section timing (diagnostic)
    int trav;    // TRAV_FAST / TRAV_REFERENCE / TRAV_BRUTE (resolved, never AUTO)
    bool defer = false;  // TRAV_FAST: deferred exact sphere tests (TRAV_FAST_DEFER kernels)
    bool pool = false;   // chunked passes run the stage-compacted pool kernel (pt_pool_kernel)
};

// sb == nullptr: the sequential-pixel kernel; else the chunked kernel over sb's pass.
hipError_t launch_render_ref(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream);
hipError_t launch_render_fp32(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                              const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream);
// Per-pixel in-order sum of a chunked pass's sample buffer + outputs + stats.
hipError_t launch_accum(const DevScene& S, const RtRegion& reg, const RenderOut& out, int tiles_x,
                        const SampleBuf& sb, hipStream_t stream);
// One adaptive-sampling round's accumulate / convergence pass over the pass's slots.
hipError_t launch_adapt(const DevScene& S, const RtRegion& reg, const RenderOut& out, int tiles_x,
                        const SampleBuf& sb, const AdaptRound& ar, hipStream_t stream);
// Resets the stats words / counters / tile counter before a render.
hipError_t launch_init_stats(unsigned long long* stats, unsigned long long* counters, unsigned int* tile_counter,
                             hipStream_t stream);
// Closest hit through the device traversal for a batch of rays (parity tests).
hipError_t launch_world_hit_ref(const DevScene& S, int trav, int n, const float* orig, const float* dir,
                                double* out, hipStream_t stream);

// Device transcendental probe (V8 fixture tests): out[3k..3k+2] = cos, sin of 2 pi xi, pow(xi, 5).
hipError_t launch_math_probe(int n, const uint32_t* u, double* out, hipStream_t stream);
hipError_t launch_fp64_probe(int n, const double* x, double* out, hipStream_t stream);

// Scatter of tile-packed slabs into the full-frame layout (frame.hip).
hipError_t launch_tiles_unpack(const void* slabs, int groups, int slab_tiles, const RtRegion& reg, int width,
                               int channels, int elem_bytes, void* frame, hipStream_t stream);

// LDS bytes per workgroup for the traversal stack (fast / reference) or the
// per-lane candidate bounds of the nearest-first brute force.
// `lds_tree`: the launch's tree is LDS-resident (LDSS > 0), whose fast-walk stack entries are 16-bit
// (StackT, pt_kernel.hpp)
inline size_t stack_lds_bytes(int stack_depth, int trav, int n_prims, bool lds_tree = false) {
    if (trav == TRAV_BRUTE)  // larger forced brute-force scenes take the in-order loop (no LDS)
        return n_prims <= kBruteMaxPrims ? (size_t)std::max(n_prims, 1) * kStackStride * sizeof(uint16_t) : 0;
    const size_t d = (size_t)(stack_depth > 0 ? stack_depth : 1);
    const size_t e = lds_tree ? sizeof(StackT<1>) : sizeof(StackT<0>);
    return d * kStackStride * e;
}

// The kernel template instance of a launch (one per scalar precision unit: pt_ref.hip,
// pt_fp32.hip). sb == nullptr: the sequential-pixel kernel; else the chunked kernel, or the
// pool kernel (product brute-force builds; RT_POOL_PROF adds its ref-precision timer build).
template <class Real, bool EMIT, int INSTR, int TRAV, int LDSS>
hipError_t dispatch_kernel(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                           const SampleBuf* sb, bool pool, hipStream_t stream) {
    if (sb && pool) {
        if constexpr (!EMIT && TRAV == TRAV_BRUTE && (INSTR == 0 || (RT_POOL_PROF && INSTR == 2 && sizeof(Real) == 8))) {
            hipLaunchKernelGGL((pt_pool_kernel<Real, TRAV, LDSS>), dim3(g.grid), dim3(kBlockPool), g.lds_bytes, stream,
                               S, reg, out, g.tiles_x, *sb);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    }
    if (sb)
        hipLaunchKernelGGL((pt_chunk_kernel<Real, EMIT, INSTR, TRAV, LDSS>), dim3(g.grid), dim3(kBlockChunk),
                           g.lds_bytes, stream, S, reg, out, g.tiles_x, *sb);
    else
        hipLaunchKernelGGL((pt_render_kernel<Real, EMIT, INSTR, TRAV, LDSS>), dim3(g.grid), dim3(kBlock), g.lds_bytes,
                           stream, S, reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

template <class Real, bool EMIT, int INSTR, int TRAV>
hipError_t dispatch_level(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                          const SampleBuf* sb, bool pool, hipStream_t stream) {
    // LDS residency levels (pt_kernel.hpp scene_prologue); never with the reference traversal
    constexpr int L1 = trav_fast(TRAV) ? 1 : 0, L2 = TRAV == TRAV_REFERENCE ? 0 : 2;
    if (g.lds_level >= 2) return dispatch_kernel<Real, EMIT, INSTR, TRAV, L2>(S, reg, out, g, sb, pool, stream);
    if (g.lds_level == 1) return dispatch_kernel<Real, EMIT, INSTR, TRAV, L1>(S, reg, out, g, sb, pool, stream);
    return dispatch_kernel<Real, EMIT, INSTR, TRAV, 0>(S, reg, out, g, sb, pool, stream);
}

template <class Real, int TRAV>
hipError_t dispatch_variant(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                            const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    if (v.count == 2)
        return v.emit ? dispatch_level<Real, true, 2, TRAV>(S, reg, out, g, sb, v.pool, stream)
                      : dispatch_level<Real, false, 2, TRAV>(S, reg, out, g, sb, v.pool, stream);
    if (v.count == 1)
        return v.emit ? dispatch_level<Real, true, 1, TRAV>(S, reg, out, g, sb, v.pool, stream)
                      : dispatch_level<Real, false, 1, TRAV>(S, reg, out, g, sb, v.pool, stream);
    return v.emit ? dispatch_level<Real, true, 0, TRAV>(S, reg, out, g, sb, v.pool, stream)
                  : dispatch_level<Real, false, 0, TRAV>(S, reg, out, g, sb, v.pool, stream);
}

template <class Real>
hipError_t dispatch_render(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                           const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    if (v.trav == TRAV_BRUTE) return dispatch_variant<Real, TRAV_BRUTE>(v, S, reg, out, g, sb, stream);
    if (v.trav == TRAV_FAST)
        return v.defer ? dispatch_variant<Real, TRAV_FAST_DEFER>(v, S, reg, out, g, sb, stream)
                       : dispatch_variant<Real, TRAV_FAST>(v, S, reg, out, g, sb, stream);
    return dispatch_variant<Real, TRAV_REFERENCE>(v, S, reg, out, g, sb, stream);
}

}  // namespace rt
