// fp32 fast-mode build of the path tracer (Real = float). Same algorithm and
// draw order as the ref build; parity with the ref oracle is tolerance-based.
#include "launch.hpp"

namespace rt {

template <bool EMIT, int INSTR, int TRAV, int LDSS>
static hipError_t go2(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                      const SampleBuf* sb, int pk, hipStream_t stream) {
    if (sb && pk == 2) {  // walker-pool kernel: product BVH builds
        if constexpr (!EMIT && INSTR != 1 && trav_fast(TRAV) && (LDSS == 0 || LDSS == 3)) {
            hipLaunchKernelGGL((pt_wpool_kernel<float, TRAV, LDSS, INSTR == 2>), dim3(g.grid), dim3(kBlockWPool), g.lds_bytes,
                               stream, S, reg, out, g.tiles_x, *sb);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    }
    if constexpr (LDSS == 3) return hipErrorInvalidValue;  // the walker-pool kernel's level only
    if (sb && pk == 1) {  // stage-compacted pool kernel: product brute-force builds only
        if constexpr (!EMIT && INSTR == 0 && TRAV == TRAV_BRUTE) {
            hipLaunchKernelGGL((pt_pool_kernel<float, TRAV, LDSS>), dim3(g.grid), dim3(kBlockPool), g.lds_bytes, stream,
                               S, reg, out, g.tiles_x, *sb);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    }
    if (sb)
        hipLaunchKernelGGL((pt_chunk_kernel<float, EMIT, INSTR, TRAV, LDSS>), dim3(g.grid), dim3(kBlockChunk), g.lds_bytes,
                           stream, S, reg, out, g.tiles_x, *sb);
    else
        hipLaunchKernelGGL((pt_render_kernel<float, EMIT, INSTR, TRAV, LDSS>), dim3(g.grid), dim3(kBlock), g.lds_bytes,
                           stream, S, reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

template <bool EMIT, int INSTR, int TRAV>
static hipError_t go(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                     const SampleBuf* sb, int pk, hipStream_t stream) {
    // LDS residency levels (pt_kernel.hpp scene_prologue); never with the reference traversal
    constexpr int L1 = trav_fast(TRAV) ? 1 : 0, L2 = TRAV == TRAV_REFERENCE ? 0 : 2;
    if (g.lds_level == 3) {  // the walker-pool kernel's walk-data-only level
        if constexpr (trav_fast(TRAV)) return go2<EMIT, INSTR, TRAV, 3>(S, reg, out, g, sb, pk, stream);
        else return hipErrorInvalidValue;
    }
    if (g.lds_level >= 2) return go2<EMIT, INSTR, TRAV, L2>(S, reg, out, g, sb, pk, stream);
    if (g.lds_level == 1) return go2<EMIT, INSTR, TRAV, L1>(S, reg, out, g, sb, pk, stream);
    return go2<EMIT, INSTR, TRAV, 0>(S, reg, out, g, sb, pk, stream);
}

template <int TRAV>
static hipError_t go_t(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                       const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    if (v.count == 2) return v.emit ? go<true, 2, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream) : go<false, 2, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream);
    if (v.count == 1) return v.emit ? go<true, 1, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream) : go<false, 1, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream);
    return v.emit ? go<true, 0, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream) : go<false, 0, TRAV>(S, reg, out, g, sb, v.wpool ? 2 : v.pool ? 1 : 0, stream);
}

hipError_t launch_render_fp32(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    if (v.trav == TRAV_BRUTE) return go_t<TRAV_BRUTE>(v, S, reg, out, g, sb, stream);
    if (v.trav == TRAV_FAST)
        return v.defer ? go_t<TRAV_FAST_DEFER>(v, S, reg, out, g, sb, stream) : go_t<TRAV_FAST>(v, S, reg, out, g, sb, stream);
    return go_t<TRAV_REFERENCE>(v, S, reg, out, g, sb, stream);
}

}  // namespace rt
