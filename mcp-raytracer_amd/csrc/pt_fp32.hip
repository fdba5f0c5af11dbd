// fp32 fast-mode build of the path tracer (Real = float). Same algorithm and
// draw order as the ref build; parity with the ref oracle is tolerance-based.
#include "launch.hpp"

namespace rt {

template <bool EMIT, bool COUNT, int TRAV>
static hipError_t go(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                     hipStream_t stream) {
    hipLaunchKernelGGL((pt_render_kernel<float, EMIT, COUNT, TRAV>), dim3(g.grid), dim3(kBlock), g.lds_bytes,
                       stream, S, reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

template <int TRAV>
static hipError_t go_t(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                       const LaunchGeom& g, hipStream_t stream) {
    if (v.emit) return v.count ? go<true, true, TRAV>(S, reg, out, g, stream) : go<true, false, TRAV>(S, reg, out, g, stream);
    return v.count ? go<false, true, TRAV>(S, reg, out, g, stream) : go<false, false, TRAV>(S, reg, out, g, stream);
}

hipError_t launch_render_fp32(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, hipStream_t stream) {
    if (v.trav == TRAV_BRUTE) return go_t<TRAV_BRUTE>(v, S, reg, out, g, stream);
    if (v.trav == TRAV_FAST) return go_t<TRAV_FAST>(v, S, reg, out, g, stream);
    return go_t<TRAV_REFERENCE>(v, S, reg, out, g, stream);
}

}  // namespace rt
