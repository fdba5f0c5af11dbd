// fp32 fast-mode build of the path tracer (Real = float). Same algorithm and
// draw order as the ref build; parity with the ref oracle is tolerance-based.
#include "launch.hpp"

namespace rt {

template <bool EMIT, bool COUNT>
static hipError_t go(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                     hipStream_t stream) {
    hipLaunchKernelGGL((pt_render_kernel<float, EMIT, COUNT>), dim3(g.grid), dim3(kBlock), g.lds_bytes, stream, S,
                       reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

hipError_t launch_render_fp32(bool emit, bool count, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                              const LaunchGeom& g, hipStream_t stream) {
    if (emit) return count ? go<true, true>(S, reg, out, g, stream) : go<true, false>(S, reg, out, g, stream);
    return count ? go<false, true>(S, reg, out, g, stream) : go<false, false>(S, reg, out, g, stream);
}

}  // namespace rt
