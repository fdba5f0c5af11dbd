// fp32 fast-mode build of the path tracer (Real = float). Same algorithm and
// draw order as the ref build; parity with the ref oracle is tolerance-based.
#include "launch.hpp"

namespace rt {

template <bool EMIT, bool COUNT, bool FAST>
static hipError_t go(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                     hipStream_t stream) {
    hipLaunchKernelGGL((pt_render_kernel<float, EMIT, COUNT, FAST>), dim3(g.grid), dim3(kBlock), g.lds_bytes,
                       stream, S, reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

hipError_t launch_render_fp32(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                              const LaunchGeom& g, hipStream_t stream) {
    if (v.fast) {
        if (v.emit) return v.count ? go<true, true, true>(S, reg, out, g, stream) : go<true, false, true>(S, reg, out, g, stream);
        return v.count ? go<false, true, true>(S, reg, out, g, stream) : go<false, false, true>(S, reg, out, g, stream);
    }
    if (v.emit) return v.count ? go<true, true, false>(S, reg, out, g, stream) : go<true, false, false>(S, reg, out, g, stream);
    return v.count ? go<false, true, false>(S, reg, out, g, stream) : go<false, false, false>(S, reg, out, g, stream);
}

}  // namespace rt
