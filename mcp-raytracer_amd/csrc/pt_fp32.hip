// fp32 fast-mode build of the path tracer (Real = float). Same algorithm and
// draw order as the ref build; parity with the ref oracle is tolerance-based.
#include "launch.hpp"

namespace rt {

hipError_t launch_render_fp32(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                              const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    return dispatch_render<float>(v, S, reg, out, g, sb, stream);
}

}  // namespace rt
