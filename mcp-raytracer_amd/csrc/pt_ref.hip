// Reference-precision build of the path tracer (Real = double, fp32 vector
// stores). Compiled with -ffp-contract=off so every scalar op rounds exactly as
// the reference's JS doubles do.
#include "launch.hpp"

namespace rt {

template <bool EMIT, bool COUNT, int TRAV>
static hipError_t go(const DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g,
                     hipStream_t stream) {
    hipLaunchKernelGGL((pt_render_kernel<double, EMIT, COUNT, TRAV>), dim3(g.grid), dim3(kBlock), g.lds_bytes,
                       stream, S, reg, out, g.tiles_x, g.my_tiles);
    return hipGetLastError();
}

template <int TRAV>
static hipError_t go_t(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                       const LaunchGeom& g, hipStream_t stream) {
    if (v.emit) return v.count ? go<true, true, TRAV>(S, reg, out, g, stream) : go<true, false, TRAV>(S, reg, out, g, stream);
    return v.count ? go<false, true, TRAV>(S, reg, out, g, stream) : go<false, false, TRAV>(S, reg, out, g, stream);
}

hipError_t launch_render_ref(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, hipStream_t stream) {
    if (v.trav == TRAV_BRUTE) return go_t<TRAV_BRUTE>(v, S, reg, out, g, stream);
    if (v.trav == TRAV_FAST) return go_t<TRAV_FAST>(v, S, reg, out, g, stream);
    return go_t<TRAV_REFERENCE>(v, S, reg, out, g, stream);
}

__global__ void init_stats_kernel(unsigned long long* stats, unsigned long long* counters,
                                  unsigned int* tile_counter) {
    const int t = threadIdx.x;
    if (t < ST_WORDS) stats[t] = (t == ST_SMIN || t == ST_BMIN) ? ~0ull : 0ull;
    if (counters && t < CT_WORDS) counters[t] = 0ull;
    if (t == 0) *tile_counter = 0u;
}

hipError_t launch_init_stats(unsigned long long* stats, unsigned long long* counters, unsigned int* tile_counter,
                             hipStream_t stream) {
    hipLaunchKernelGGL(init_stats_kernel, dim3(1), dim3(64), 0, stream, stats, counters, tile_counter);
    return hipGetLastError();
}

// out per ray: {hit, t, p.xyz, n.xyz, front, prim}
template <int TRAV>
__global__ __launch_bounds__(kBlock) void world_hit_kernel(DevScene S, int n, const float* orig, const float* dir,
                                                           double* out) {
    extern __shared__ int lds_stack[];
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const V3 o = v3(orig[3 * k], orig[3 * k + 1], orig[3 * k + 2]);
    const V3 d = v3(dir[3 * k], dir[3 * k + 1], dir[3 * k + 2]);
    const RayK<double> r = make_ray<double>(o, d);
    double t = 0;
    int* stk = lds_stack + threadIdx.x;
    float* stkt = reinterpret_cast<float*>(lds_stack) + (size_t)S.cam.stack_depth * kBlock + threadIdx.x;
    const int h = closest_hit_any<double, false, TRAV>(S, S.cam.n_prims, r, t, stk, stkt, nullptr);
    double* w = out + 10 * (size_t)k;
    w[0] = h >= 0;
    w[1] = h >= 0 ? t : 0.0;
    for (int a = 2; a < 10; ++a) w[a] = 0.0;
    w[9] = h;
    if (h >= 0) {
        const RtPrim pr = S.prims[h];
        const V3 p = ray_at<double>(o, d, t);
        V3 nrm;
        bool front;
        if (pr.type == PRIM_SPHERE) {
            nrm = divs<double>(sub(p, ld3(pr.g0)), sphere_radius<double>(pr));
            front = dot<double>(d, nrm) <= 0.0;
            if (!front) nrm = neg(nrm);
        } else {
            const V3 pn = ld3(pr.g3);
            front = dot<double>(d, pn) <= 0.0;
            nrm = front ? pn : neg(pn);
        }
        w[2] = p.x; w[3] = p.y; w[4] = p.z;
        w[5] = nrm.x; w[6] = nrm.y; w[7] = nrm.z;
        w[8] = front;
    }
}

hipError_t launch_world_hit_ref(const DevScene& S, int trav, int n, const float* orig, const float* dir,
                                double* out, hipStream_t stream) {
    const int grid = (n + kBlock - 1) / kBlock;
    const size_t lds = stack_lds_bytes(S.cam.stack_depth, TRAV_FAST);  // largest footprint
    if (trav == TRAV_BRUTE)
        hipLaunchKernelGGL(world_hit_kernel<TRAV_BRUTE>, dim3(grid), dim3(kBlock), lds, stream, S, n, orig, dir, out);
    else if (trav == TRAV_FAST)
        hipLaunchKernelGGL(world_hit_kernel<TRAV_FAST>, dim3(grid), dim3(kBlock), lds, stream, S, n, orig, dir, out);
    else
        hipLaunchKernelGGL(world_hit_kernel<TRAV_REFERENCE>, dim3(grid), dim3(kBlock), lds, stream, S, n, orig, dir,
                           out);
    return hipGetLastError();
}

}  // namespace rt
