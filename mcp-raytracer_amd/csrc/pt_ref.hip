// Reference-precision build of the path tracer (Real = double, fp32 vector
// stores). Compiled with -ffp-contract=off so every scalar op rounds exactly as
// the reference's JS doubles do.
#include "launch.hpp"

#include <algorithm>
#include <cstdlib>

namespace rt {

hipError_t launch_render_ref(const KernelVariant& v, const DevScene& S, const RtRegion& reg, const RenderOut& out,
                             const LaunchGeom& g, const SampleBuf* sb, hipStream_t stream) {
    return dispatch_render<double>(v, S, reg, out, g, sb, stream);
}

__global__ void init_stats_kernel(unsigned long long* stats, unsigned long long* counters,
                                  unsigned int* tile_counter) {
    const int t = threadIdx.x;
    if (t < ST_WORDS) stats[t * kStatStride] = (t == ST_SMIN || t == ST_BMIN) ? ~0ull : 0ull;
    if (counters && t < kCounterWords) counters[t] = 0ull;
    if (t < 2) tile_counter[t] = 0u;  // bulk and tail item counters
}

constexpr int kAccBlock = 256;
constexpr int kAccUnroll = 8;
// Adds every pixel's samples in sample order (PixelStats.add), then
// finalColor / u8 / RenderStats exactly as the sequential kernel.
__global__ __launch_bounds__(kAccBlock) void pt_accum_kernel(DevScene S0, RtRegion reg, RenderOut out, int tiles_x,
                                                              SampleBuf sb) {
    const RtCamera& C = S0.cam;
    const int lane = threadIdx.x & (kWave - 1);
    PixStats st;
    // grid-stride over the pass's pixel slots: few blocks, one stats merge per block
    for (int slot = blockIdx.x * blockDim.x + threadIdx.x; slot < sb.slots; slot += gridDim.x * blockDim.x) {
        int i, j;
        item_pixel(reg, tiles_x, sb.tile0 + slot / 64, slot % 64, i, j);
        if (i < min(reg.x + reg.width, C.width) && j < min(reg.y + reg.height, C.height)) {
            V3 color = v3(0, 0, 0);
            unsigned long long bsum = 0;
            int bmin = 0x7fffffff, bmax = 0;
            const int n = C.n_samples;
            // kAccUnroll loads in flight; sample-major records are coalesced across the
            // wave, slot-major ones are one contiguous run per lane
            const size_t stride = (size_t)sb.stride_s;
            int k = 0;
            if (sb.rec12) {  // {r, g, b} records: the path kernel reduced the bounce statistics
                             // (bsum 0, bmin / bmax at their neutral values here)
                // (addresses in floats: a 3-element vector type's size is 16 bytes, its loads 12)
                const float* rec3 = reinterpret_cast<const float*>(sb.rec) + 3 * (size_t)slot * sb.stride_slot;
                const size_t step = 3 * stride;
                for (; k + kAccUnroll <= n; k += kAccUnroll) {
                    RecF3 r[kAccUnroll];
#pragma unroll
                    for (int m = 0; m < kAccUnroll; ++m) r[m] = *reinterpret_cast<const RecF3*>(rec3 + (size_t)(k + m) * step);
#pragma unroll
                    for (int m = 0; m < kAccUnroll; ++m) color = add(color, v3(r[m].x, r[m].y, r[m].z));
                }
                for (; k < n; ++k) {
                    const RecF3 r = *reinterpret_cast<const RecF3*>(rec3 + (size_t)k * step);
                    color = add(color, v3(r.x, r.y, r.z));
                }
            }
            const float4* rec = sb.rec + (size_t)slot * sb.stride_slot;
            for (; k + kAccUnroll <= n; k += kAccUnroll) {
                float4 r[kAccUnroll];
#pragma unroll
                for (int m = 0; m < kAccUnroll; ++m) r[m] = rec[(size_t)(k + m) * stride];
#pragma unroll
                for (int m = 0; m < kAccUnroll; ++m) {
                    color = add(color, v3(r[m].x, r[m].y, r[m].z));
                    const int b = __float_as_int(r[m].w);
                    bsum += (unsigned long long)b;
                    bmin = min(bmin, b);
                    bmax = max(bmax, b);
                }
            }
            for (; k < n; ++k) {
                const float4 r = rec[(size_t)k * stride];
                color = add(color, v3(r.x, r.y, r.z));
                const int b = __float_as_int(r.w);
                bsum += (unsigned long long)b;
                bmin = min(bmin, b);
                bmax = max(bmax, b);
            }
            const uint32_t opix = out.packed ? (uint32_t)sb.tile0 * kWave + (uint32_t)slot
                                             : (uint32_t)j * (uint32_t)C.width + (uint32_t)i;
            finish_pixel(C, out, opix, color, n, bsum, bmin, bmax, st);
        }
    }
    // RenderStats.merge: waves -> LDS -> one lane per block
    __shared__ unsigned long long red[kAccBlock / kWave][7];
    const int w = threadIdx.x / kWave;
    const unsigned long long v[7] = {wave_sum(st.pixels), wave_sum(st.samples), wave_min(st.smin), wave_max(st.smax),
                                     wave_sum(st.b),      wave_min(st.bmin),    wave_max(st.bmax)};
    if (lane == 0)
        for (int q = 0; q < 7; ++q) red[w][q] = v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a[7];
        for (int q = 0; q < 7; ++q) a[q] = red[0][q];
        for (int u = 1; u < kAccBlock / kWave; ++u) {
            a[0] += red[u][0];
            a[1] += red[u][1];
            a[2] = min(a[2], red[u][2]);
            a[3] = max(a[3], red[u][3]);
            a[4] += red[u][4];
            a[5] = min(a[5], red[u][5]);
            a[6] = max(a[6], red[u][6]);
        }
        stats_atomics(out, a[0], a[1], a[2], a[3], a[4], a[5], a[6], 0ull);
    }
}

// One round of adaptive sampling (src/camera.ts:400-425, pixelConverged 348-368):
// every pixel of the round's active list adds the round's samples to its running
// PixelStats in sample order, checking convergence after each one exactly as the
// reference's while loop does (pixel_converged tests n % aBatch itself), and stops
// at the first converged check - samples the round rendered past it are dropped,
// so the result is the sequential loop's. Finished pixels (converged or n ==
// samples) get finalColor / u8 / RenderStats; the rest carry their state to the
// next round's active list (order irrelevant: every pixel's result depends on its
// own samples only). One atomic per block-iteration appends to the list.
__global__ __launch_bounds__(kAccBlock) void pt_adapt_kernel(DevScene S0, RtRegion reg, RenderOut out, int tiles_x,
                                                              SampleBuf sb, AdaptRound ar) {
    const RtCamera& C = S0.cam;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const double rtx = 1.0 / (double)tiles_x;
    const int endX = min(reg.x + reg.width, C.width), endY = min(reg.y + reg.height, C.height);
    PixStats st;
    unsigned long long st_err = 0;
    __shared__ unsigned int wcnt[kAccBlock / kWave];
    __shared__ unsigned int wbase;
    const int stride = gridDim.x * blockDim.x;
    const int n_iter = (sb.slots + stride - 1) / stride;  // block-uniform trip count (the append syncs)
    for (int it = 0; it < n_iter; ++it) {
        const int a = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
        int i = 0, j = 0;
        const bool valid = a < sb.slots && slot_pixel(sb, reg, tiles_x, rtx, endX, endY, a, i, j);
        const int ls = valid ? (sb.act ? sb.act[a] : sb.tile0 * kWave + a) : 0;
        bool carry = false, likely = false;
        if (valid) {
            V3 color = v3(0, 0, 0);
            int n = 0, bmin = 0x7fffffff, bmax = 0;
            unsigned long long bsum = 0;
            double sIll = 0.0, sIll2 = 0.0;
            unsigned long long err = 0;  // error flags of the samples kept (SampleBuf::err_in_rec)
            if (sb.s_base > 0) {
                const AdaptPix q = ar.state[ls];
                color = v3(q.c.x, q.c.y, q.c.z);
                n = __float_as_int(q.c.w);
                sIll = q.ill.x;
                sIll2 = q.ill.y;
                bsum = (unsigned long long)(uint32_t)q.b.x | ((unsigned long long)(uint32_t)q.b.w << 32);
                bmin = q.b.y;
                bmax = q.b.z;
            }
            bool done = false;
            const float4* rec = sb.rec + (size_t)a * sb.stride_slot;
            // fmod(n, aBatch) == 0 is n % aBatch == 0 for an integral aBatch: count down to those n
            // (the fp64 fmod per sample was most of this kernel's arithmetic)
            const double abd = C.a_batch;
            const bool ib = abd >= 1.0 && abd < 2147483648.0 && abd == ::floor(abd);
            const int batch = ib ? (int)abd : 1;
            int until = ib ? batch - n % batch : 0;  // samples to add until n is the next multiple
            for (int k = 0; k < ar.len && !done; ++k) {
                // PixelStats.add (renderStats.ts:76-88), then the while condition
                const float4 r = rec[(size_t)k * sb.stride_s];
                const V3 c = v3(r.x, r.y, r.z);
                color = add(color, c);
                ++n;
                const uint32_t bw = __float_as_uint(r.w);
                const int b = (int)(bw & kRecBounceMask);
                err |= (unsigned long long)(bw >> kRecErrShift);
                bsum += (unsigned long long)b;
                bmin = min(bmin, b);
                bmax = max(bmax, b);
                const double il = illuminance(c);
                sIll += il;
                sIll2 += il * il;
                if (ib) {
                    const bool check = --until == 0;
                    if (check) until = batch;
                    done = n >= C.n_samples || (check && pixel_converged_at_batch(C, n, sIll, sIll2));
                } else {
                    done = n >= C.n_samples || pixel_converged(C, n, sIll, sIll2);
                }
            }
            st_err |= err;
            if (done) {
                const uint32_t opix = out.packed ? (uint32_t)ls : (uint32_t)j * (uint32_t)C.width + (uint32_t)i;
                finish_pixel(C, out, opix, color, n, bsum, bmin, bmax, st);
            } else {
                AdaptPix q;
                q.c = make_float4(color.x, color.y, color.z, __int_as_float(n));
                q.ill = make_double2(sIll, sIll2);
                q.b = make_int4((int)(uint32_t)bsum, bmin, bmax, (int)(uint32_t)(bsum >> 32));
                ar.state[ls] = q;
                carry = true;
                // round-length rule only (never a result): would pixelConverged's interval,
                // 1.96 sqrt(var / n) <= aTolerance * mean at the current mean and variance,
                // close by n = horizon? (zero or NaN variance: at the next check)
                const double mean = sIll / n;
                const double var = n > 1 ? (sIll2 - (sIll * sIll) / n) / (n - 1) : 0.0;
                likely = !(var > 0.0) ||
                         (mean > 0.0 && 3.8416 * var <= (double)ar.horizon * C.a_tolerance * C.a_tolerance * mean * mean);
            }
        }
        {
            const unsigned long long ml = __ballot(likely);
            if (lane == 0 && ml) atomicAdd(ar.next_count + 1, (unsigned int)__popcll(ml));
        }
        // append the carried pixels: one atomic per block and iteration
        const unsigned long long m = __ballot(carry);
        if (lane == 0) wcnt[w] = (unsigned int)__popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned int tot = 0;
            for (int q = 0; q < kAccBlock / kWave; ++q) {
                const unsigned int c = wcnt[q];
                wcnt[q] = tot;
                tot += c;
            }
            wbase = tot ? atomicAdd(ar.next_count, tot) : 0u;
        }
        __syncthreads();
        if (carry) {
            const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            ar.next_act[wbase + wcnt[w] + (unsigned int)r] = ls;
        }
        __syncthreads();
    }
    __shared__ unsigned long long red[kAccBlock / kWave][8];
    const unsigned long long v[8] = {wave_sum(st.pixels), wave_sum(st.samples), wave_min(st.smin), wave_max(st.smax),
                                     wave_sum(st.b),      wave_min(st.bmin),    wave_max(st.bmax), wave_or(st_err)};
    if (lane == 0)
        for (int q = 0; q < 8; ++q) red[w][q] = v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t[8];
        for (int q = 0; q < 8; ++q) t[q] = red[0][q];
        for (int u = 1; u < kAccBlock / kWave; ++u) {
            t[0] += red[u][0];
            t[1] += red[u][1];
            t[2] = min(t[2], red[u][2]);
            t[3] = max(t[3], red[u][3]);
            t[4] += red[u][4];
            t[5] = min(t[5], red[u][5]);
            t[6] = max(t[6], red[u][6]);
            t[7] |= red[u][7];
        }
        stats_atomics(out, t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7]);
    }
}

hipError_t launch_adapt(const DevScene& S, const RtRegion& reg, const RenderOut& out, int tiles_x,
                        const SampleBuf& sb, const AdaptRound& ar, hipStream_t stream) {
    const int grid = std::max(1, std::min((sb.slots + kAccBlock - 1) / kAccBlock, 2 * 256 * 1024 / kAccBlock));
    hipLaunchKernelGGL(pt_adapt_kernel, dim3(grid), dim3(kAccBlock), 0, stream, S, reg, out, tiles_x, sb, ar);
    return hipGetLastError();
}

hipError_t launch_accum(const DevScene& S, const RtRegion& reg, const RenderOut& out, int tiles_x,
                        const SampleBuf& sb, hipStream_t stream) {
    // at most 1024 blocks (4 per CU), grid-stride beyond: the accumulate pass streams the records
    // at ~5.6 TB/s either way; 1024 measured 2-3 % faster than 2048 or 4096 (Cornell 0.47 ->
    // 0.455 ms, rain 3.19 -> 3.10 ms; profiles/r04/acc/). RT_AMD_ACC_BLOCKS overrides (A/B).
    const char* e = std::getenv("RT_AMD_ACC_BLOCKS");
    const int cap = e ? std::max(1, std::atoi(e)) : 1024;
    const int grid = std::max(1, std::min((sb.slots + kAccBlock - 1) / kAccBlock, cap));
    hipLaunchKernelGGL(pt_accum_kernel, dim3(grid), dim3(kAccBlock), 0, stream, S, reg, out, tiles_x, sb);
    return hipGetLastError();
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
    const int h = closest_hit_any<double, false, TRAV>(S, S.cam.n_prims, r, t, stk, nullptr);
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

// The device's Math.cos / Math.sin of the cosine-PDF angle and Schlick's
// Math.pow(x, 5), with the path code's own expressions (pt_kernel.hpp path_post,
// dielectric_dir): phi = 2 * PI * xi, xi = u * 2^-32.
__global__ void math_probe_kernel(int n, const uint32_t* u, double* out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double xi = (double)u[k] * (1.0 / 4294967296.0);
    const double phi = 2.0 * K<double>::PI * xi;
    double sn, cs;
    m_sincos(phi, sn, cs);
    out[3 * k] = cs;
    out[3 * k + 1] = sn;
    out[3 * k + 2] = pow5(xi);
}

// rt_debug_fp64: the restricted-domain sqrt / reciprocal (rt_math.hpp) beside the general ones
__global__ void fp64_probe_kernel(int n, const double* x, double* out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double v = x[k];
    out[4 * k] = sqrt_rn(v);
    out[4 * k + 1] = ::sqrt(v);
    out[4 * k + 2] = rcp_rn(v);
    out[4 * k + 3] = 1.0 / v;
}
hipError_t launch_fp64_probe(int n, const double* x, double* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fp64_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, x, out);
    return hipGetLastError();
}

hipError_t launch_math_probe(int n, const uint32_t* u, double* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, u, out);
    return hipGetLastError();
}

hipError_t launch_world_hit_ref(const DevScene& S, int trav, int n, const float* orig, const float* dir,
                                double* out, hipStream_t stream) {
    const int grid = (n + kBlock - 1) / kBlock;
    const size_t lds = std::max(stack_lds_bytes(S.cam.stack_depth, TRAV_FAST, S.cam.n_prims),
                                stack_lds_bytes(S.cam.stack_depth, TRAV_BRUTE, S.cam.n_prims));  // largest footprint
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
