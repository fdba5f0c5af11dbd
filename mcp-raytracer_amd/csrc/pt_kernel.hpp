// The path-tracing hot path as one persistent HIP kernel for gfx950.
//
// Restates, per lane, Camera.renderRegion's pixel loop (src/camera.ts:388-431)
// with getRay (176-210), the rayColor recursion turned into a bounce loop
// (221-319), BVH traversal (src/geometry/bvh.ts:128-146, aabb.ts:30-55,
// hittableList.ts:71-87), sphere/quad/plane intersection (src/entities/*),
// material scatter (src/materials/*), the mixture-PDF light sampling
// (src/geometry/pdf.ts) and the spp accumulate (src/render-utils/renderStats.ts:76-88).
//
// Work decomposition (MI355X): a wave owns an 8x8 pixel tile, one pixel per
// lane; waves pull tiles from a global atomic counter (persistent grid, load
// balanced across the 256 CUs / 8 XCDs). Each lane renders its pixel's samples
// in order - the reference accumulates samples sequentially in fp32, so the
// per-pixel order is part of the result - but lanes are NOT synchronised per
// sample: a lane whose path terminates immediately starts its next sample in
// the same loop trip (path regeneration), so the wave runs for
// max_lane(sum of path lengths), not sum_samples(max_lane(path length)).
// The BVH traversal stack lives in LDS, lane-interleaved ([depth][lane]) so
// every push/pop is a conflict-free ds_write/ds_read_b32.
//
// Numerics: `Real` = double restates the reference exactly (fp64 scalars,
// fp32 vector stores; built with -ffp-contract=off); Real = float is the fp32
// fast mode. See rt_math.hpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "rt_math.hpp"
#include "scene.hpp"

namespace rt {

// The scene lives in one device buffer ("blob"): [tnodes][tprims][tsph][prims][mats][lights][nodes],
// 16-byte aligned sections. When [tnodes][prims] fits, every workgroup copies
// it into LDS (LDS-resident launch): traversal and primitive reads are LDS reads.
struct DevScene {
    const RtTNode* __restrict__ tnodes; // fast traversal: children-in-parent nodes (blob start)
    const RtPrim* __restrict__ prims;   // global, or LDS in an LDS-resident launch
    const RtPrim* __restrict__ gprims;  // always the global copy (scalar-load reads)
    const RtPre* __restrict__ gpre;     // brute-force pre-filter records (global, scalar-load reads)
    int32_t n_pre;                      // ... and their count (pairs count once)
    const RtExact* __restrict__ xrec;   // brute-force exact-test records (LDS when resident), slot order
    int32_t off_xrec;                   // byte offset of xrec in the blob
    const int32_t* __restrict__ tprims; // fast-traversal leaves -> primitive slots (LDS when resident)
    const float4* __restrict__ tsph;    // per tprims entry: sphere {centre, fp32 radius} or NaNs (LDS when resident)
    const RtMat* __restrict__ mats;
    const RtLight* __restrict__ lights;
    const RtLight* __restrict__ glights; // always the global copy (scalar-load reads)
    const RtNode* __restrict__ nodes;   // the reference's boxes (reference traversal)
    const RtOnb* __restrict__ onbs;     // [slot][precision][face] for slots < n_onb (LDS at level 2)
    int32_t n_onb;                      // planar primitives' ONB table covers slots [0, n_onb)
    int32_t off_onbs;                   // byte offset of onbs in the blob
    const uint4* __restrict__ blob;     // the whole scene: [tnodes][tprims][tsph][prims][mats][lights][nodes]
    int32_t lds_words;                  // 16-byte words of the blob prefix copied to LDS (LDSS 1: [tnodes][tprims][tsph][prims],
                                        // LDSS 2: also [mats][lights])
    int32_t off_prims;                  // byte offset of prims in the blob
    int32_t off_mats;                   // byte offset of mats in the blob
    int32_t off_lights;                 // byte offset of lights in the blob
    int32_t off_tprims;                 // byte offset of tprims in the blob
    int32_t off_tsph;                   // byte offset of tsph in the blob
    int32_t lds_stack_bytes;            // LDS bytes of the traversal stack (scene follows)
    int32_t lds_pool_off;               // pool kernel: byte offset of the per-wave path pools (after the scene)
    int32_t lds_node_pad;               // LDS copy: one 16-byte pad row after each 4-wide node (t4 nodes, or 0)
    int32_t t4_stride;                  // bytes between 4-wide nodes where the walk reads them (128 or 144)
    int32_t n_top;                      // launches walking the tree from global memory: nodes [0, n_top)
                                        // (breadth-first: the tree's top) have a padded copy in LDS
    const char* top_lds;                // ... after the traversal stack (scene_view; LDSS 0 only)
    const RtLeafSph* __restrict__ tsph2; // trees walked from global memory: leaf-order sphere records with
                                         // the fp64 radius and the slot (one load per exact test), or null
    int32_t nearfar;                    // 4-wide node step picks near / far rows by the ray's signs (t4_step);
                                        // scene_view sets a constant per LDS level (see there)
    int32_t troot;                      // fast traversal root reference
    RtNode root_box;                    // fast traversal root box (padded)
    RtCamera cam;
    double mix_total;  // MixturePDF.totalWeight for [0.5, 0.5/nL x nL]
    double light_w;    // 0.5 / nL
};

// Stats words (u64): pixels, samples total, samples min, samples max,
// bounces total, bounces min, bounces max, error flags.
enum { ST_PIXELS = 0, ST_SAMPLES, ST_SMIN, ST_SMAX, ST_BOUNCES, ST_BMIN, ST_BMAX, ST_ERROR, ST_WORDS };
// Each stats word on a 128-byte line of its own (stats[k * kStatStride]): the atomics of
// thousands of waves on one line serialise (~90 per us per line).
constexpr int kStatStride = 16;
// Instrumentation words (u64): the algorithmic-work counts of SURVEY.md §8d.
enum {
    CT_NODE = 0, CT_SPHERE, CT_QUAD, CT_PLANE, CT_MATERIAL, CT_LIGHT_QUAD, CT_LIGHT_SPHERE,
    CT_BOUNCES, CT_DIFFUSE, CT_SAMPLES, CT_RAYS,
    CT_EXACT,       // primitives whose exact fp64 test ran (per lane)
    CT_EXACT_WAVE,  // exact-test blocks a wave executed (any lane), counted once per wave
    CT_CAND0,       // brute force: rays with no pre-filter candidate
    CT_CAND2,       // brute force: rays with two or more pre-filter candidates
    CT_EXACT2,      // brute force: rays that needed two or more exact tests
    CT_WORDS
};
enum : unsigned long long { ERR_NO_BACKGROUND = 1ull, ERR_EMIT_STACK = 2ull };
constexpr int kRecErrShift = 30;  // error flags in a sample record's bounce word (SampleBuf::err_in_rec)
constexpr uint32_t kRecBounceMask = (1u << kRecErrShift) - 1u;
// Diagnostic build (INSTR == 2): wave-cycles spent in each section of the path
// loop (s_memtime, summed over waves), stored after the CT_WORDS counters.
enum {
    PR_NEWPATH = 0, PR_RR, PR_HIT, PR_MISS, PR_HITREC, PR_SCATTER, PR_SAMPLE, PR_PDF, PR_ACC, PR_TILE,
    PR_NODE, PR_LEAF,  // lane counts only (no cycles): node-step and leaf-test iterations of the walk
    PR_WNODE, PR_WLEAF,  // resumable walk: cycles of its node-step loops / leaf phases (part of PR_HIT's walk)
    PR_LOOP, PR_TRIPS, PR_WORDS
};
// INSTR == 2 also records, per section k < PR_LOOP, the lanes active when a wave
// ended it (summed, at CT_WORDS + PR_WORDS + k) and how many times a wave did
// (at CT_WORDS + PR_WORDS + PR_LOOP + k): active lanes per execution of a section.
struct Prof;  // diagnostic section timer (below)
template <bool PROF>
__device__ __forceinline__ void pcount(Prof& pf, int k);
template <bool PROF>
__device__ __forceinline__ void psec(Prof& pf, int k);
constexpr int kCounterWords = 64;  // CT_WORDS + PR_WORDS + 2 * PR_LOOP, rounded up
static_assert(CT_WORDS + PR_WORDS + 2 * PR_LOOP <= kCounterWords, "counter words");

struct RenderOut {
    uint8_t* rgb;        // W*H*3 (full frame layout), may be null
    float* radiance;     // W*H*3, may be null
    int32_t* px_samples; // W*H, may be null
    int32_t* px_bounces; // W*H, may be null
    unsigned long long* stats;     // ST_WORDS words, kStatStride apart
    unsigned long long* counters;  // kCounterWords (instrumented builds only)
    unsigned int* tile_counter;
    // 0: outputs in full-frame layout (index j*W + i); 1: tile-packed slab, the
    // pixel of lane l of this launch's k-th tile at k*64 + l (multi-GPU gather)
    int32_t packed;
};

// Closest-hit strategies; all return the reference's hit bit-for-bit (see the
// functions below). AUTO is resolved on the host.
enum Traversal : int32_t { TRAV_FAST = 0, TRAV_REFERENCE = 1, TRAV_BRUTE = 2, TRAV_AUTO = 3,
                           TRAV_FAST_DEFER = 4 };  // kernel-internal: FAST with deferred exact sphere tests
constexpr bool trav_fast(int t) { return t == TRAV_FAST || t == TRAV_FAST_DEFER; }
constexpr int kBruteMaxPrims = 16;  // AUTO picks BRUTE up to this many primitives (nearest-first form: <= 32)

constexpr int kWave = 64;
// Persistent workgroups, one per CU, sharing one LDS scene copy:
//   sequential kernel 768 threads (12 waves = 3 per SIMD, <= 168 VGPRs),
//   chunked kernel 1024 threads (16 waves = 4 per SIMD, <= 128 VGPRs).
constexpr int kBlock = 768;
constexpr int kBlockChunk = 1024;
constexpr int kStackStride = 1024;  // LDS traversal-stack column stride (>= any block size)
// Stack entries of the fast walk: 16-bit in launches whose tree is LDS-resident (its
// node references and leaf codes ~(first << 3 | count) fit an int16: at most ~1,000 nodes and
// primitives fit the LDS copy), so the stack takes half the LDS and the material / light tables
// fit beside it (LDS residency level 2); 32-bit where the tree is walked from global memory.
// Entries hold a node reference only (a popped subtree is culled one level later by its
// children's slab tests).
template <int LDSS>
using StackT = typename std::conditional<(LDSS > 0), int16_t, int32_t>::type;
constexpr int kTile = 8;          // 8x8 pixels per wave-tile
constexpr int kEmitStack = 128;   // emission terms kept for the right fold (EMIT builds)

// ---------------------------------------------------------------------------
// Seeded replacement for Math.random: PCG32 (XSH-RR) stream per (seed, pixel,
// sample), consumed in the reference's draw order.
// ---------------------------------------------------------------------------
// seed_mix = splitmix64(seed), precomputed per camera (RtCamera::seed_mix)
__device__ __forceinline__ uint64_t rng_init(uint64_t seed_mix, uint32_t pixel, uint32_t sample) {
    return splitmix64((((uint64_t)pixel << 32) | sample) ^ seed_mix);
}
__device__ __forceinline__ uint32_t rng_u32(uint64_t& s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}
template <class Real> __device__ __forceinline__ Real uniform(uint64_t& s);
template <> __device__ __forceinline__ double uniform<double>(uint64_t& s) {
    return (double)rng_u32(s) * (1.0 / 4294967296.0);
}
template <> __device__ __forceinline__ float uniform<float>(uint64_t& s) {
    return (float)(rng_u32(s) >> 8) * (1.0f / 16777216.0f);
}

// Math.* on the scalar type.
__device__ __forceinline__ double m_cos(double x) { return ::cos(x); }
__device__ __forceinline__ float m_cos(float x) { return ::cosf(x); }
__device__ __forceinline__ double m_sin(double x) { return ::sin(x); }
__device__ __forceinline__ float m_sin(float x) { return ::sinf(x); }
// Math.cos(x) and Math.sin(x) of one argument: ocml's sincos evaluates the sine and cosine
// polynomials once (separate sin + cos calls each evaluate both and select) and returns
// bit-for-bit sin(x) and cos(x) (tools/probes/sincos_check: all 2^32 cosine-PDF angles, fp64
// and fp32). Cornell 7718 -> 7933 Msamples/s (profiles/r01/sincos/).
template <class Real>
__device__ __forceinline__ void m_sincos(Real x, Real& s, Real& c) {
    if constexpr (sizeof(Real) == 8) ::sincos(x, &s, &c);
    else ::sincosf(x, &s, &c);
}
// Math.pow(x, 5) of Schlick's approximation (src/materials/dielectric.ts:98),
// correctly rounded: x^5 in double-double (exact x^2 and x^4 products via FMA),
// then one rounding. V8's and glibc's pow are within 1 ulp of this value (and
// differ from it for ~0.1 % of arguments); it only feeds `reflectance > xi`.
// The oracle computes the same correctly rounded value independently (binary128).
__device__ __forceinline__ double pow5(double x) {
    const double h2 = x * x, l2 = ::fma(x, x, -h2);
    const double h4 = h2 * h2, l4 = ::fma(h2, h2, -h4) + 2.0 * h2 * l2;
    const double h5 = h4 * x, l5 = ::fma(h4, x, -h5) + l4 * x;
    return h5 + l5;
}
__device__ __forceinline__ float pow5(float x) {
    const float x2 = x * x;
    return x2 * x2 * x;
}
__device__ __forceinline__ double m_abs(double x) { return ::fabs(x); }
__device__ __forceinline__ float m_abs(float x) { return ::fabsf(x); }
// Math.sqrt. (Routing it through rt_math.hpp sqrt_rn behind a range test was no faster anywhere:
// the branch costs what the skipped scaling steps save, profiles/r04/fp64/.)
__device__ __forceinline__ double m_sqrt(double x) { return ::sqrt(x); }
__device__ __forceinline__ float m_sqrt(float x) { return ::sqrtf(x); }

template <class Real> struct K {
    static constexpr Real PI = (Real)3.141592653589793;
    static constexpr Real TMIN = (Real)0.001;
};

__device__ __forceinline__ V3 ld3(const float* p) { return V3{p[0], p[1], p[2]}; }

// Wave-uniform reads of scene records that are never written during a launch:
// through the constant address space, so the compiler emits scalar loads
// (s_load, scalar cache) instead of vector loads with full memory latency.
template <class T>
__device__ __forceinline__ T ld_uniform(const T* base, int k) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    typedef const __attribute__((address_space(4))) uint32_t* CW;
    const CW src = (CW)(const void*)(base + k);
    T out;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = src[i];
    return out;
}

// Per-ray constants reused by every node and primitive test.
template <class Real> struct RayK {
    V3 o, d;
    Real inv[3];  // 1/d[a] (AABB.hit computes it per node; same value)
    Real a;       // d.lengthSquared() (Sphere.hit computes it per sphere; same value)
};

template <class Real>
__device__ __forceinline__ RayK<Real> make_ray(V3 o, V3 d) {
    RayK<Real> r;
    r.o = o;
    r.d = d;
    r.inv[0] = (Real)1 / (Real)d.x;
    r.inv[1] = (Real)1 / (Real)d.y;
    r.inv[2] = (Real)1 / (Real)d.z;
    r.a = len2<Real>(d);
    return r;
}

// The ray as the exact (Real) tests inside a traversal loop see it: o and d
// pass through an empty asm so their conversions to Real (and |d|^2) are
// redone per test instead of being hoisted out of the loop as long-lived fp64
// values - which the register allocator then spills to scratch every trip.
// Values are unchanged; the tests run on a small fraction of loop iterations.
template <class Real>
__device__ __forceinline__ RayK<Real> ray_at_use(const RayK<Real>& r) {
    RayK<Real> q = r;
    asm volatile("" : "+v"(q.o.x), "+v"(q.o.y), "+v"(q.o.z), "+v"(q.d.x), "+v"(q.d.y), "+v"(q.d.z));
    q.a = len2<Real>(q.d);
    return q;
}

// AABB.hit (src/geometry/aabb.ts:30-55): each axis is clipped against the
// ORIGINAL interval (the reference does not carry tMin/tMax across axes);
// comparisons keep the reference's NaN behaviour.
template <class Real>
__device__ __forceinline__ bool box_hit(const RtNode& n, const RayK<Real>& r, Real tmin, Real tmax) {
    const float o[3] = {r.o.x, r.o.y, r.o.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const Real invD = r.inv[a];
        Real t0 = ((Real)n.bmin[a] - (Real)o[a]) * invD;
        Real t1 = ((Real)n.bmax[a] - (Real)o[a]) * invD;
        if (invD < (Real)0) { Real tmp = t0; t0 = t1; t1 = tmp; }
        const Real lo = t0 > tmin ? t0 : tmin;
        const Real hi = t1 < tmax ? t1 : tmax;
        if (hi <= lo) return false;
    }
    return true;
}

template <class Real> __device__ __forceinline__ Real sphere_radius(const RtPrim& p);
template <> __device__ __forceinline__ double sphere_radius<double>(const RtPrim& p) { return p.s0; }
template <> __device__ __forceinline__ float sphere_radius<float>(const RtPrim& p) { return p.g0[3]; }
// 1 / radius (Vec3.divide's reciprocal, vec3.ts:126-130), computed on the host with the same
// IEEE division: sphere records carry it in g1 (double bits in g1[0..1], fp32 in g1[2]).
template <class Real> __device__ __forceinline__ Real sphere_inv_radius(const RtPrim& p);
template <> __device__ __forceinline__ double sphere_inv_radius<double>(const RtPrim& p) {
    return __hiloint2double(__float_as_int(p.g1[1]), __float_as_int(p.g1[0]));
}
template <> __device__ __forceinline__ float sphere_inv_radius<float>(const RtPrim& p) { return p.g1[2]; }
template <class Real> __device__ __forceinline__ Real plane_d(const RtPrim& p);
template <> __device__ __forceinline__ double plane_d<double>(const RtPrim& p) { return p.s0; }
template <> __device__ __forceinline__ float plane_d<float>(const RtPrim& p) { return p.g0[3]; }

// Sphere.hit root selection (src/entities/sphere.ts:45-65); returns t only.
template <class Real>
__device__ __forceinline__ bool sphere_t_cr(V3 c, Real rad, const RayK<Real>& r, Real tmin, Real tmax, Real& t) {
    const V3 oc = sub(r.o, c);
    const Real halfB = dot<Real>(oc, r.d);
    const Real cc = len2<Real>(oc) - rad * rad;
    const Real disc = halfB * halfB - r.a * cc;
    if (disc < (Real)0) return false;
    const Real sq = m_sqrt(disc);
    Real root = (-halfB - sq) / r.a;
    if (!(tmin < root && root < tmax)) {
        root = (-halfB + sq) / r.a;
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}
template <class Real>
__device__ __forceinline__ bool sphere_t(const RtPrim& p, const RayK<Real>& r, Real tmin, Real tmax, Real& t) {
    return sphere_t_cr<Real>(ld3(p.g0), sphere_radius<Real>(p), r, tmin, tmax, t);
}

// Plane.intersect (src/entities/plane.ts:55-77) + Quad bounds (quad.ts:50-76).
template <class Real, bool QUAD>
__device__ __forceinline__ bool planar_t(const RtPrim& p, const RayK<Real>& r, Real tmin, Real tmax, Real& t) {
    const V3 n = ld3(p.g3);
    const Real denom = dot<Real>(n, r.d);
    if (m_abs(denom) < (Real)1e-8) return false;
    const Real tt = (plane_d<Real>(p) - dot<Real>(n, r.o)) / denom;
    if (!(tmin < tt && tt < tmax)) return false;
    if (QUAD) {
        const V3 ip = ray_at<Real>(r.o, r.d, tt);
        const V3 ph = sub(ip, ld3(p.g0));
        const V3 w = ld3(p.g4);
        const Real alpha = dot<Real>(w, cross<Real>(ph, ld3(p.g2)));
        const Real beta = dot<Real>(w, cross<Real>(ld3(p.g1), ph));
        if (alpha < (Real)0 || alpha > (Real)1 || beta < (Real)0 || beta > (Real)1) return false;
    }
    t = tt;
    return true;
}

constexpr float kTminLo = 0.001f * (1.0f - 1e-5f);  // below the reference's tMin with margin (fp32 tests)
// fp32 pre-filter error model: every estimate below is an fp32 evaluation of the
// reference's fp64 formula, off by at most a few tens of ulps of the operand
// magnitudes (products of fp32 values are exact in fp64). kRel (~170 ulps)
// bounds that with a wide margin; the margins scale with |o|, |d|, |Q|, r so
// they hold for any scene scale. Hardware rcp/sqrt (<= 1 ulp) are inside kRel.
constexpr float kRel = 1e-5f;

// The fp32 conservative filters (slab tests, sphere / planar / axis-quad pre-filters, the
// FRay constants, the culling bound) may contract a*b+c into one FMA even in the ref TU,
// which is compiled with -ffp-contract=off because the reference's JS arithmetic never
// fuses. That flag must keep holding for the fp64 path and for the fp32 vector stores of
// the exact tests, so contraction is opened per function body (RT_FP32_FUSED, a block-
// scoped pragma: it marks only the operations written inside that block, and inlining
// keeps the marks per operation). A filter's result reaches the output only through the
// exact fp64 test it lets through, so the filter may round differently as long as it stays
// conservative. Every margin below is of the form c * u * (sum of the magnitudes of the
// terms): a fused a*b+c rounds once where the unfused form rounds twice, so each margin
// still bounds it. The one changed form is the slab test, which no longer subtracts first
// (see slab_t4 / FRay::eps). Before: SQ_INSTS_VALU_FMA_F32 was 0.0 % of VALU
// on Cornell ref, 1.0 % on spheres-500 and 0.5 % on spheres-100k.
#define RT_FP32_FUSED _Pragma("clang fp contract(fast)")

// Axis-aligned quad (scene.cpp encode_axis_quad): Plane.intersect + Quad's
// alpha/beta test with the terms that are exact zeros dropped. Every kept
// operation is the reference's own (a product of two fp32 values is exact in
// double, x - (+-0) = x, sums with +-0 are exact), so t and the accept/reject
// decision are bit-identical to planar_t - provided no 0*inf/NaN term would
// have turned the reference's result into NaN, which the finiteness guard
// reproduces (a non-finite off-axis ray component makes the reference miss).
// One specialisation per axis code (constant indices: no selects, no branches).
template <class Real, int CODE>
__device__ __forceinline__ bool aquad_t_c(const RtPrim& p, V3 o3, V3 d3, Real tmin, Real tmax, Real& t) {
    constexpr int a = (CODE - 1) % 3, vflag = (CODE - 1) / 3;
    constexpr int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
    const float o[3] = {o3.x, o3.y, o3.z}, d[3] = {d3.x, d3.y, d3.z};
    if (!(::isfinite(o[ia]) && ::isfinite(d[ia]) && ::isfinite(o[ib]) && ::isfinite(d[ib]))) return false;
    const Real na = (Real)p.g3[a];
    const Real denom = na * (Real)d[a];
    if (m_abs(denom) < (Real)1e-8) return false;
    const Real tt = (plane_d<Real>(p) - na * (Real)o[a]) / denom;
    if (!(tmin < tt && tt < tmax)) return false;
    // Ray.at(t) in-plane components, hit point minus Q (fp32 stores)
    const float ph1 = (o[ia] + (float)((Real)d[ia] * tt)) - p.g0[ia];
    const float ph2 = (o[ib] + (float)((Real)d[ib] * tt)) - p.g0[ib];
    const Real sw = (Real)p.g3[3];
    const Real alpha = sw * (Real)(ph1 * p.g2[3]);
    const Real beta = sw * (Real)(ph2 * p.g1[3]);
    if (alpha < (Real)0 || alpha > (Real)1 || beta < (Real)0 || beta > (Real)1) return false;
    t = tt;
    return true;
}

// fp32 pre-filter of aquad_t_c: false only when the exact test surely rejects or
// gives no t <= thi.
// `lo` (all pre-filters): a lower bound of the exact t the test can return.
// Fields: na = n[a], D, q1 = Q[ia], q2 = Q[ib], sw = +-w[a], sv = v[iv], su = u[iu] (RtPre order).
template <int CODE>
__device__ __forceinline__ bool aquad_maybe_v(float na, float D, float q1, float q2, float sw, float sv, float su,
                                              const float* o, const float* d, float dn, float thi, float& lo) {
    RT_FP32_FUSED
    constexpr int a = (CODE - 1) % 3, vflag = (CODE - 1) / 3;
    constexpr int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
    const float denom = na * d[a];
    lo = kTminLo;
    if (!(::fabsf(denom) > 1e-3f * dn)) return true;  // near-parallel: decide exactly
    const float no = na * o[a];
    const float idn = __builtin_amdgcn_rcpf(denom);
    const float t = (D - no) * idn;
    const float et = kRel * ((::fabsf(D) + ::fabsf(no)) * ::fabsf(idn) + 2.0f * ::fabsf(t)) + 1e-30f;
    if (t + et < kTminLo || t - et > thi) return false;
    lo = t - et;
    const float ph1 = o[ia] + t * d[ia] - q1;
    const float ph2 = o[ib] + t * d[ib] - q2;
    const float alpha = sw * (ph1 * sv);
    const float beta = sw * (ph2 * su);
    // in-plane hit-point error, times |w_a v| (alpha) / |w_a u| (beta)
    const float dp1 = et * ::fabsf(d[ia]) + kRel * (::fabsf(o[ia]) + ::fabsf(t * d[ia]) + ::fabsf(q1));
    const float dp2 = et * ::fabsf(d[ib]) + kRel * (::fabsf(o[ib]) + ::fabsf(t * d[ib]) + ::fabsf(q2));
    const float ea = ::fabsf(sw * sv) * dp1 + 1e-4f;
    const float eb = ::fabsf(sw * su) * dp2 + 1e-4f;
    return !(alpha < -ea || alpha > 1.0f + ea || beta < -eb || beta > 1.0f + eb);
}
template <int CODE>
__device__ __forceinline__ bool aquad_maybe_c(const RtPrim& p, const float* o, const float* d, float dn, float thi,
                                              float& lo) {
    constexpr int a = (CODE - 1) % 3, vflag = (CODE - 1) / 3;
    constexpr int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
    return aquad_maybe_v<CODE>(p.g3[a], p.g0[3], p.g0[ia], p.g0[ib], p.g3[3], p.g2[3], p.g1[3], o, d, dn, thi, lo);
}

template <class Real>
__device__ __forceinline__ bool aquad_t(const RtPrim& p, int code, V3 o, V3 d, Real tmin, Real tmax, Real& t) {
    switch (code) {
        case 1: return aquad_t_c<Real, 1>(p, o, d, tmin, tmax, t);
        case 2: return aquad_t_c<Real, 2>(p, o, d, tmin, tmax, t);
        case 3: return aquad_t_c<Real, 3>(p, o, d, tmin, tmax, t);
        case 4: return aquad_t_c<Real, 4>(p, o, d, tmin, tmax, t);
        case 5: return aquad_t_c<Real, 5>(p, o, d, tmin, tmax, t);
        default: return aquad_t_c<Real, 6>(p, o, d, tmin, tmax, t);
    }
}
__device__ __forceinline__ bool aquad_maybe(const RtPrim& p, int code, const float* o, const float* d, float dn,
                                            float thi, float& lo) {
    switch (code) {
        case 1: return aquad_maybe_c<1>(p, o, d, dn, thi, lo);
        case 2: return aquad_maybe_c<2>(p, o, d, dn, thi, lo);
        case 3: return aquad_maybe_c<3>(p, o, d, dn, thi, lo);
        case 4: return aquad_maybe_c<4>(p, o, d, dn, thi, lo);
        case 5: return aquad_maybe_c<5>(p, o, d, dn, thi, lo);
        default: return aquad_maybe_c<6>(p, o, d, dn, thi, lo);
    }
}

// aquad_t_c with the axis code as a runtime value (one code path for lanes
// testing different walls): the same operations on the same operands.
__device__ __forceinline__ float sel3(float x, float y, float z, int i) { return i == 0 ? x : (i == 1 ? y : z); }
constexpr uint32_t aquad_axes(int field) {  // 2-bit fields per code 1..6: a, ia, ib
    uint32_t m = 0;
    for (int c = 1; c <= 6; ++c) {
        const int a = (c - 1) % 3, vflag = (c - 1) / 3;
        const int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
        m |= (uint32_t)(field == 0 ? a : field == 1 ? ia : ib) << (2 * c);
    }
    return m;
}
template <class Real>
__device__ __forceinline__ bool aquad_t_rt(const RtPrim& p, int code, V3 o3, V3 d3, Real tmin, Real tmax, Real& t) {
    const int a = (int)((aquad_axes(0) >> (2 * code)) & 3u);
    const int ia = (int)((aquad_axes(1) >> (2 * code)) & 3u);
    const int ib = (int)((aquad_axes(2) >> (2 * code)) & 3u);
    const float oa = sel3(o3.x, o3.y, o3.z, a), da = sel3(d3.x, d3.y, d3.z, a);
    const float o1 = sel3(o3.x, o3.y, o3.z, ia), d1 = sel3(d3.x, d3.y, d3.z, ia);
    const float o2 = sel3(o3.x, o3.y, o3.z, ib), d2 = sel3(d3.x, d3.y, d3.z, ib);
    if (!(::isfinite(o1) && ::isfinite(d1) && ::isfinite(o2) && ::isfinite(d2))) return false;
    const Real na = (Real)sel3(p.g3[0], p.g3[1], p.g3[2], a);
    const Real denom = na * (Real)da;
    if (m_abs(denom) < (Real)1e-8) return false;
    const Real tt = (plane_d<Real>(p) - na * (Real)oa) / denom;
    if (!(tmin < tt && tt < tmax)) return false;
    const float ph1 = (o1 + (float)((Real)d1 * tt)) - sel3(p.g0[0], p.g0[1], p.g0[2], ia);
    const float ph2 = (o2 + (float)((Real)d2 * tt)) - sel3(p.g0[0], p.g0[1], p.g0[2], ib);
    const Real sw = (Real)p.g3[3];
    const Real alpha = sw * (Real)(ph1 * p.g2[3]);
    const Real beta = sw * (Real)(ph2 * p.g1[3]);
    if (alpha < (Real)0 || alpha > (Real)1 || beta < (Real)0 || beta > (Real)1) return false;
    t = tt;
    return true;
}
__device__ __forceinline__ int aquad_code(const RtPrim& p) { return __float_as_int(p.g4[3]); }

template <class Real, bool COUNT>
__device__ __forceinline__ bool prim_t(const RtPrim& p, const RayK<Real>& r, Real tmin, Real tmax, Real& t,
                                       uint32_t* cnt) {
    if (p.type == PRIM_SPHERE) {
        if (COUNT) cnt[CT_SPHERE]++;
        return sphere_t<Real>(p, r, tmin, tmax, t);
    }
    if (p.type == PRIM_QUAD) {
        if (COUNT) cnt[CT_QUAD]++;
        return planar_t<Real, true>(p, r, tmin, tmax, t);
    }
    if (COUNT) cnt[CT_PLANE]++;
    return planar_t<Real, false>(p, r, tmin, tmax, t);
}

// BVHNode.hit restated as an explicit DFS with the same visiting order: the
// box is tested when a node is entered with the closest-so-far interval, left
// subtree before right, leaf primitives in leaf order with a narrowing max.
// `stk` points at this lane's column of the LDS stack (stride kStackStride ints).
template <class Real, bool COUNT, class SK>
__device__ __forceinline__ int closest_hit(const DevScene& S, const RayK<Real>& r, Real& t_hit, SK* stk,
                                           uint32_t* cnt) {
    const Real tmin = K<Real>::TMIN;
    Real tmax = (Real)__builtin_inf();
    int hit = -1;
    int sp = 0;
    int node = 0;
    while (true) {
        const RtNode nd = S.nodes[node];
        if (COUNT) cnt[CT_NODE]++;
        bool descend = false;
        if (box_hit<Real>(nd, r, tmin, tmax)) {
            if (nd.b < 0) {
                const int end = nd.a - nd.b;
                for (int k = nd.a; k < end; ++k) {
                    Real t;
                    if (prim_t<Real, COUNT>(S.prims[k], r, tmin, tmax, t, cnt)) {
                        tmax = t;
                        hit = k;
                    }
                }
            } else {
                stk[sp * kStackStride] = (SK)nd.b;
                ++sp;
                node = nd.a;
                descend = true;
            }
        }
        if (!descend) {
            if (sp == 0) break;
            --sp;
            node = stk[sp * kStackStride];
        }
    }
    t_hit = tmax;
    return hit;
}

// ---------------------------------------------------------------------------
// Fast traversal with the SAME result.
//
// The reference tests primitive k with the closest-so-far interval and keeps
// it iff its first root t_k in (0.001, inf) satisfies t_k < tmax (strict), in
// DFS leaf order. So its answer is the lexicographic minimum of (t_k, leaf
// slot) over all primitives - independent of visiting order - provided no box
// containing a valid hit is culled. This traversal therefore
//   * culls with a strict fp32 slab test (the reference's per-axis test culls
//     far less) on boxes padded outward by ~1e-6 relative, accepting ties,
//   * visits the nearer child first and culls stacked nodes against the best t,
//   * rejects a primitive from an fp32 estimate only when it is clearly not a
//     candidate, and otherwise computes t_k with the reference's exact
//     arithmetic (Real) and compares (t, slot) lexicographically.
// The parity tests check it bit-for-bit against both the oracle and the
// reference-order traversal above.
// ---------------------------------------------------------------------------
struct FRay {
    float o[3];
    float d[3];
    float inv[3];  // 1/d with zero components replaced by +-1e-30 (no 0*inf NaNs)
    float noi[3];  // -(o * inv): the slab planes' t = fma(b, inv, noi)
    float eps;     // absolute t slack of the fused slab test (>= 2u max|o * inv|, see slab_t)
    float pthr;    // |d[a]| at or below which an axis quad counts as near-parallel (inf: every one)
    int nrow[3];   // byte offset in a 4-wide node of axis a's near-plane row (bmin[a], or bmax[a] when inv[a] < 0)
    float a;       // |d|^2
    float ia;      // ~1/|d|^2
    float on;      // |o| (rounded up)
    float dn;      // |d| (rounded up)
};

__device__ __forceinline__ FRay make_fray(V3 o, V3 d) {
    RT_FP32_FUSED
    FRay f;
    f.o[0] = o.x; f.o[1] = o.y; f.o[2] = o.z;
    f.d[0] = d.x; f.d[1] = d.y; f.d[2] = d.z;
    float m = 0.0f, mall = 0.0f;
    const float dmax = ::fmaxf(::fmaxf(::fabsf(d.x), ::fabsf(d.y)), ::fabsf(d.z));
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float c = f.d[a];
        const float cc = ::fabsf(c) < 1e-30f ? ::copysignf(1e-30f, c) : c;
        f.inv[a] = __builtin_amdgcn_rcpf(cc);  // <= 1 ulp: a common factor of an axis' two planes
        f.noi[a] = -(f.o[a] * f.inv[a]);
        const float an = ::fabsf(f.noi[a]);
        mall = ::fmaxf(mall, an);
        // near-parallel axes (|d_a| < 1e-3 max|d|) stay out of eps (an exact zero
        // component, inv = 1e30, made eps ~1e24 and every box accepted). Their planes need no
        // absolute slack: the fused error is u|o_a inv_a| + relative terms, and for a face b
        // either |o_a| <= 4 (1 + |b|), where the box's outward padding of 1e-6 (1 + |b|)
        // (scene.cpp make_fast_nodes) is >= 2u|o_a| in coordinates, so the padded face's computed
        // t stays outside the unpadded face's exact t; or |o_a| > 4 (1 + |b|), where
        // |t_a| = |b - o_a| |inv_a| >= 0.75 |o_a inv_a| and the error is relative, <= 2.7u |t_a|,
        // inside slab_accept's relative 2e-6 (~33u) with the rcp and fma roundings (~3u).
        m = ::fabsf(c) >= 1e-3f * dmax ? ::fmaxf(m, an) : m;
        f.nrow[a] = 16 * a + (f.inv[a] < 0.0f ? 48 : 0);
    }
    // 1e-6 * max|o * inv| ~ 16 u: covers the rounding of o * inv at both ends of the interval
    f.eps = m * 1e-6f;
    f.a = d.x * d.x + d.y * d.y + d.z * d.z;
    f.ia = __builtin_amdgcn_rcpf(f.a);
    f.dn = __builtin_amdgcn_sqrtf(f.a) * (1.0f + kRel);
    f.pthr = 1e-3f * f.dn;
    if (!(mall < 1e37f)) {  // o * inv overflowed (|o| > ~1e7 with an axis-parallel d): cull nothing
#pragma unroll
        for (int a = 0; a < 3; ++a) f.inv[a] = f.noi[a] = 0.0f;
        f.eps = __builtin_inff();
        f.pthr = __builtin_inff();  // and every axis quad is decided exactly
    }
    f.on = __builtin_amdgcn_sqrtf(o.x * o.x + o.y * o.y + o.z * o.z) * (1.0f + kRel);
    return f;
}

// The slab test's entry / exit parameter of the plane x_a = b: t = fma(b, inv, -o*inv), one
// FMA instead of (b - o) * inv. The unfused form's error is relative to |t|; the fused one's
// is absolute, |err| <= u (|o * inv| + |t|): the rounding of o * inv (FRay::noi) and the
// final one, u = 2^-24. The acceptance test tn <= tf * 1.000002 + eps covers it: the u|t|
// part is inside the relative 2e-6 (tn and tf are both positive whenever the box can hold a
// hit, t > 0.001), the u|o * inv| part of either end inside eps = 1e-6 max_a |o_a inv_a|
// (~16 u). On top of that every box is padded by 1e-6 (1 + |b|) (scene.cpp make_fast_nodes),
// the margin the unfused test already relied on for the exact hit point.
// A ray whose o * inv overflows gets inv = noi = 0, eps = inf: t = 0 on every plane (NaN
// on an infinite bound, which fminf / fmaxf ignore), tf = min(thi, 0) >= 0, and the test
// accepts every box - still the reference's hit, at brute-force cost (|o| > ~1e7 only).
__device__ __forceinline__ float slab_t(float b, const FRay& f, int a) { return __builtin_fmaf(b, f.inv[a], f.noi[a]); }
// Two-float vectors for packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: one instruction
// for both elements, the same IEEE operation on each); operand pairs in aligned register pairs,
// broadcast scalars by op_sel.
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pf2_of(float x) { return pf2{x, x}; }
__device__ __forceinline__ pf2 pf2_fma(pf2 a, pf2 b, pf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ pf2 pf2_abs(pf2 a) { return __builtin_elementwise_abs(a); }
__device__ __forceinline__ bool slab_accept(float tn, float tf, const FRay& f) {
    return tn <= __builtin_fmaf(tf, 1.000002f, f.eps);
}

template <class R>
__device__ __forceinline__ bool slab(const RtNode& n, const R& f, float thi, float& tnear) {
    if (n.bmin[0] != n.bmin[0]) return false;  // box the reference can never enter
    float tn = kTminLo, tf = thi;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t0 = slab_t(n.bmin[a], f, a);
        const float t1 = slab_t(n.bmax[a], f, a);
        tn = ::fmaxf(tn, ::fminf(t0, t1));
        tf = ::fminf(tf, ::fmaxf(t0, t1));
    }
    tnear = tn;
    return slab_accept(tn, tf, f);
}

// 4-wide node `ref` where the walk reads it: the blob (global, 128-byte nodes) or the LDS copy,
// where each node is followed by a 16-byte pad row (scene_prologue). A ds_read_b128 serves 16
// lanes per LDS cycle, 16 bytes each, from bank (address / 4) mod 64: with 128-byte nodes, row r
// of node i sits at bank 32 i + 4 r (mod 64), only two bank windows for the 16 lanes reading that
// row of their (different) nodes - up to 8-way conflicts (spheres-500: 40 % of the LDS-array
// cycles were bank conflicts, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE). At 144 bytes the
// window is 36 i + 4 r: 16 distinct windows for i mod 16.
// A launch that walks the tree from global memory (LDSS 0: spheres-100k's 2.8 MB of nodes) keeps
// the tree's top - the first n_top nodes in breadth-first order, the part every walk starts with -
// in LDS beside the stack (t4_step reads a node from there or from global memory: two loads in two
// branches, so each stays a ds_read / global_load - one generic pointer made them flat loads,
// 3.5 % slower on spheres-100k).
// (a 24-bit multiply, full rate: node indices stay below 2^24, scene.cpp make_t4nodes)
__device__ __forceinline__ const RtT4Node* t4_node(const DevScene& S, int ref) {
    return reinterpret_cast<const RtT4Node*>(reinterpret_cast<const char*>(S.tnodes) +
                                             (size_t)__umul24((unsigned)ref, (unsigned)S.t4_stride));
}
struct T4Rows {
    float4 nr[3], fr[3];  // per axis: the four children's near-plane / far-plane coordinates
    int4 rf;
};
// A node's rows through a pointer of address space AS (1 global, 3 LDS, 0 generic: whatever the
// compiler infers): typed loads of distinct address spaces in the two branches of t4_step cannot
// be merged into one flat load. The ray's direction signs pick which row of each axis is the near
// plane (FRay::nrow): the slab test then needs no min / max per plane pair (below).
template <int AS>
__device__ __forceinline__ void t4_rows(const void* nd0, const FRay& f, bool nf, T4Rows& R) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(AS))) v4* P4;
    typedef const __attribute__((address_space(AS))) char* PC;
    const PC b = (PC)__builtin_assume_aligned(nd0, 16);
    auto f4 = [](v4 v) { return make_float4(v.x, v.y, v.z, v.w); };
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int nrow = nf ? f.nrow[a] : 16 * a;
        R.nr[a] = f4(*(P4)(b + nrow));
        R.fr[a] = f4(*(P4)(b + (32 * a + 48 - nrow)));  // the other row of axis a
    }
    const v4 r = *(P4)(b + 96);
    R.rf = make_int4(__float_as_int(r.x), __float_as_int(r.y), __float_as_int(r.z), __float_as_int(r.w));
}

// One step of the 4-wide walk (RtT4Node) at node `nd`: the slab tests of its four children,
// the nearest hit child is returned as the next reference and the other hit children are
// pushed farthest first (so the nearer pop first); with no hit child the next reference is
// popped (kTravDone when the stack is empty). Branch-free:
//  * each child's key is its entry distance's bits (a positive float orders as its bits), or
//    ~0 for a miss / empty slot; (key, reference) pairs go through a 5-exchange network
//    (one compare, min / max of the keys, two selects of the references per exchange).
//    (Round 4 also tried keys carrying the child index in their low two bits, sorted alone
//    with min / max and the references re-read from the node afterwards: 4 dependent loads
//    per step - spheres-100k, whose tree is walked from global memory, lost 14 %.)
//  * with n hit children the pairs s1..s3 are written in the order s3, s2, s1 at stack
//    positions sp + max(n - 1 - j, 0), so s_{n-1} .. s1 land at sp .. sp + n - 2 and the
//    writes of missed children land at sp, overwritten or above the new top. No write
//    goes past sp + 2: at a node of level L (root 1) the stack holds at most 3 (L - 1)
//    entries (3 per ancestor), so writes stay below 3 t4depth <= stack_depth - 2 entries
//    (scene.cpp: stack_depth = max(..., 3 t4depth + 1) + 1).
// The pair sort and stack pushes of a 4-wide node step (below): keys k (entry-distance bits, ~0
// for a miss), child references r, n hit children.
template <int STRIDE, class SK>
__device__ __forceinline__ int t4_push(uint32_t (&k)[4], int (&r)[4], int n, SK* stk, int& sp) {
    auto cx = [&](int i, int j) {
        const bool sw = k[j] < k[i];
        const uint32_t lo = min(k[i], k[j]), hi = max(k[i], k[j]);
        const int ri = r[i], rj = r[j];
        k[i] = lo;
        k[j] = hi;
        r[i] = sw ? rj : ri;
        r[j] = sw ? ri : rj;
    };
    cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
    const int popped = stk[max(sp - 1, 0) * STRIDE];
#pragma unroll
    for (int j = 3; j >= 1; --j) stk[max(sp + n - 1 - j, sp) * STRIDE] = (SK)r[j];
    const int next = n > 0 ? r[0] : (sp > 0 ? popped : kT4Empty);  // (kT4Empty = kTravDone)
    sp = n > 0 ? sp + n - 1 : max(sp - 1, 0);
    return next;
}

template <int STRIDE, class SK>
__device__ __forceinline__ int t4_step(const DevScene& S, int ref, const FRay& f, float thi, SK* stk, int& sp) {
    T4Rows R;
    const bool nf = S.nearfar;
    if (ref < S.n_top) t4_rows<3>(S.top_lds + (size_t)ref * (sizeof(RtT4Node) + 16), f, nf, R);
    else if (S.n_top > 0) t4_rows<1>(t4_node(S, ref), f, nf, R);  // (LDSS 0: the rest is in global memory)
    else t4_rows<0>(t4_node(S, ref), f, nf, R);
    const float bn[3][4] = {{R.nr[0].x, R.nr[0].y, R.nr[0].z, R.nr[0].w}, {R.nr[1].x, R.nr[1].y, R.nr[1].z, R.nr[1].w},
                            {R.nr[2].x, R.nr[2].y, R.nr[2].z, R.nr[2].w}};
    const float bf[3][4] = {{R.fr[0].x, R.fr[0].y, R.fr[0].z, R.fr[0].w}, {R.fr[1].x, R.fr[1].y, R.fr[1].z, R.fr[1].w},
                            {R.fr[2].x, R.fr[2].y, R.fr[2].z, R.fr[2].w}};
    const int cr[4] = {R.rf.x, R.rf.y, R.rf.z, R.rf.w};
    uint32_t k[4];
    int r[4];
    int n = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        // near / far plane t per axis: the same two values min / max would pick (fma is monotone
        // in b for a fixed inv, so the sign of inv orders the planes; a NaN plane - an infinite
        // bound times inv = 0 - is ignored by fmaxf / fminf either way). (Round 6: the 24 plane
        // FMAs as 12 packed v_pk_fma_f32 ran 1.2-2.4 % slower on the BVH configs, profiles/r06/pairs/.)
        float tn = kTminLo, tf = thi;
        if (nf) {
            tn = ::fmaxf(::fmaxf(::fmaxf(slab_t(bn[0][c], f, 0), slab_t(bn[1][c], f, 1)), slab_t(bn[2][c], f, 2)), tn);
            tf = ::fminf(::fminf(::fminf(slab_t(bf[0][c], f, 0), slab_t(bf[1][c], f, 1)), slab_t(bf[2][c], f, 2)), tf);
        } else {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float t0 = slab_t(bn[a][c], f, a);
                const float t1 = slab_t(bf[a][c], f, a);
                tn = ::fmaxf(tn, ::fminf(t0, t1));
                tf = ::fminf(tf, ::fmaxf(t0, t1));
            }
        }
        const bool hit = (cr[c] != kT4Empty) & slab_accept(tn, tf, f);
        k[c] = hit ? __float_as_uint(tn) : ~0u;
        r[c] = cr[c];
        n += hit ? 1 : 0;
    }
    return t4_push<STRIDE>(k, r, n, stk, sp);
}

// fp32 pre-filters: false only when the exact test surely gives no t <= thi.
// The sphere roots' absolute error bound, kRel (|oc| |d| + |b| + sq) / a (+ a denormal floor),
// with |oc| |d| bounded without a square root (round 4: one v_sqrt fewer per test): a |oc|^2 =
// b^2 - disc + a r^2, and the exact disc >= -2 tol once the computed one passed -tol (its
// rounding is far below tol), so |oc| |d| <= |b| + |d| r + sqrt(2 tol) <= |b| + dn r + 1.5 sq
// (sq >= sqrt(tol)); the bound used, kRel (2 |b| + dn r + 3 sq) / a, is never smaller.
__device__ __forceinline__ float sphere_et(float b, float r, float sq, const FRay& f) {
    RT_FP32_FUSED
    return kRel * (2.0f * ::fabsf(b) + f.dn * r + 3.0f * sq) * f.ia + 1e-30f;
}
__device__ __forceinline__ bool sphere_maybe(float4 g, const FRay& f, float thi, float& lo) {
    RT_FP32_FUSED
    const float ox = f.o[0] - g.x, oy = f.o[1] - g.y, oz = f.o[2] - g.z;  // = the reference's oc
    const float b = ox * f.d[0] + oy * f.d[1] + oz * f.d[2];
    const float r = g.w;
    const float oo = ox * ox + oy * oy + oz * oz;
    const float disc = b * b - f.a * (oo - r * r);
    // every term of disc is bounded by a*(|oc|^2 + r^2) (b^2 <= a|oc|^2); the
    // bound holds through the cancellation of |oc|^2 - r^2 for rays leaving the surface
    const float tol = 4.0f * kRel * f.a * (oo + r * r) + 1e-30f;
    if (disc < -tol) return false;
    const float sq = __builtin_amdgcn_sqrtf(::fmaxf(disc, 0.0f) + tol) * (1.0f + kRel);
    const float et = sphere_et(b, r, sq, f);
    if ((-b + sq) * f.ia * (1.0f + kRel) + et < kTminLo) return false;
    const float r1 = (-b - sq) * f.ia;
    lo = r1 - ::fabsf(r1) * kRel - et;  // <= the first root; the second is larger
    if (lo > thi) return false;
    return true;
}

// sphere_maybe plus, when the sphere is SURELY hit at some t > 0.001 (the exact
// discriminant is positive and the larger root exceeds tMin under the same error
// model), an upper bound `hi` of the t the exact test will return (+inf otherwise).
// A surely-hit candidate's `hi` may cull the walk before its exact test runs.
__device__ __forceinline__ bool sphere_maybe_hi(float4 g, const FRay& f, float thi, float& lo, float& hi) {
    RT_FP32_FUSED
    const float ox = f.o[0] - g.x, oy = f.o[1] - g.y, oz = f.o[2] - g.z;
    const float b = ox * f.d[0] + oy * f.d[1] + oz * f.d[2];
    const float r = g.w;
    const float oo = ox * ox + oy * oy + oz * oz;
    const float disc = b * b - f.a * (oo - r * r);
    const float tol = 4.0f * kRel * f.a * (oo + r * r) + 1e-30f;
    if (disc < -tol) return false;
    const float sq = __builtin_amdgcn_sqrtf(::fmaxf(disc, 0.0f) + tol) * (1.0f + kRel);
    const float et = sphere_et(b, r, sq, f);
    const float hi2 = (-b + sq) * f.ia * (1.0f + kRel) + et;  // >= every root
    if (hi2 < kTminLo) return false;
    const float r1 = (-b - sq) * f.ia;
    lo = r1 - ::fabsf(r1) * kRel - et;  // <= the first root; the second is larger
    if (lo > thi) return false;
    hi = __builtin_inff();
    const float dm = disc - tol;  // <= the exact discriminant
    if (dm > 0.0f) {
        const float sql = __builtin_amdgcn_sqrtf(dm) * (1.0f - kRel);  // <= its square root
        const float r2 = (-b + sql) * f.ia;
        const float r2lo = r2 - ::fabsf(r2) * kRel - et;                // <= the larger root
        if (r2lo > 0.001f * (1.0f + 1e-5f)) hi = hi2 * (1.0f + 4e-6f) + 1e-30f;
    }
    return true;
}

template <bool QUAD>
__device__ __forceinline__ bool planar_maybe(const RtPrim& p, const FRay& f, float thi, float& lo) {
    RT_FP32_FUSED
    const float nx = p.g3[0], ny = p.g3[1], nz = p.g3[2];
    const float denom = nx * f.d[0] + ny * f.d[1] + nz * f.d[2];
    lo = kTminLo;
    if (!(::fabsf(denom) > 1e-3f * f.dn)) return true;  // near-parallel: decide exactly
    const float no = nx * f.o[0] + ny * f.o[1] + nz * f.o[2];
    const float D = p.g0[3];
    const float idn = __builtin_amdgcn_rcpf(denom);
    const float t = (D - no) * idn;
    // |n| = 1: num error <= kRel(|D| + |o|), denominator error <= kRel|d| (< 1% of |denom|)
    const float et = (kRel * (::fabsf(D) + f.on) + 2.0f * kRel * f.dn * ::fabsf(t)) * ::fabsf(idn) +
                     kRel * ::fabsf(t) + 1e-30f;
    if (t + et < kTminLo || t - et > thi) return false;
    lo = t - et;
    if (!QUAD) return true;
    const float px = f.o[0] + t * f.d[0] - p.g0[0];
    const float py = f.o[1] + t * f.d[1] - p.g0[1];
    const float pz = f.o[2] + t * f.d[2] - p.g0[2];
    const float ux = p.g1[0], uy = p.g1[1], uz = p.g1[2];
    const float vx = p.g2[0], vy = p.g2[1], vz = p.g2[2];
    const float wx = p.g4[0], wy = p.g4[1], wz = p.g4[2];
    // alpha = w . (ph x v), beta = w . (u x ph)
    const float alpha = wx * (py * vz - pz * vy) + wy * (pz * vx - px * vz) + wz * (px * vy - py * vx);
    const float beta = wx * (uy * pz - uz * py) + wy * (uz * px - ux * pz) + wz * (ux * py - uy * px);
    // hit-point error (t error, Ray.at's and ph's roundings) times |w||v| / |w||u| (scene.cpp)
    const float dp = et * f.dn + kRel * (f.on + ::fabsf(t) * f.dn + ::fabsf(p.g0[0]) + ::fabsf(p.g0[1]) +
                                         ::fabsf(p.g0[2]) + ::fabsf(px) + ::fabsf(py) + ::fabsf(pz));
    const float ea = p.g2[3] * dp + 1e-4f, eb = p.g1[3] * dp + 1e-4f;
    if (alpha < -ea || alpha > 1.0f + ea || beta < -eb || beta > 1.0f + eb) return false;
    return true;
}

// Exact candidate t (reference arithmetic) of primitive p on (0.001, inf).
__device__ __forceinline__ void count_exact(uint32_t* cnt) {
    cnt[CT_EXACT]++;
    const unsigned long long m = __ballot(1);
    if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) cnt[CT_EXACT_WAVE]++;
}

template <class Real, bool COUNT>
__device__ __forceinline__ bool prim_candidate(const RtPrim& p, const RayK<Real>& r, const FRay& f, float thi,
                                               Real& t, uint32_t* cnt) {
    const Real inf = (Real)__builtin_inf();
    float lo;
    if (p.type == PRIM_SPHERE) {
        if (COUNT) cnt[CT_SPHERE]++;
        if (!sphere_maybe(make_float4(p.g0[0], p.g0[1], p.g0[2], p.g0[3]), f, thi, lo)) return false;
        if (COUNT) count_exact(cnt);
        return sphere_t<Real>(p, r, K<Real>::TMIN, inf, t);
    }
    if (p.type == PRIM_QUAD) {
        if (COUNT) cnt[CT_QUAD]++;
        const int code = aquad_code(p);
        if (code != 0) {
            if (!aquad_maybe(p, code, f.o, f.d, f.dn, thi, lo)) return false;
            if (COUNT) count_exact(cnt);
            return aquad_t<Real>(p, code, r.o, r.d, K<Real>::TMIN, inf, t);
        }
        if (!planar_maybe<true>(p, f, thi, lo)) return false;
        if (COUNT) count_exact(cnt);
        return planar_t<Real, true>(p, r, K<Real>::TMIN, inf, t);
    }
    if (COUNT) cnt[CT_PLANE]++;
    if (!planar_maybe<false>(p, f, thi, lo)) return false;
    return planar_t<Real, false>(p, r, K<Real>::TMIN, inf, t);
}

template <class Real>
__device__ __forceinline__ float upper_f(Real t) {
    RT_FP32_FUSED
    // fp32 value >= t (rounded up with margin) used to cull against the best hit.
    const float x = (float)t;
    return x + ::fabsf(x) * 4e-6f + 1e-30f;
}

// `stk`: this lane's column of the LDS node stack.
// Walks the children-in-parent tree (RtTNode): one 64-byte node read tests
// both children; the nearer hit child is taken, the farther pushed (with its
// entry distance when kStackTnear, culled on pop against the best hit).
//
// Lanes of a wave reach leaves at different steps. Node steps and leaf tests run as two
// separate loops: a lane that reaches a leaf
// parks it and keeps walking nodes until every lane still walking holds a
// parked leaf, then the wave tests leaves together - otherwise nearly every
// node step would also pay for some lane's (four times longer) leaf test.
// Node steps taken while a leaf is parked cull with a possibly stale bound;
// that only costs extra node tests (the answer is the (t, slot) minimum).
constexpr int kTravDone = (int)0x80000000;  // no node / leaf (leaf refs are ~v, v < 2^31 - 1)

// Deferred exact sphere tests (DEFER, TRAV_FAST_DEFER kernels): a leaf's sphere that passes the
// fp32 pre-filter becomes this lane's PENDING candidate instead of being tested
// exactly on the spot - lanes reach leaves at different steps, so an in-loop
// fp64 test ran with a handful of active lanes (spheres-100k: 14 wave-level
// exact blocks per ray-trip for 1.0 tests per ray). A surely-hit candidate's
// upper bound culls the walk meanwhile; a second candidate resolves the first;
// the walk's end resolves the last, batched over the lanes finishing together.
// Exact t and the (t, slot) minimum are unchanged.
template <class Real, bool COUNT>
__device__ __forceinline__ void resolve_pending(const DevScene& S, const RayK<Real>& r, float& thi, Real& best_t,
                                                int& best, int& pk, uint32_t* cnt) {
    // (pk < 0: nothing pending)
    if (pk >= 0) {
        if (COUNT) count_exact(cnt);
        Real t;
        if (sphere_t<Real>(S.prims[pk], ray_at_use<Real>(r), K<Real>::TMIN, (Real)__builtin_inf(), t) &&
            (t < best_t || (t == best_t && pk < best))) {
            best_t = t;
            best = pk;
            thi = ::fminf(thi, upper_f<Real>(t));
        }
        pk = -1;
    }
}

// A leaf's primitives in leaf order: the fp32 pre-filter from the compact leaf-order record, then
// the exact test (or, with DEFER, the pending-candidate rule). L2 (trees walked from global memory):
// one 32-byte record per primitive (S.tsph2) that also carries the fp64 radius and the
// slot, so a sphere's exact test needs no dependent tprims -> RtPrim loads (two L2 round trips).
// (Round 5 also tried loading a leaf's four records before its first test, and loading a
// parked leaf's record when it is parked: spheres-100k 37.1 -> 44.8 and 30.0 -> 36.0 ms,
// profiles/r05/coop_v2_prefetch/, leaf_pre/ - dropped.)
template <class Real, bool COUNT, bool DEFER, bool L2 = false>
__device__ __forceinline__ void leaf_test(const DevScene& S, int ref, const RayK<Real>& r, const FRay& f, float& thi,
                                          Real& best_t, int& best, int& pk, float& plo, uint32_t* cnt) {
    const int v = ~ref;
    const int first = v >> 3;
    const int end = first + (v & 7);
    for (int m = first; m < end; ++m) {
        if constexpr (L2 && !DEFER) {
            const RtLeafSph q = S.tsph2[m];
            Real t;
            bool cand;
            if (q.r32 == q.r32) {  // sphere
                if (COUNT) cnt[CT_SPHERE]++;
                float lo;
                if (!sphere_maybe(make_float4(q.c[0], q.c[1], q.c[2], q.r32), f, thi, lo)) continue;
                if (COUNT) count_exact(cnt);
                cand = sphere_t_cr<Real>(v3(q.c[0], q.c[1], q.c[2]), sizeof(Real) == 8 ? (Real)q.r64 : (Real)q.r32,
                                         ray_at_use<Real>(r), K<Real>::TMIN, (Real)__builtin_inf(), t);
            } else {
                cand = prim_candidate<Real, COUNT>(S.prims[q.slot], ray_at_use<Real>(r), f, thi, t, cnt);
            }
            if (cand && (t < best_t || (t == best_t && q.slot < best))) {
                best_t = t;
                best = q.slot;
                thi = ::fminf(thi, upper_f<Real>(t));
            }
            continue;
        }
        const float4 g = S.tsph[m];
        Real t;
        int k;  // reference leaf slot (the tie-break key)
        bool cand;
        if (g.w == g.w) {  // sphere: pre-filter from the compact leaf-order record
            if (COUNT) cnt[CT_SPHERE]++;
            float lo;
            if constexpr (DEFER) {
            float hi;
            if (!sphere_maybe_hi(g, f, thi, lo, hi)) continue;
            k = S.tprims[m];
            // a second candidate: one surely hit before the pending one's lower bound
            // replaces it untested (t_new <= hi < plo <= t_pending); otherwise the
            // pending one is settled first
            if (pk >= 0 && !(hi < plo)) resolve_pending<Real, COUNT>(S, r, thi, best_t, best, pk, cnt);
            if (lo <= thi) {
                pk = k;
                plo = lo;
                thi = ::fminf(thi, hi);
            }
            continue;
            } else {
            if (!sphere_maybe(g, f, thi, lo)) continue;
            if (COUNT) count_exact(cnt);
            k = S.tprims[m];
            cand = sphere_t<Real>(S.prims[k], ray_at_use<Real>(r), K<Real>::TMIN, (Real)__builtin_inf(), t);
            }
        } else {
            k = S.tprims[m];
            cand = prim_candidate<Real, COUNT>(S.prims[k], ray_at_use<Real>(r), f, thi, t, cnt);
        }
        if (cand && (t < best_t || (t == best_t && k < best))) {
            best_t = t;
            best = k;
            thi = ::fminf(thi, upper_f<Real>(t));
        }
    }
}

template <class Real, bool COUNT, bool DEFER, class SK>
__device__ __forceinline__ int closest_hit_fast(const DevScene& S, const RayK<Real>& r, Real& t_hit, SK* stk,
                                                uint32_t* cnt) {
    const FRay f = make_fray(r.o, r.d);
    Real best_t = (Real)__builtin_inf();
    int best = -1;
    int pk = -1;  // pending (deferred) exact sphere test
    float plo = 0.0f;  // its lower bound
    float thi = __builtin_inff();
    float tn0;
    if (COUNT) cnt[CT_NODE]++;
    if (!slab(S.root_box, f, thi, tn0)) {
        t_hit = best_t;
        return -1;
    }
    int sp = 0;
    // next stacked entry (kTravDone when the stack is empty)
    auto pop = [&]() -> int {
        if (sp > 0) {
            --sp;
            return stk[sp * kStackStride];
        }
        return kTravDone;
    };
    // one 4-wide node step: the nearest hit child is next, the other hit
    // children are pushed farthest first (so the nearer pop first)
    auto node_step = [&](int ref) -> int {
        if (COUNT) cnt[CT_NODE] += 4;
        return t4_step<kStackStride>(S, ref, f, thi, stk, sp);
    };
    int ref = S.troot;
    int leaf = kTravDone;  // parked leaf
    while (ref != kTravDone || leaf != kTravDone) {
        while (ref >= 0) {
            ref = node_step(ref);
            if (ref < 0 && ref != kTravDone && leaf == kTravDone) {
                leaf = ref;
                ref = pop();
            }
            if (__ballot(leaf == kTravDone) == 0ull) break;  // every walking lane holds a leaf
        }
        if (leaf == kTravDone && ref != kTravDone) {  // the walk stopped on a leaf (or started on one)
            leaf = ref;
            ref = pop();
        }
        while (leaf != kTravDone) {
            leaf_test<Real, COUNT, DEFER>(S, leaf, r, f, thi, best_t, best, pk, plo, cnt);
            leaf = kTravDone;
            if (ref < 0 && ref != kTravDone) {  // the walk also stopped on a leaf
                leaf = ref;
                ref = pop();
            }
        }
    }
    resolve_pending<Real, COUNT>(S, r, thi, best_t, best, pk, cnt);  // the whole wave at once
    t_hit = best_t;
    return best;
}

// ---------------------------------------------------------------------------
// Resumable fast traversal (chunked kernel). closest_hit_fast keeps
// the whole wave in its loop until the lane with the longest walk is done - a
// ray grazing a field of spheres can need ten times the mean node visits, and
// every other lane idles meanwhile. Here a lane's walk state persists across
// the wave's loop iterations: the wave walks until `min_ready` of its lanes are
// done, they shade and start their next rays, and the long walks continue next
// to them. Same walk (culling, parked leaves, (t, slot) minimum) as
// closest_hit_fast, so the same hit.
// ---------------------------------------------------------------------------
template <class Real>
struct FastWalk {
    int ref, leaf, sp, best;
    int pk;     // pending (deferred) exact sphere test, resolved by fast_walk_resolve
    float plo;  // its lower bound
    float thi;
    Real best_t;
};

template <class Real, bool COUNT>
__device__ __forceinline__ void fast_walk_begin(const DevScene& S, V3 o, V3 d, FastWalk<Real>& W, uint32_t* cnt) {
    const FRay f = make_fray(o, d);
    W.best_t = (Real)__builtin_inf();
    W.best = -1;
    W.thi = __builtin_inff();
    W.sp = 0;
    W.pk = -1;
    W.leaf = kTravDone;
    float tn0;
    if (COUNT) cnt[CT_NODE]++;
    W.ref = slab(S.root_box, f, W.thi, tn0) ? S.troot : kTravDone;
}

// Called by the whole wave with uniform control flow; lanes with `walking`
// advance their walks. Returns when no lane walks, or (unless `drain`) after at
// least one round once `min_ready` lanes of the wave are not walking.
template <class Real, bool COUNT, bool DEFER, bool PROF = false, int STRIDE = kStackStride, bool L2 = false,
          class SK = int>
__device__ __forceinline__ void fast_walk_rounds(const DevScene& S, V3 o, V3 d, FastWalk<Real>& W, bool& walking,
                                                 SK* stk, int min_ready, bool drain, uint32_t* cnt, Prof* pf = nullptr) {
    const FRay f = make_fray(o, d);
    const RayK<Real> r = make_ray<Real>(o, d);
    int rounds = 0;
    while (true) {
        const unsigned long long wm = __ballot(walking);
        if (wm == 0ull) break;
        if (rounds > 0 && !drain && kWave - __popcll(wm) >= min_ready) break;
        ++rounds;
        if (walking) {
            int sp = W.sp;
            float thi = W.thi;
            auto pop = [&]() -> int {
                if (sp > 0) {
                    --sp;
                    return stk[sp * STRIDE];
                }
                return kTravDone;
            };
            auto node_step = [&](int ref) -> int {
                if (COUNT) cnt[CT_NODE] += 4;
                return t4_step<STRIDE>(S, ref, f, thi, stk, sp);
            };
            // one round of closest_hit_fast's parked-leaf walk
            int ref = W.ref, leaf = W.leaf;
            while (ref >= 0) {
                if (PROF) pcount<PROF>(*pf, PR_NODE);
                ref = node_step(ref);
                if (ref < 0 && ref != kTravDone && leaf == kTravDone) {
                    leaf = ref;
                    ref = pop();
                }
                if (__ballot(leaf == kTravDone) == 0ull) break;  // every walking lane holds a leaf
            }
            if (PROF) psec<PROF>(*pf, PR_WNODE);
            if (leaf == kTravDone && ref != kTravDone) {
                leaf = ref;
                ref = pop();
            }
            while (leaf != kTravDone) {
                if (PROF) pcount<PROF>(*pf, PR_LEAF);
                leaf_test<Real, COUNT, DEFER, L2>(S, leaf, r, f, thi, W.best_t, W.best, W.pk, W.plo, cnt);
                leaf = kTravDone;
                if (ref < 0 && ref != kTravDone) {
                    leaf = ref;
                    ref = pop();
                }
            }
            if (PROF) psec<PROF>(*pf, PR_WLEAF);
            W.ref = ref;
            W.leaf = leaf;
            W.sp = sp;
            W.thi = thi;
            if (ref == kTravDone && leaf == kTravDone) walking = false;
        }
    }
}

// The exact test of a finished walk's pending candidate (called by the lanes whose
// walks ended, together, before they shade).
template <class Real, bool COUNT>
__device__ __forceinline__ void fast_walk_resolve(const DevScene& S, V3 o, V3 d, FastWalk<Real>& W, uint32_t* cnt) {
    const RayK<Real> r = make_ray<Real>(o, d);
    resolve_pending<Real, COUNT>(S, r, W.thi, W.best_t, W.best, W.pk, cnt);
}

// Small scenes: test every primitive in leaf order. The answer is the same
// lexicographic minimum of (t, leaf slot) the fast traversal returns (valid
// under the same condition, SceneBuild::fast_ok). The loop bound and the
// primitive index are wave-uniform, so primitive records come through scalar
// loads and no lane waits on a BVH stack.
template <class Real, bool COUNT>
__device__ __forceinline__ int closest_hit_brute(const DevScene& S, int n_prims, const RayK<Real>& r, Real& t_hit,
                                                 uint32_t* cnt) {
    const FRay f = make_fray(r.o, r.d);
    Real best_t = (Real)__builtin_inf();
    int best = -1;
    float thi = __builtin_inff();
    for (int k = 0; k < n_prims; ++k) {
        Real t;
        const RtPrim p = ld_uniform(S.gprims, k);
        if (prim_candidate<Real, COUNT>(p, r, f, thi, t, cnt) && t < best_t) {
            best_t = t;
            best = k;
            thi = upper_f<Real>(t);
        }
    }
    t_hit = best_t;
    return best;
}

// Nearest-first brute force (up to kBruteMaxPrims primitives). The loop above runs primitive
// k's exact test whenever ANY lane of the wave needs it - lanes hit different
// walls, so a wave executes nearly every primitive's exact test per ray while
// each lane needs about one. Here pass 1 (wave-uniform, scalar primitive
// loads) only runs the fp32 pre-filters and keeps, per lane, the candidate set
// and each candidate's lower bound on t (in this lane's LDS column `lot`).
// Pass 2 exact-tests each lane's candidates nearest-first through one
// type-generic code path per primitive type, and stops once the nearest
// remaining lower bound lies beyond the best hit. Same (t, slot) minimum.
template <bool COUNT>
__device__ __forceinline__ bool prim_maybe(const RtPrim& p, const FRay& f, float& lo, uint32_t* cnt) {
    const float thi = __builtin_inff();
    if (p.type == PRIM_SPHERE) {
        if (COUNT) cnt[CT_SPHERE]++;
        return sphere_maybe(make_float4(p.g0[0], p.g0[1], p.g0[2], p.g0[3]), f, thi, lo);
    }
    if (p.type == PRIM_QUAD) {
        if (COUNT) cnt[CT_QUAD]++;
        const int code = aquad_code(p);
        if (code != 0) return aquad_maybe(p, code, f.o, f.d, f.dn, thi, lo);
        return planar_maybe<true>(p, f, thi, lo);
    }
    if (COUNT) cnt[CT_PLANE]++;
    return planar_maybe<false>(p, f, thi, lo);
}

// The reference's exact t of primitive p on (0.001, inf); per-lane p.
template <class Real>
__device__ __forceinline__ bool prim_exact(const RtPrim& p, const RayK<Real>& r, Real& t) {
    const Real inf = (Real)__builtin_inf();
    if (p.type == PRIM_SPHERE) return sphere_t<Real>(p, r, K<Real>::TMIN, inf, t);
    if (p.type == PRIM_QUAD) {
        const int code = aquad_code(p);
        if (code != 0) return aquad_t_rt<Real>(p, code, r.o, r.d, K<Real>::TMIN, inf, t);
        return planar_t<Real, true>(p, r, K<Real>::TMIN, inf, t);
    }
    return planar_t<Real, false>(p, r, K<Real>::TMIN, inf, t);
}

// The record's two 16-byte loads, issued together and waited for once: the empty asm takes the
// loaded words as its operands, so the loads cannot sink to their first uses (the compiler did
// that: kind, then s0, then the fields - dependent round trips again).
__device__ __forceinline__ RtExact xrec_load(const RtExact* px) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4* src = reinterpret_cast<const u4*>(px);
    u4 w0 = src[0], w1 = src[1];
    __asm__ volatile("" : "+v"(w0), "+v"(w1));
    struct W {
        u4 a, b;
    } w{w0, w1};
    return __builtin_bit_cast(RtExact, w);
}
// The nearest-first pass's exact test, from the primitive's RtExact record: prim_exact's
// operations on the same operands (the record holds the RtPrim fields aquad_t_c / sphere_t
// read), with the sphere's root and the axis-aligned quad's plane t through ONE division -
// lanes of a wave test different primitive types, and each type's block costs the whole wave;
// the prologues stay per type, the division (the longest piece of either) is shared: sphere_t's
// (-h - sqrt(disc)) / a and aquad_t_rt's (D - n.o) / (n.d). PRE_OTHER records take prim_exact
// on the RtPrim `p` (read only there).
template <class Real>
__device__ __forceinline__ bool prim_exact_rec(const RtExact& x, const RtPrim& p, const RayK<Real>& r, Real& t) {
    const Real inf = (Real)__builtin_inf();
    const int code = x.kind & 7;
    const bool sph = code == PRE_SPHERE;
    if (code == PRE_OTHER) return prim_exact<Real>(p, r, t);
    const Real s0 = (Real)x.s0;  // the JS double, or the fp32 mode's (float) s0 = RtPrim g0[3]
    Real num, den, halfB = (Real)0, sq = (Real)0;
    float o1 = 0.f, d1 = 0.f, o2 = 0.f, d2 = 0.f;
    if (sph) {
        const V3 c = V3{x.f[0], x.f[1], x.f[2]};
        const V3 oc = sub(r.o, c);
        halfB = dot<Real>(oc, r.d);
        const Real cc = len2<Real>(oc) - s0 * s0;
        const Real disc = halfB * halfB - r.a * cc;
        if (disc < (Real)0) return false;
        sq = m_sqrt(disc);
        num = -halfB - sq;
        den = r.a;
    } else {
        const int a = (int)((aquad_axes(0) >> (2 * code)) & 3u);
        const int ia = (int)((aquad_axes(1) >> (2 * code)) & 3u);
        const int ib = (int)((aquad_axes(2) >> (2 * code)) & 3u);
        const V3 o3 = r.o, d3 = r.d;
        const float oa = sel3(o3.x, o3.y, o3.z, a), da = sel3(d3.x, d3.y, d3.z, a);
        o1 = sel3(o3.x, o3.y, o3.z, ia);
        d1 = sel3(d3.x, d3.y, d3.z, ia);
        o2 = sel3(o3.x, o3.y, o3.z, ib);
        d2 = sel3(d3.x, d3.y, d3.z, ib);
        if (!(::isfinite(o1) && ::isfinite(d1) && ::isfinite(o2) && ::isfinite(d2))) return false;
        const Real na = (x.kind & kExactNegNa) ? (Real)-1 : (Real)1;  // n[a], exactly +-1
        den = na * (Real)da;
        if (m_abs(den) < (Real)1e-8) return false;
        num = s0 - na * (Real)oa;
    }
    Real q = num / den;
    if (sph) {
        if (!(K<Real>::TMIN < q && q < inf)) {
            q = (-halfB + sq) / r.a;
            if (!(K<Real>::TMIN < q && q < inf)) return false;
        }
    } else {
        if (!(K<Real>::TMIN < q && q < inf)) return false;
        const float ph1 = (o1 + (float)((Real)d1 * q)) - x.f[0];
        const float ph2 = (o2 + (float)((Real)d2 * q)) - x.f[1];
        const Real sw = (Real)x.f[2];
        const Real alpha = sw * (Real)(ph1 * x.f[3]);
        const Real beta = sw * (Real)(ph2 * x.f[4]);
        if (alpha < (Real)0 || alpha > (Real)1 || beta < (Real)0 || beta > (Real)1) return false;
    }
    t = q;
    return true;
}

// The brute-force pass's axis-quad pre-filter over an RtPre record {x_a, sv, su, -Q[ia] sv - 1/2,
// -Q[ib] su - 1/2, kRel qm} (qm = max(|Q[ia]|, |Q[ib]|)). The plane's t comes from the ray's slab
// constants, t = fma(x_a, inv[a], noi[a]), instead of a reciprocal of n.d per quad, and alpha - 1/2,
// beta - 1/2 are two FMAs each on host-folded products (round 4: 45 -> ~16 VALU per quad).
// Error of t, first order (u = 2^-24): inv = (1/d)(1 + e1), |e1| <= 2u (v_rcp_f32, 1 ulp);
// noi = -o inv (1 + e2) and x_a = x*(1 + e3), |e2|, |e3| <= u (x* = D / n_a, the exact test's
// plane); the fma rounds once more (e4). With t* = (x* - o) / d the exact test's t,
//   t - t* = t* e1 + inv (x* e3 - o e2) + t e4,  |t - t*| <= 2u |t*| + u (|x* inv| + |noi|) + u |t|
//                                                          <= 2u |noi| + 4u |t|   (|x* inv| <= |t| + |noi|)
// (the exact test's own double rounding is ~1e-16 relative). et = kEt (|t| + |noi|), kEt = 1e-6
// ~ 17u, covers each term 4x over. Round 2/3 used kRel = 1e-5 here: a ray leaving a wall at
// x_a = 555 has |noi| = 555 / |d_a|, so the wall it starts on stayed a candidate (lower bound
// < 0: tested FIRST) unless |d_a| > 5.5 - never - so it was tested first, and then the wall the
// ray does hit; at kEt the wall it leaves is rejected whenever |d_a| > ~0.56 (the exact test
// could only return a self-hit t = (x* - o) / d ~ 3e-5 / |d_a| > 0.001 below |d_a| ~ 0.03).
// The in-plane coordinate o + t d - Q is off by at most et |d| + a few u (|o| + |t d| + |Q|),
// which dp = (|t| + |noi|) c1 + c0 + kRel qm bounds (c1 = (kEt + kRel) dn, c0 = kRel on +
// 1e-30 dn: QuadPreRay; |o| <= on, |d| <= dn, |Q| <= qm), times |sv| (|su|) in alpha (beta).
// The window test alpha in [-ea, 1 + ea], ea = |sv| dp + 1e-4 (the absolute part covers alpha's
// own rounding near [0, 1], and the host's folding of the 1/2), is |alpha - 1/2| - |sv| dp <=
// 1/2 + 1e-4, one FMA with source modifiers, compared against kWin (1e-6 more for that FMA's own
// rounding); a NaN passes. Near-parallel rays (|d[a]| <= 1e-3 |d|, or a ray whose slab constants
// overflowed: pthr = inf) are decided by the exact test.
constexpr float kEt = 1e-6f;
constexpr float kWin = 0.5f + 1e-4f + 1e-6f;
struct QuadPreRay {
    float c1, c0;
};
__device__ __forceinline__ QuadPreRay quad_pre_ray(const FRay& f) {
    RT_FP32_FUSED
    return QuadPreRay{(kEt + kRel) * f.dn, kRel * f.on + 1e-30f * f.dn};
}
template <int CODE>
__device__ __forceinline__ bool aquad_maybe_pre(const float* v, const FRay& f, const QuadPreRay& qr, float& lo) {
    RT_FP32_FUSED
    constexpr int a = (CODE - 1) % 3, vflag = (CODE - 1) / 3;
    constexpr int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
    const float xa = v[0], sv = v[1], su = v[2], nq1 = v[3], nq2 = v[4], qk = v[5];
    lo = kTminLo;
    if (!(::fabsf(f.d[a]) > f.pthr)) return true;
    const float t = __builtin_fmaf(xa, f.inv[a], f.noi[a]);
    const float tn = ::fabsf(t) + ::fabsf(f.noi[a]);
    const float et = __builtin_fmaf(kEt, tn, 1e-30f);
    if (t + et < kTminLo) return false;
    lo = t - et;
    const float alpha = __builtin_fmaf(__builtin_fmaf(t, f.d[ia], f.o[ia]), sv, nq1);  // alpha - 1/2
    const float beta = __builtin_fmaf(__builtin_fmaf(t, f.d[ib], f.o[ib]), su, nq2);   // beta - 1/2
    const float dp = __builtin_fmaf(tn, qr.c1, qr.c0 + qk);
    const float wa = __builtin_fmaf(-::fabsf(sv), dp, ::fabsf(alpha));
    const float wb = __builtin_fmaf(-::fabsf(su), dp, ::fabsf(beta));
    return !(wa > kWin) && !(wb > kWin);
}

// Pre-filters of a PAIR of primitives in packed fp32 (RtPre PRE_SPHERE2 / PRE_QUAD2): the same
// operations as sphere_maybe / aquad_maybe_pre, element by element, on two-float vectors that
// the compiler issues as v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (one instruction for both
// primitives; the record's element pairs sit in aligned SGPR pairs, the ray's operands are
// broadcast with op_sel). Branch-free: both results are computed and masked. The margins are
// the single tests' (a filter may round differently as long as it stays conservative; the
// pair's window margin uses the larger qk of the two).

__device__ __forceinline__ void sphere_maybe2(const float* v, const FRay& f, bool& m0, bool& m1, float& lo0,
                                              float& lo1) {
    RT_FP32_FUSED
    const pf2 cx = {v[0], v[1]}, cy = {v[2], v[3]}, cz = {v[4], v[5]}, r = {v[6], v[7]}, rr = {v[8], v[9]};
    const pf2 ox = pf2_of(f.o[0]) - cx, oy = pf2_of(f.o[1]) - cy, oz = pf2_of(f.o[2]) - cz;
    const pf2 b = pf2_fma(oz, pf2_of(f.d[2]), pf2_fma(oy, pf2_of(f.d[1]), ox * pf2_of(f.d[0])));
    const pf2 oo = pf2_fma(oz, oz, pf2_fma(oy, oy, ox * ox));
    const pf2 disc = pf2_fma(b, b, -(pf2_of(f.a) * (oo - rr)));
    const pf2 tol = pf2_fma(pf2_of(4.0f * kRel * f.a), oo + rr, pf2_of(1e-30f));
    const pf2 dt = __builtin_elementwise_max(disc, pf2_of(0.0f)) + tol;
    const pf2 sq = pf2{__builtin_amdgcn_sqrtf(dt.x), __builtin_amdgcn_sqrtf(dt.y)} * pf2_of(1.0f + kRel);
    // sphere_et: kRel (2 |b| + dn r + 3 sq) ia + 1e-30
    const pf2 e0 = pf2_fma(pf2_of(3.0f), sq, pf2_fma(pf2_of(f.dn), r, pf2_of(2.0f) * pf2_abs(b)));
    const pf2 et = pf2_fma(e0, pf2_of(kRel * f.ia), pf2_of(1e-30f));
    const pf2 far = pf2_fma((sq - b) * pf2_of(f.ia), pf2_of(1.0f + kRel), et);
    const pf2 r1 = (-b - sq) * pf2_of(f.ia);
    const pf2 lo = pf2_fma(-pf2_abs(r1), pf2_of(kRel), r1) - et;
    m0 = !(disc.x < -tol.x) && !(far.x < kTminLo);
    m1 = !(disc.y < -tol.y) && !(far.y < kTminLo);
    lo0 = lo.x;
    lo1 = lo.y;
}

template <int CODE>
__device__ __forceinline__ void aquad_maybe_pre2(const float* v, const FRay& f, const QuadPreRay& qr, bool& m0,
                                                 bool& m1, float& lo0, float& lo1) {
    RT_FP32_FUSED
    constexpr int a = (CODE - 1) % 3, vflag = (CODE - 1) / 3;
    constexpr int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
    const pf2 xa = {v[0], v[1]}, sv = {v[2], v[3]}, su = {v[4], v[5]}, nq1 = {v[6], v[7]}, nq2 = {v[8], v[9]};
    const pf2 nsv = {v[10], v[11]}, nsu = {v[12], v[13]};
    const float qk = v[14];
    const pf2 t = pf2_fma(xa, pf2_of(f.inv[a]), pf2_of(f.noi[a]));
    const float an = ::fabsf(f.noi[a]);
    const pf2 tn = {::fabsf(t.x) + an, ::fabsf(t.y) + an};  // source modifiers, no masks
    const pf2 et = pf2_fma(pf2_of(kEt), tn, pf2_of(1e-30f));
    const pf2 te = t + et;
    const pf2 lo = t - et;
    const pf2 alpha = pf2_fma(pf2_fma(t, pf2_of(f.d[ia]), pf2_of(f.o[ia])), sv, nq1);  // alpha - 1/2
    const pf2 beta = pf2_fma(pf2_fma(t, pf2_of(f.d[ib]), pf2_of(f.o[ib])), su, nq2);   // beta - 1/2
    const pf2 dp = pf2_fma(tn, pf2_of(qr.c1), pf2_of(qr.c0 + qk));
    const pf2 wa = pf2_fma(nsv, dp, pf2_abs(alpha));
    const pf2 wb = pf2_fma(nsu, dp, pf2_abs(beta));
    const bool par = !(::fabsf(f.d[a]) > f.pthr);  // near-parallel: the exact test decides
    m0 = par || (!(te.x < kTminLo) && !(wa.x > kWin) && !(wb.x > kWin));
    m1 = par || (!(te.y < kTminLo) && !(wa.y > kWin) && !(wb.y > kWin));
    lo0 = par ? kTminLo : lo.x;
    lo1 = par ? kTminLo : lo.y;
}

// The brute-force pass's per-lane candidate bounds live in fp16 LDS columns (half the
// LDS of fp32: room for more pool slots). A stored bound must stay a lower bound: clamped
// at 0 (every hit has t > 0.001) and converted toward zero (v_cvt_pkrtz: round down for
// non-negative values; above 65504 it saturates to 65504, still below). A NaN bound stores
// 0, the smallest bound: such a candidate is tested before any other and never ends the
// nearest-first loop (0 <= every best t), so it is always tested.
__device__ __forceinline__ float lot_clamp(float lo) { return lo > 0.0f ? lo : 0.0f; }
__device__ __forceinline__ uint16_t lot_store(float lo) {
    const auto h = __builtin_amdgcn_cvt_pkrtz(lot_clamp(lo), 0.0f);
    return __builtin_bit_cast(uint16_t, h[0]);
}
__device__ __forceinline__ float lot_load(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
// This lane's fp16 column base (stk = the block's LDS base + threadIdx.x, as int*).
template <class SK>
__device__ __forceinline__ uint16_t* lot_column(SK* stk) {
    return reinterpret_cast<uint16_t*>(stk - threadIdx.x) + threadIdx.x;
}

struct NoHook {
    __device__ void operator()() const {}
};
// `after_prefilter`: called once the pre-filter pass is done (diagnostic section timer).
template <class Real, bool COUNT, class Hook = NoHook>
__device__ __forceinline__ int closest_hit_brute_nf(const DevScene& S, int n_prims, const RayK<Real>& r, Real& t_hit,
                                                    uint16_t* lot, uint32_t* cnt, Hook after_prefilter = Hook()) {
    (void)n_prims;  // the records (S.n_pre) cover the primitives; the mask holds their slots
    const FRay f = make_fray(r.o, r.d);
    const QuadPreRay qr = quad_pre_ray(f);
    uint32_t mask = 0u;
    for (int g = 0; g < S.n_pre; ++g) {
        // one scalar load (wave-uniform). (Round 4 tried issuing the next record's load an
        // iteration ahead: the two records' SGPRs pushed the pool kernel into SGPR spills,
        // Cornell path kernel 13.93 -> 14.65 ms; profiles/r04/ahead/.)
        const RtPre q = ld_uniform(S.gpre, g);
        const int kind = q.head & 0xff, k0 = (q.head >> 8) & 0xff, k1 = q.head >> 16;
        const float* v = q.f;
        if (kind >= PRE_SPHERE2) {  // a pair
            bool m0, m1;
            float lo0, lo1;
            if (kind == PRE_SPHERE2) {
                if (COUNT) cnt[CT_SPHERE] += 2;
                sphere_maybe2(v, f, m0, m1, lo0, lo1);
            } else {
                if (COUNT) cnt[CT_QUAD] += 2;
                switch (kind - PRE_QUAD2) {
                    case 1: aquad_maybe_pre2<1>(v, f, qr, m0, m1, lo0, lo1); break;
                    case 2: aquad_maybe_pre2<2>(v, f, qr, m0, m1, lo0, lo1); break;
                    case 3: aquad_maybe_pre2<3>(v, f, qr, m0, m1, lo0, lo1); break;
                    case 4: aquad_maybe_pre2<4>(v, f, qr, m0, m1, lo0, lo1); break;
                    case 5: aquad_maybe_pre2<5>(v, f, qr, m0, m1, lo0, lo1); break;
                    default: aquad_maybe_pre2<6>(v, f, qr, m0, m1, lo0, lo1); break;
                }
            }
            // both bounds in one conversion. (The halves are taken as integer bits: with h[1]
            // stored directly this compiler stored the LOW half for both.)
            const uint32_t hw = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(lot_clamp(lo0), lot_clamp(lo1)));
            if (m0) {
                lot[k0 * kStackStride] = (uint16_t)hw;
                mask |= 1u << k0;
            }
            if (m1) {
                lot[k1 * kStackStride] = (uint16_t)(hw >> 16);
                mask |= 1u << k1;
            }
            continue;
        }
        float lo;
        bool maybe;
        if (kind == PRE_SPHERE) {
            if (COUNT) cnt[CT_SPHERE]++;
            maybe = sphere_maybe(make_float4(v[0], v[1], v[2], v[3]), f, __builtin_inff(), lo);
        } else if (kind != PRE_OTHER) {
            if (COUNT) cnt[CT_QUAD]++;
            switch (kind) {
                case 1: maybe = aquad_maybe_pre<1>(v, f, qr, lo); break;
                case 2: maybe = aquad_maybe_pre<2>(v, f, qr, lo); break;
                case 3: maybe = aquad_maybe_pre<3>(v, f, qr, lo); break;
                case 4: maybe = aquad_maybe_pre<4>(v, f, qr, lo); break;
                case 5: maybe = aquad_maybe_pre<5>(v, f, qr, lo); break;
                default: maybe = aquad_maybe_pre<6>(v, f, qr, lo); break;
            }
        } else {
            maybe = prim_maybe<COUNT>(ld_uniform(S.gprims, k0), f, lo, cnt);
        }
        if (maybe) {
            lot[k0 * kStackStride] = lot_store(lo);
            mask |= 1u << k0;
        }
    }
    after_prefilter();
    Real best_t = (Real)__builtin_inf();
    int best = -1;
    float thi = __builtin_inff();
    int n_exact = 0;
    if (COUNT) {
        cnt[CT_CAND0] += mask == 0u ? 1u : 0u;
        cnt[CT_CAND2] += __popc(mask) >= 2 ? 1u : 0u;
    }
    while (mask != 0u) {
        // nearest remaining candidate (stored bounds are never NaN: lot_store)
        int kb = __builtin_ctz(mask);
        float lb = lot_load(lot[kb * kStackStride]);
        for (uint32_t m = mask & (mask - 1u); m != 0u; m &= m - 1u) {
            const int k = __builtin_ctz(m);
            const float l = lot_load(lot[k * kStackStride]);
            if (l < lb) {
                lb = l;
                kb = k;
            }
        }
        if (lb > thi) break;  // every remaining candidate's t exceeds the best hit
        mask &= ~(1u << kb);
        if (COUNT) {
            count_exact(cnt);
            if (++n_exact == 2) cnt[CT_EXACT2]++;
        }
        Real t;
        // ref precision: the ray as is, not ray_at_use - its fp64 conversions may then be
        // scheduled while the record loads are in flight (13.14 -> 13.11 ms,
        // profiles/r06/pairs/r06_rayhoist/). The fp32 build keeps ray_at_use: there |d|^2 may be
        // contracted (fma) differently where make_ray is inlined, and the pool and chunked kernels
        // must return the same hits (test_pool_kernel_equals_chunked_kernel caught 613 pixels).
        const bool hit = sizeof(Real) == 8
                             ? prim_exact_rec<Real>(xrec_load(S.xrec + kb), S.prims[kb], r, t)
                             : prim_exact_rec<Real>(xrec_load(S.xrec + kb), S.prims[kb], ray_at_use<Real>(r), t);
        if (hit && (t < best_t || (t == best_t && kb < best))) {
            best_t = t;
            best = kb;
            thi = upper_f<Real>(t);
        }
    }
    t_hit = best_t;
    return best;
}

// ONBasis (src/geometry/onbasis.ts:18-51)
struct Onb {
    V3 u, v, w;
};
template <class Real>
__device__ __forceinline__ Onb make_onb(V3 n) {
    Onb b;
    b.w = unit<Real>(n);
    const V3 a = m_abs((Real)b.w.x) > (Real)0.9 ? v3(0, 1, 0) : v3(1, 0, 0);
    b.v = unit<Real>(cross<Real>(b.w, a));
    b.u = cross<Real>(b.w, b.v);
    return b;
}
template <class Real>
__device__ __forceinline__ V3 onb_local(const Onb& b, V3 a) {
    return add(add(scale<Real>(b.u, (Real)a.x), scale<Real>(b.v, (Real)a.y)), scale<Real>(b.w, (Real)a.z));
}

// Vec3.randomInUnitSphere (src/geometry/vec3.ts:285-292): 3 draws per try.
template <class Real>
__device__ __forceinline__ V3 random_in_unit_sphere(uint64_t& rng) {
    while (true) {
        const Real x = (Real)-1 + (Real)2 * uniform<Real>(rng);
        const Real y = (Real)-1 + (Real)2 * uniform<Real>(rng);
        const Real z = (Real)-1 + (Real)2 * uniform<Real>(rng);
        const V3 p = mk<Real>(x, y, z);
        if (len2<Real>(p) < (Real)1) return p;
    }
}

// Dielectric.scatter direction (src/materials/dielectric.ts:44-98). Draws one
// random only when refraction is possible (short-circuit ||).
template <class Real>
__device__ __forceinline__ V3 dielectric_dir(Real ior, bool front, V3 din, V3 n, uint64_t& rng, bool& reflected) {
    const Real ratio = front ? ((Real)1 / ior) : ior;
    const V3 ud = unit<Real>(din);
    const Real cosT = js_min<Real>(dot<Real>(neg(ud), n), (Real)1);
    const Real sinT = m_sqrt((Real)1 - cosT * cosT);
    const bool cannot = ratio * sinT > (Real)1;
    bool refl = cannot;
    if (!refl) {
        Real r0 = ((Real)1 - ratio) / ((Real)1 + ratio);
        r0 = r0 * r0;
        const Real reflectance = r0 + ((Real)1 - r0) * pow5((Real)1 - cosT);
        refl = reflectance > uniform<Real>(rng);
    }
    reflected = refl;
    if (refl) return reflect<Real>(ud, n);
    // Vec3.refract (src/geometry/vec3.ts:193-209)
    const V3 perp = scale<Real>(add(ud, scale<Real>(n, cosT)), ratio);
    const V3 par = scale<Real>(n, -m_sqrt(m_abs((Real)1 - len2<Real>(perp))));
    return add(perp, par);
}

enum ScatterKind { SC_NONE = 0, SC_SPEC = 1, SC_PDF = 2 };

// Material.scatter over the flat material table; Mixed and Layered follow
// their children iteratively (mixedMaterial.ts:38-44, layeredMaterial.ts:36-53).
template <class Real>
__device__ __forceinline__ int scatter(const DevScene& S, int mi, V3 din, V3 n, bool front, uint64_t& rng, V3& att,
                                       V3& dir, int* pdf_mat = nullptr) {
    while (true) {
        const RtMat m = S.mats[mi];
        switch (m.type) {
            case MAT_LAMBERT:
                att = ld3(m.color);
                if (pdf_mat) *pdf_mat = mi;  // att is this material's albedo
                return SC_PDF;
            case MAT_METAL: {
                const V3 refl = reflect<Real>(unit<Real>(din), n);
                const Real fuzz = (Real)m.p0;
                V3 f = refl;
                if (fuzz > (Real)0) f = add(refl, scale<Real>(random_in_unit_sphere<Real>(rng), fuzz));
                if (dot<Real>(f, n) <= (Real)0) return SC_NONE;
                att = ld3(m.color);
                dir = f;
                return SC_SPEC;
            }
            case MAT_GLASS: {
                bool r;
                dir = dielectric_dir<Real>((Real)m.p0, front, din, n, rng, r);
                att = v3(1, 1, 1);
                return SC_SPEC;
            }
            case MAT_MIXED:
                mi = uniform<Real>(rng) < (Real)m.p0 ? m.c0 : m.c1;
                continue;
            case MAT_LAYERED: {
                bool r;
                const V3 d2 = dielectric_dir<Real>((Real)S.mats[m.c0].p0, front, din, n, rng, r);
                if (r) {
                    att = v3(1, 1, 1);
                    dir = d2;
                    return SC_SPEC;
                }
                din = d2;  // the refracted ray becomes rIn for the inner material
                mi = m.c1;
                continue;
            }
            default:  // MAT_LIGHT and DefaultMaterial: no scatter
                return SC_NONE;
        }
    }
}

// Quad.pdfValue / Sphere.pdfValue (quad.ts:123-140, sphere.ts:106-131):
// re-intersect the light on (0.001, inf), not occlusion-aware.
template <class Real, bool COUNT, bool UNIFORM = false>
__device__ __forceinline__ Real light_pdf_value(const DevScene& S, const RtLight& L, V3 origin, V3 dir,
                                                uint32_t* cnt) {
    const RtPrim p = UNIFORM ? ld_uniform(S.gprims, L.prim) : S.prims[L.prim];
    const RayK<Real> r = make_ray<Real>(origin, dir);
    Real t;
    if (L.type == PRIM_QUAD) {
        if (COUNT) cnt[CT_LIGHT_QUAD]++;
        const int code = aquad_code(p);
        const bool hit = code != 0 ? aquad_t<Real>(p, code, origin, dir, K<Real>::TMIN, (Real)__builtin_inf(), t)
                                   : planar_t<Real, true>(p, r, K<Real>::TMIN, (Real)__builtin_inf(), t);
        if (!hit) return (Real)0;
        const V3 hp = ray_at<Real>(origin, dir, t);
        const V3 n = ld3(p.g3);
        const bool front = dot<Real>(dir, n) <= (Real)0;
        const V3 hn = front ? n : neg(n);
        const Real d2 = len2<Real>(sub(hp, origin));
        const Real cosine = m_abs(dot<Real>(dir, hn));
        return d2 / ((Real)L.area * cosine);
    }
    if (COUNT) cnt[CT_LIGHT_SPHERE]++;
    if (!sphere_t<Real>(p, r, K<Real>::TMIN, (Real)__builtin_inf(), t)) return (Real)0;
    const Real rad = sphere_radius<Real>(p);
    const Real d2 = len2<Real>(sub(ld3(p.g0), origin));
    if (d2 <= rad * rad) return (Real)1 / ((Real)4 * K<Real>::PI);
    const Real cosT = m_sqrt((Real)1 - rad * rad / d2);
    const Real solid = (Real)2 * K<Real>::PI * ((Real)1 - cosT);
    return (Real)1 / solid;
}

// Quad.pdfRandomVec / Sphere.pdfRandomVec (quad.ts:148-158, sphere.ts:140-147)
template <class Real>
__device__ __forceinline__ V3 light_generate(const DevScene& S, const RtLight& L, V3 origin, uint64_t& rng) {
    const RtPrim p = S.prims[L.prim];
    if (L.type == PRIM_QUAD) {
        const Real alpha = uniform<Real>(rng);
        const Real beta = uniform<Real>(rng);
        const V3 rp = add(add(ld3(p.g0), scale<Real>(ld3(p.g1), alpha)), scale<Real>(ld3(p.g2), beta));
        return unit<Real>(sub(rp, origin));
    }
    const V3 oc = sub(ld3(p.g0), origin);
    const Real d2 = len2<Real>(oc);
    const Onb b = make_onb<Real>(oc);
    // Vec3.randomToSphere (src/geometry/vec3.ts:345-351)
    const Real rad = sphere_radius<Real>(p);
    const Real r1 = uniform<Real>(rng);
    const Real r2 = uniform<Real>(rng);
    const Real z = (Real)1 + r2 * (m_sqrt((Real)1 - rad * rad / d2) - (Real)1);
    const Real phi = (Real)2 * K<Real>::PI * r1;
    const Real s = m_sqrt((Real)1 - z * z);
    Real sn, cs;
    m_sincos(phi, sn, cs);
    return onb_local<Real>(b, mk<Real>(cs * s, sn * s, z));
}

// CosinePDF.value (src/geometry/pdf.ts:43-46)
// x / PI, correctly rounded: q = RN(x * RN(1/PI)) corrected once by the exact
// residual x - q*PI (fma) - Markstein's theorem for a correctly rounded reciprocal
// gives RN(x / PI) (also checked on 4e8 doubles in (0, 1], tools/probes/div_pi.c);
// 3 fp64 operations instead of the division sequence.
__device__ __forceinline__ double div_pi(double x) {
    constexpr double kPi = 3.141592653589793, kInvPi = 1.0 / 3.141592653589793;
    const double q = x * kInvPi;
    const double r = __builtin_fma(-q, kPi, x);
    return __builtin_fma(r, kInvPi, q);
}
__device__ __forceinline__ float div_pi(float x) { return x / K<float>::PI; }

template <class Real>
__device__ __forceinline__ Real cosine_value(const Onb& b, V3 dir) {
    const Real c = dot<Real>(unit<Real>(dir), b.w);
    return c <= (Real)0 ? (Real)0 : div_pi(c);
}

// writeColorToBuffer (src/camera.ts:455-472) into a Uint8ClampedArray.
__device__ __forceinline__ uint8_t to_u8(float c) {
    const double r = ::sqrt((double)c);
    const double v = ::floor(255.999 * r);
    if (!(v > 0.0)) return 0;
    if (v >= 255.0) return 255;
    return (uint8_t)v;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_min(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { unsigned long long x = __shfl_xor(v, o, 64); v = x < v ? x : v; }
    return v;
}
__device__ __forceinline__ unsigned long long wave_max(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { unsigned long long x = __shfl_xor(v, o, 64); v = x > v ? x : v; }
    return v;
}

// pixelConverged (src/camera.ts:348-368), in JS doubles. pixel_converged_at_batch is its test
// for an n already known to satisfy n % aBatch == 0 (pt_adapt_kernel counts down to those n
// for an integral aBatch instead of an fp64 fmod per sample).
__device__ __forceinline__ bool pixel_converged_at_batch(const RtCamera& c, int n, double sIll, double sIll2);
__device__ __forceinline__ bool pixel_converged(const RtCamera& c, int n, double sIll, double sIll2) {
    if (c.a_tolerance <= 0.0 || c.samples <= 1.0 || n < 2) return false;
    const double rem = ::fmod((double)n, c.a_batch);
    if (rem != 0.0) return false;  // also NaN
    return pixel_converged_at_batch(c, n, sIll, sIll2);
}
__device__ __forceinline__ bool pixel_converged_at_batch(const RtCamera& c, int n, double sIll, double sIll2) {
    if (c.a_tolerance <= 0.0 || c.samples <= 1.0 || n < 2) return false;
    const double mean = sIll / n;
    const double var = (sIll2 - (sIll * sIll) / n) / (n - 1);
    if (var <= 0.0 || var != var) return true;
    const double ci = 1.96 * ::sqrt(var) / ::sqrt((double)n);
    return ci <= c.a_tolerance * mean;
}

// The camera/options block as seen through an opaque kernarg pointer. Reading
// it this way inside the path loop stops the compiler from hoisting ~30 fp64
// conversions of loop-invariant camera fields into VGPRs for the whole kernel
// (the kernarg segment is constant memory: these are cheap scalar loads).
typedef const __attribute__((address_space(4))) char* KArgPtr;
__device__ __forceinline__ const RtCamera& cam_opaque() {
    KArgPtr p = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const RtCamera*)(p + offsetof(DevScene, cam));  // addrspacecast; inferred back to constant
}

template <class Real, bool COUNT, int TRAV, class SK>
__device__ __forceinline__ int closest_hit_any(const DevScene& S, int n_prims, const RayK<Real>& r, Real& t, SK* stk,
                                               uint32_t* cnt) {
    if (TRAV == TRAV_BRUTE) {
        if (n_prims <= kBruteMaxPrims)
            return closest_hit_brute_nf<Real, COUNT>(S, n_prims, r, t, lot_column(stk), cnt);
        return closest_hit_brute<Real, COUNT>(S, n_prims, r, t, cnt);
    }
    if (trav_fast(TRAV)) return closest_hit_fast<Real, COUNT, TRAV == TRAV_FAST_DEFER>(S, r, t, stk, cnt);
    return closest_hit<Real, COUNT>(S, r, t, stk, cnt);
}

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

// Diagnostic section timer (INSTR == 2), wave view: every psec() ends the
// wave's current section - whichever of its lanes execute it - and charges the
// wave-cycles since the previous psec() of ANY lane to it, together with the
// active lanes at that point. The wave's clock and sums live in one LDS slot per
// wave, updated by the first active lane, so time spent in code that only some
// lanes run is attributed once, to that code.
// Slot words: [0] last stamp, [1] start stamp, [2 + k] cycles of section k
// (k = PR_TRIPS: loop trips), [2 + PR_WORDS + k] active lanes, [2 + 2 PR_WORDS + k] executions.
constexpr int kProfSlot = 2 + 3 * PR_WORDS;
constexpr int kProfWaves = 16;  // >= waves per workgroup of either kernel
struct Prof {
    unsigned long long* w;  // this wave's LDS slot
};
template <bool PROF>
__device__ __forceinline__ void prof_init(Prof& pf, unsigned long long* lds, int lane) {
    if (PROF) {
        pf.w = lds + (threadIdx.x >> 6) * kProfSlot;
        if (lane == 0) {
            for (int k = 0; k < kProfSlot; ++k) pf.w[k] = 0ull;
            const unsigned long long n = __builtin_amdgcn_s_memtime();
            pf.w[0] = n;
            pf.w[1] = n;
        }
    }
}
template <bool PROF>
__device__ __forceinline__ void psec(Prof& pf, int k) {
    if (PROF) {
        const unsigned long long m = __ballot(1);
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) {
            const unsigned long long n = __builtin_amdgcn_s_memtime();
            pf.w[2 + k] += n - pf.w[0];
            pf.w[0] = n;
            pf.w[2 + PR_WORDS + k] += (unsigned long long)__popcll(m);
            pf.w[2 + 2 * PR_WORDS + k] += 1ull;
        }
    }
}
// Lane count of one execution of section k, without charging cycles (loop bodies too
// short for a timer: node steps, leaf tests).
template <bool PROF>
__device__ __forceinline__ void pcount(Prof& pf, int k) {
    if (PROF) {
        const unsigned long long m = __ballot(1);
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) {
            pf.w[2 + PR_WORDS + k] += (unsigned long long)__popcll(m);
            pf.w[2 + 2 * PR_WORDS + k] += 1ull;
        }
    }
}
template <bool PROF>
__device__ __forceinline__ void prof_trip(Prof& pf) {
    if (PROF) {
        const unsigned long long m = __ballot(1);
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) pf.w[2 + PR_TRIPS] += 1ull;
    }
}

// One path (one rayColor recursion) in flight on a lane.
template <bool EMIT>
struct Path {
    uint64_t rng;
    V3 o, d, T;
    int bounces;
    int em_n;
    V3 em[EMIT ? kEmitStack : 1];
};

// Camera.getRay (src/camera.ts:176-210) for sample `sample` of pixel (i, j).
// pixel00Loc + i*pixelDeltaU + j*pixelDeltaV (src/camera.ts:181), fixed per pixel.
// The scalings by the integers i, j (< 2^16) are fp32 multiplies: an fp32 times an
// integer below 2^24 is exact in double, so the double product rounded to fp32 is
// the fp32 product (rt_math.hpp identities) - the ref build's result, bit for bit.
template <class Real>
__device__ __forceinline__ V3 pixel_center(const RtCamera& C, int i, int j) {
    return add(add(ld3(C.pixel00), scale<float>(ld3(C.du), (float)i)), scale<float>(ld3(C.dv), (float)j));
}

template <class Real, bool EMIT>
__device__ __forceinline__ void path_begin(const RtCamera& C, Path<EMIT>& P, V3 pc, uint32_t pix, uint32_t sample) {
    P.rng = rng_init(C.seed_mix, pix, sample);
    const V3 du = ld3(C.du), dv = ld3(C.dv), cen = ld3(C.center);
    V3 ps = pc;
    if (C.samples > 1.0) {
        const Real px = (Real)-0.5 + uniform<Real>(P.rng);
        const Real py = (Real)-0.5 + uniform<Real>(P.rng);
        ps = add(add(pc, scale<Real>(du, px)), scale<Real>(dv, py));
    }
    P.o = cen;
    P.d = sub(ps, cen);
    if (C.aperture > 0.0) {
        V3 rd;
        while (true) {  // Vec3.randomInUnitDisk (vec3.ts:357-364)
            const Real a = (Real)2 * uniform<Real>(P.rng) - (Real)1;
            const Real b = (Real)2 * uniform<Real>(P.rng) - (Real)1;
            rd = mk<Real>(a, b, (Real)0);
            if (len2<Real>(rd) < (Real)1) break;
        }
        const V3 off = add(scale<Real>(ld3(C.ddu), (Real)rd.x), scale<Real>(ld3(C.ddv), (Real)rd.y));
        P.o = add(cen, off);
        P.d = sub(ps, P.o);
    }
    P.T = v3(1, 1, 1);
    P.bounces = 0;
    P.em_n = 0;
}

// One level of rayColor (src/camera.ts:221-319). Returns true when the path
// ends; `c` is then the sample's radiance (the recursion's emitted + ... right
// fold included).
// The emission right fold of a terminated path (EMIT builds).
template <bool EMIT>
__device__ __forceinline__ void fold_emission(const Path<EMIT>& P, V3& c) {
    if (EMIT) {
        for (int k = min(P.em_n, kEmitStack) - 1; k >= 0; --k) c = add(P.em[k], c);
    }
}

// First half of a rayColor level: the depth cut-off and Russian roulette
// (src/camera.ts:221-235). Returns true when the path ends here (`c` is then
// the sample's radiance), false when its ray must be traced next.
template <class Real, bool EMIT, bool PROF>
__device__ __forceinline__ bool path_pre(const RtCamera& C, Path<EMIT>& P, Prof& pf, V3& c) {
    bool term = false;
    c = v3(0, 0, 0);
    if (P.bounces >= C.depth) {
        term = true;
    } else if (C.roulette && P.bounces >= C.roulette_depth) {
        const Real mc = js_max<Real>(js_max<Real>((Real)P.T.x, (Real)P.T.y), (Real)P.T.z);
        const Real p = js_min<Real>(mc, (Real)0.95);
        if (uniform<Real>(P.rng) > p) term = true;
        else P.T = divs<Real>(P.T, p);
    }
    if (term) fold_emission<EMIT>(P, c);
    psec<PROF>(pf, PR_RR);
    return term;
}

// The stages of the second half of a rayColor level (src/camera.ts:236-319),
// shared by path_post and the stage-compacted pool kernel.

// Miss: the background gradient times the throughput (camera.ts:236-244).
template <class Real, bool EMIT, bool PROF>
__device__ __forceinline__ V3 miss_color(const RtCamera& C, const Path<EMIT>& P, unsigned long long& st_err,
                                         Prof& pf) {
    if (!C.has_background) st_err |= ERR_NO_BACKGROUND;
    const V3 ud = unit<Real>(P.d);
    const Real a = (Real)0.5 * ((Real)ud.y + (Real)1);
    const V3 c = mulv(add(scale<Real>(ld3(C.bg_top), (Real)1 - a), scale<Real>(ld3(C.bg_bottom), a)), P.T);
    psec<PROF>(pf, PR_MISS);
    return c;
}

// Hit record (sphere.ts:67-84, quad.ts:72-83, plane.ts:246-259) and the
// material's emission and scatter (camera.ts:246-262). Returns the scatter kind;
// `planar` = the primitive has a fixed normal (quad / plane: ONB table lookup).
template <class Real, bool EMIT, bool COUNT, bool PROF>
__device__ __forceinline__ int shade_hit(const DevScene& S, Path<EMIT>& P, int h, Real t, uint32_t* cnt, Prof& pf,
                                         V3& p, V3& nrm, bool& front, bool& planar, V3& emitted, V3& att, V3& sdir,
                                         int* pdf_mat = nullptr) {
    if (COUNT) cnt[CT_MATERIAL]++;
    const RtPrim pr = S.prims[h];
    p = ray_at<Real>(P.o, P.d, t);
    planar = pr.type != PRIM_SPHERE;
    if (!planar) {
        nrm = scale<Real>(sub(p, ld3(pr.g0)), sphere_inv_radius<Real>(pr));  // Vec3.divide(radius)
        front = dot<Real>(P.d, nrm) <= (Real)0;
        if (!front) nrm = neg(nrm);
    } else {
        const V3 pn = ld3(pr.g3);
        front = dot<Real>(P.d, pn) <= (Real)0;
        nrm = front ? pn : neg(pn);
    }
    const RtMat hm = S.mats[pr.mat];
    emitted = mulv(ld3(hm.emitted), P.T);
    psec<PROF>(pf, PR_HITREC);
    const int kind = scatter<Real>(S, pr.mat, P.d, nrm, front, P.rng, att, sdir, pdf_mat);
    psec<PROF>(pf, PR_SCATTER);
    return kind;
}

// A diffuse (PDF) scatter: MixturePDF([CosinePDF(n), light PDFs...], [0.5,
// 0.5/nL...]) generate + value and the throughput update (camera.ts:263-315).
// Returns true when the path ends here (mixture value <= 0.0001: the caller's
// sample radiance is the level's emission); else P continues from p.
// BR: 0 = the mixture's branch decided here; 1 / 2 = the caller knows it is the
// cosine / light branch (pool kernel: the draw was classified ahead) - the light
// branch then needs only the ONB's w (CosinePDF.value), not u and v.
template <class Real, bool EMIT, bool COUNT, bool PROF, int BR = 0>
__device__ __forceinline__ bool shade_diffuse(const DevScene& S, const RtCamera& C, Path<EMIT>& P, int h, bool planar,
                                              bool front, V3 p, V3 nrm, V3 att, uint32_t* cnt, Prof& pf) {
    if (COUNT) cnt[CT_DIFFUSE]++;
    Onb b;
    if (planar && h < S.n_onb) {
        const RtOnb& ob = S.onbs[(h * 2 + (sizeof(Real) == 4 ? 1 : 0)) * 2 + (front ? 0 : 1)];
        if (BR != 2) {
            b.u = ld3(ob.u);
            b.v = ld3(ob.v);
        }
        b.w = ld3(ob.w);
    } else if (BR == 2) {
        b.w = unit<Real>(nrm);  // make_onb's w
    } else {
        b = make_onb<Real>(nrm);
    }
    const Real total = (Real)S.mix_total;
    const bool total1 = S.mix_total == 1.0;  // x * 1 and x / 1 are exact: skip them (uniform branch)
    const Real lw = (Real)S.light_w;
    const Real u0 = uniform<Real>(P.rng);
    const Real rnd = total1 ? u0 : u0 * total;
    Real partial = (Real)0.5;
    V3 gdir;
    if (BR == 1 || (BR == 0 && (rnd < partial || C.n_lights == 0))) {
        const Real r1 = uniform<Real>(P.rng);
        const Real r2 = uniform<Real>(P.rng);
        const Real phi = (Real)2 * K<Real>::PI * r1;
        const Real sr2 = m_sqrt(r2);
        Real sn, cs;
        m_sincos(phi, sn, cs);
        gdir = onb_local<Real>(b, mk<Real>(cs * sr2, sn * sr2, m_sqrt((Real)1 - r2)));
    } else {
        int pick = C.n_lights - 1;
        for (int l = 0; l < C.n_lights; ++l) {
            partial += lw;
            if (rnd < partial) { pick = l; break; }
        }
        gdir = light_generate<Real>(S, S.lights[pick], p, P.rng);  // pick: per lane
    }
    psec<PROF>(pf, PR_SAMPLE);
    const Real cv = cosine_value<Real>(b, gdir);
    Real sum = (Real)0.5 * cv;
    for (int l = 0; l < C.n_lights; ++l)
        sum += lw * light_pdf_value<Real, COUNT, true>(S, ld_uniform(S.glights, l), p, gdir, cnt);
    const Real pv = total1 ? sum : sum / total;
    bool term = false;
    if (pv <= (Real)0.0001) {
        term = true;
    } else {
        const V3 brdf = scale<Real>(att, cv);
        P.T = divs<Real>(mulv(P.T, brdf), pv);
        P.o = p;
        P.d = gdir;
    }
    psec<PROF>(pf, PR_PDF);
    return term;
}

// Second half: given the closest hit (h, t) of the path's ray, the miss /
// emission / scatter / light sampling of the same level (src/camera.ts:236-319).
// Returns true when the path ends (`c` = the sample's radiance).
template <class Real, bool EMIT, bool COUNT, bool PROF>
__device__ __forceinline__ bool path_post(const DevScene& S, const RtCamera& C, Path<EMIT>& P, int h, Real t,
                                          uint32_t* cnt, unsigned long long& st_err, Prof& pf, V3& c) {
    bool term = false;
    c = v3(0, 0, 0);
    if (h < 0) {
        term = true;
        c = miss_color<Real, EMIT, PROF>(C, P, st_err, pf);
    } else {
        V3 p, nrm, emitted, att, sdir;
        bool front, planar;
        const int kind = shade_hit<Real, EMIT, COUNT, PROF>(S, P, h, t, cnt, pf, p, nrm, front, planar, emitted, att,
                                                            sdir);
        if (kind == SC_NONE) {
            term = true;
            c = emitted;
        } else {
            ++P.bounces;
            if (kind == SC_SPEC) {
                P.T = mulv(P.T, att);
                P.o = p;
                P.d = sdir;
            } else if (shade_diffuse<Real, EMIT, COUNT, PROF>(S, C, P, h, planar, front, p, nrm, att, cnt, pf)) {
                term = true;
                c = emitted;
            }
            if (EMIT && !term) {
                if (P.em_n < kEmitStack) P.em[P.em_n] = emitted;
                else st_err |= ERR_EMIT_STACK;
                ++P.em_n;
            }
        }
    }
    // emitted.add(rayColor(...)) at every level: a right fold.
    if (term) fold_emission<EMIT>(P, c);
    return term;
}

// One level of rayColor (src/camera.ts:221-319): path_pre, the closest hit,
// path_post. Returns true when the path ends; `c` is then the sample's radiance
// (the recursion's emitted + ... right fold included).
template <class Real, bool EMIT, bool COUNT, bool PROF, int TRAV, class SK>
__device__ __forceinline__ bool path_trip(const DevScene& S, const RtCamera& C, Path<EMIT>& P, SK* stk, uint32_t* cnt,
                                          unsigned long long& st_err, Prof& pf, V3& c) {
    if (path_pre<Real, EMIT, PROF>(C, P, pf, c)) return true;
    const RayK<Real> ray = make_ray<Real>(P.o, P.d);
    Real t;
    if (COUNT) cnt[CT_RAYS]++;
    const int h = closest_hit_any<Real, COUNT, TRAV>(S, C.n_prims, ray, t, stk, cnt);
    psec<PROF>(pf, PR_HIT);
    return path_post<Real, EMIT, COUNT, PROF>(S, C, P, h, t, cnt, st_err, pf, c);
}

// Per-pixel result: finalColor (src/camera.ts:326-340) + writeColorToBuffer
// (455-472) + RenderStats.addPixel (renderStats.ts:21-35).
struct PixStats {
    unsigned long long pixels = 0, samples = 0, smin = ~0ull, smax = 0, b = 0, bmin = ~0ull, bmax = 0;
};
// `opix`: the pixel's output index (full-frame j*W + i, or its tile-packed slot).
__device__ __forceinline__ void finish_pixel(const RtCamera& C, const RenderOut& out, uint32_t opix, V3 color, int n,
                                             unsigned long long bsum, int bmin, int bmax, PixStats& st) {
    V3 fin;
    if (C.mode == MODE_BOUNCES) {
        const double avg = n > 0 ? (double)bsum / (double)n : 0.0;
        fin = mk<double>(0.0, 0.0, js_min<double>(avg / (double)C.depth_raw, 1.0));
    } else if (C.mode == MODE_SAMPLES) {
        fin = mk<double>(js_min<double>((double)n / C.samples, 1.0), 0.0, 0.0);
    } else {
        fin = divs<double>(color, (double)n);
    }
    const size_t off = (size_t)opix * 3;
    if (out.radiance) {
        out.radiance[off] = fin.x;
        out.radiance[off + 1] = fin.y;
        out.radiance[off + 2] = fin.z;
    }
    if (out.rgb) {
        out.rgb[off] = to_u8(fin.x);
        out.rgb[off + 1] = to_u8(fin.y);
        out.rgb[off + 2] = to_u8(fin.z);
    }
    if (out.px_samples) out.px_samples[opix] = n;
    if (out.px_bounces) out.px_bounces[opix] = (int32_t)bsum;
    st.pixels += 1;
    st.samples += (unsigned long long)n;
    st.smin = min(st.smin, (unsigned long long)n);
    st.smax = max(st.smax, (unsigned long long)n);
    st.b += bsum;
    if (n > 0) st.bmin = min(st.bmin, (unsigned long long)bmin);
    st.bmax = max(st.bmax, (unsigned long long)bmax);
}

// RenderStats.merge (renderStats.ts:42-64): one atomic per word per wave.
__device__ __forceinline__ void stats_atomics(const RenderOut& out, unsigned long long sp, unsigned long long ss,
                                              unsigned long long smn, unsigned long long smx, unsigned long long sb,
                                              unsigned long long bmn, unsigned long long bmx, unsigned long long err) {
    unsigned long long* w = out.stats;
    if (sp > 0) {
        atomicAdd(&w[ST_PIXELS * kStatStride], sp);
        atomicAdd(&w[ST_SAMPLES * kStatStride], ss);
        atomicMin(&w[ST_SMIN * kStatStride], smn);
        atomicMax(&w[ST_SMAX * kStatStride], smx);
    }
    // bounce words also from the path kernels' lanes (12-byte records: LaneBounces, no pixels)
    if (sp > 0 || bmn != ~0ull) {
        atomicAdd(&w[ST_BOUNCES * kStatStride], sb);
        atomicMin(&w[ST_BMIN * kStatStride], bmn);
        atomicMax(&w[ST_BMAX * kStatStride], bmx);
    }
    if (err) atomicOr(&w[ST_ERROR * kStatStride], err);
}
__device__ __forceinline__ unsigned long long wave_or(unsigned long long v) {
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) v |= __shfl_xor(v, k, 64);
    return v;
}
__device__ __forceinline__ void publish_stats(const RenderOut& out, const PixStats& st, unsigned long long st_err,
                                              int lane) {
    const unsigned long long sp = wave_sum(st.pixels), ss = wave_sum(st.samples), sb = wave_sum(st.b);
    const unsigned long long smn = wave_min(st.smin), smx = wave_max(st.smax);
    const unsigned long long bmn = wave_min(st.bmin), bmx = wave_max(st.bmax);
    const unsigned long long err = wave_or(st_err);
    if (lane == 0) stats_atomics(out, sp, ss, smn, smx, sb, bmn, bmx, err);
}

template <bool COUNT, bool PROF>
__device__ __forceinline__ void publish_counters(const RenderOut& out, const uint32_t* cnt, Prof& pf, int lane) {
    if (COUNT) {
#pragma unroll
        for (int k = 0; k < CT_WORDS; ++k) {
            const unsigned long long v = wave_sum((unsigned long long)cnt[k]);
            if (lane == 0 && v) atomicAdd(&out.counters[k], v);
        }
    }
    if (PROF) {
        psec<PROF>(pf, PR_TILE);
        // lane 0 publishes the wave's totals from its LDS slot; PR_LOOP = the wave's lifetime
        if (lane == 0) {
            const unsigned long long life = __builtin_amdgcn_s_memtime() - pf.w[1];
            for (int k = 0; k < PR_WORDS; ++k)
                atomicAdd(&out.counters[CT_WORDS + k], k == PR_LOOP ? life : pf.w[2 + k]);
            for (int k = 0; k < PR_LOOP; ++k) {
                atomicAdd(&out.counters[CT_WORDS + PR_WORDS + k], pf.w[2 + PR_WORDS + k]);
                atomicAdd(&out.counters[CT_WORDS + PR_WORDS + PR_LOOP + k], pf.w[2 + 2 * PR_WORDS + k]);
            }
        }
    }
}

// The scene as the kernel sees it after scene_prologue: LDS-resident arrays at their
// LDS addresses (the prologue's copy of the blob prefix), the rest global.
template <int LDSS>
__device__ __forceinline__ DevScene scene_view(const DevScene& S0, int* lds_stack) {
    DevScene S = S0;
    // near / far rows (t4_step) where the tree is in LDS: spheres-500 +5.3 %, rain +2.8 %; in the
    // LDSS 0 kernels the three row offsets per ray pushed the chunk kernel from 48 to 88 bytes of
    // scratch spills and spheres-100k lost 2.3 % (profiles/r04/nearfar/). A constant per level, so
    // the unused form folds away.
    S.nearfar = LDSS > 0 ? 1 : 0;
    if (LDSS > 0) {
        S.tsph2 = nullptr;  // (fp64 leaf records: trees walked from global memory only)
    }
    if (LDSS == 0) S.top_lds = reinterpret_cast<const char*>(lds_stack) + S0.lds_stack_bytes;
    if (LDSS > 0) {
        S.n_top = 0;  // the whole tree is in LDS (a constant: the walk's reads stay ds_read)
        const char* b = reinterpret_cast<const char*>(lds_stack) + S0.lds_stack_bytes;
        S.tnodes = reinterpret_cast<const RtTNode*>(b);
        S.t4_stride = S0.lds_node_pad > 0 ? (int)sizeof(RtT4Node) + 16 : (int)sizeof(RtT4Node);
        b += (size_t)S0.lds_node_pad * 16;  // every section after the nodes moves by the pad rows
        S.tprims = reinterpret_cast<const int32_t*>(b + S0.off_tprims);
        S.tsph = reinterpret_cast<const float4*>(b + S0.off_tsph);
        S.prims = reinterpret_cast<const RtPrim*>(b + S0.off_prims);
        S.xrec = reinterpret_cast<const RtExact*>(b + S0.off_xrec);
        if (LDSS == 2) {
            S.mats = reinterpret_cast<const RtMat*>(b + S0.off_mats);
            S.lights = reinterpret_cast<const RtLight*>(b + S0.off_lights);
            S.onbs = reinterpret_cast<const RtOnb*>(b + S0.off_onbs);
        }
    }
    return S;
}

// Workgroup prologue shared by the render kernels: LDS-resident scene data
// (one cooperative copy per workgroup) and this thread's stack columns.
// LDSS 0: all scene reads from global memory; 1: the traversal data and the
// primitive records in LDS; 2: also the material and light tables. (Wave-uniform
// reads - the brute-force primitive loop, the light list - stay on scalar loads
// from the global copy.)
template <int LDSS>
__device__ __forceinline__ DevScene scene_prologue(const DevScene& S0, int* lds_stack) {
    if (LDSS == 0 && S0.n_top > 0) {  // the tree's top: n_top nodes of 8 rows, a pad row each
        uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds_stack) + S0.lds_stack_bytes);
        for (int w = threadIdx.x; w < S0.n_top * 8; w += blockDim.x) dst[w + (w >> 3)] = S0.blob[w];
        __syncthreads();
    }
    if (LDSS > 0) {
        uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds_stack) + S0.lds_stack_bytes);
        // the 4-wide nodes (8 rows each) take a pad row each (t4_node); the rest moves by those rows
        const int node_rows = S0.lds_node_pad * 8;
        for (int w = threadIdx.x; w < S0.lds_words; w += blockDim.x)
            dst[w < node_rows ? w + (w >> 3) : w + S0.lds_node_pad] = S0.blob[w];
        __syncthreads();
    }
    return scene_view<LDSS>(S0, lds_stack);
}

// ---------------------------------------------------------------------------
// Sequential-pixel kernel (adaptive sampling, and the reference-order
// traversal): a wave owns an 8x8 tile, lane = pixel, samples in order with
// per-pixel convergence checks (pixelConverged, src/camera.ts:348-368).
// Kernel arguments: S0 must stay the first parameter (cam_opaque reads it at kernarg offset 0).
// INSTR: 0 = product build, 1 = work counters, 2 = section timing.
// ---------------------------------------------------------------------------
template <class Real, bool EMIT, int INSTR, int TRAV, int LDSS>
__global__ __launch_bounds__(kBlock) void pt_render_kernel(DevScene S0, RtRegion reg, RenderOut out,
                                                                         int tiles_x, int my_tiles) {
    constexpr bool COUNT = INSTR == 1;
    constexpr bool PROF = INSTR == 2;
    extern __shared__ int lds_stack[];
    const RtCamera& C = S0.cam;
    const DevScene S = scene_prologue<LDSS>(S0, lds_stack);
    const int lane = threadIdx.x & (kWave - 1);
    StackT<LDSS>* stk = reinterpret_cast<StackT<LDSS>*>(lds_stack) + threadIdx.x;

    const int endX = min(reg.x + reg.width, C.width);
    const int endY = min(reg.y + reg.height, C.height);

    uint32_t cnt[CT_WORDS];
    if (COUNT) {
#pragma unroll
        for (int k = 0; k < CT_WORDS; ++k) cnt[k] = 0;
    }
    PixStats st;
    unsigned long long st_err = 0;
    __shared__ unsigned long long prof_lds[PROF ? kProfWaves * kProfSlot : 1];
    Prof pf;
    prof_init<PROF>(pf, prof_lds, lane);

    while (true) {
        unsigned int tile = 0;
        if (lane == 0) tile = atomicAdd(out.tile_counter, 1u);
        tile = __shfl(tile, 0, 64);
        if ((int)tile >= my_tiles) break;
        const int gt = reg.tile_group + (int)tile * reg.tile_groups;
        const int i = reg.x + (gt % tiles_x) * kTile + (lane & (kTile - 1));
        const int j = reg.y + (gt / tiles_x) * kTile + (lane / kTile);
        bool active = i < endX && j < endY && C.n_samples > 0;
        const bool valid_px = i < endX && j < endY;
        const uint32_t pix = (uint32_t)j * (uint32_t)C.width + (uint32_t)i;

        // PixelStats (src/render-utils/renderStats.ts:66-88)
        V3 color = v3(0, 0, 0);
        int n = 0;
        unsigned long long bsum = 0;
        int bmin = 0x7fffffff, bmax = 0;
        double sIll = 0.0, sIll2 = 0.0;

        bool new_path = true;
        Path<EMIT> P;
        psec<PROF>(pf, PR_TILE);
        while (active) {
            const RtCamera& C = cam_opaque();
            prof_trip<PROF>(pf);
            if (new_path) {
                path_begin<Real, EMIT>(C, P, pixel_center<Real>(C, i, j), pix, (uint32_t)n);
                new_path = false;
                psec<PROF>(pf, PR_NEWPATH);
            }
            V3 c;
            if (path_trip<Real, EMIT, COUNT, PROF, TRAV>(S, C, P, stk, cnt, st_err, pf, c)) {
                // PixelStats.add (renderStats.ts:76-88)
                color = add(color, c);
                ++n;
                bsum += (unsigned long long)P.bounces;
                bmin = min(bmin, P.bounces);
                bmax = max(bmax, P.bounces);
                if (C.adaptive) {
                    const double il = illuminance(c);
                    sIll += il;
                    sIll2 += il * il;
                }
                if (COUNT) {
                    cnt[CT_SAMPLES]++;
                    cnt[CT_BOUNCES] += (uint32_t)P.bounces;
                }
                if (n >= C.n_samples || pixel_converged(C, n, sIll, sIll2)) active = false;
                else new_path = true;
                psec<PROF>(pf, PR_ACC);
            }
        }
        if (valid_px) finish_pixel(C, out, out.packed ? tile * kWave + (uint32_t)lane : pix, color, n, bsum, bmin, bmax, st);
    }
    publish_stats(out, st, st_err, lane);
    publish_counters<COUNT, PROF>(out, cnt, pf, lane);
}

// ---------------------------------------------------------------------------
// Chunked kernel (fixed spp, no adaptive sampling): the work items are
// (pixel, chunk of kChunk consecutive samples). Every lane pulls its own items
// from its wave's pool, which refills 64 items (one tile-chunk) at a time from
// a global counter - so no lane idles while its wave finishes a tile, and the
// tail of the launch is one chunk long. Each finished sample's radiance (and
// bounce count) goes to the sample buffer; pt_accum_kernel then adds every
// pixel's samples in sample order in fp32, which is exactly PixelStats.add's
// sequence, so the image is bit-identical to the sequential kernel's.
// ---------------------------------------------------------------------------
// Guided schedule: phase p covers samples [s0[p], s0[p] + nch[p] * chunk[p]) in
// chunks of chunk[p]; items are numbered phase by phase (item_base[p]), and
// chunks halve from phase to phase, so the launch ends on 1-sample items.
constexpr int kMaxPhases = 8;
struct SampleBuf {
    float4* rec;    // record of (sample s, pixel slot) at s * stride_s + slot * stride_slot: {r, g, b, bounces (int bits)}
    int64_t stride_s, stride_slot;  // sample-major ([sample][slot]) or slot-major ([slot][sample])
    int32_t slots;  // pixel slots in this pass = pass_tiles * 64
    int32_t tile0;  // first of this pass's tiles (index among this launch's tiles)
    int32_t pool;   // items a wave takes from the global counter at a time (multiple of 64)
    int32_t n_phases;
    int32_t n_items;
    int32_t refill_min;  // idle lanes that trigger a hand-out (all-idle always does)
    int32_t min_ready;   // resumable fast traversal: lanes done walking before the wave shades
    // Adaptive-sampling rounds (pt_adapt_kernel): the pass's record slot a renders the launch
    // slot act[a] (tile * 64 + lane over the launch's tiles; tile0 is 0), samples s_base + s.
    // act == nullptr: slot a is pass tile tile0 + a / 64, lane a % 64, samples from 0.
    const int32_t* act;
    int32_t s_base;
    // Adaptive rounds: a sample's error flags (ERR_*) travel in bits 30-31 of its record's
    // bounce word instead of the launch's stats, so pt_adapt_kernel counts only the flags of
    // the samples it keeps - a round renders samples past a pixel's convergence, which the
    // reference never renders (src/camera.ts:400-425). Bounce counts stay below 2^30
    // (loop_threshold caps depth at 1e9).
    int32_t err_in_rec;
    // 12-byte records {r, g, b} (float triples at (float*)rec + 3 * index), the bounce statistics
    // reduced by the path kernel itself (LaneBounces): fixed spp in colour mode without the
    // per-pixel bounce output, where the accumulate pass needs only each pixel's colour sum in
    // sample order - RenderStats' bounce total / min / max are order-free integer reductions
    // (src/render-utils/renderStats.ts:21-35). A quarter less record traffic.
    int32_t rec12;
    int32_t s0[kMaxPhases], chunk[kMaxPhases], nch[kMaxPhases], item_base[kMaxPhases];
    double rnch[kMaxPhases];  // 1.0 / nch
};

// Adaptive sampling in rounds (pt_adapt_kernel): a pixel's running PixelStats
// between rounds (src/render-utils/renderStats.ts:66-88), by launch slot.
struct AdaptPix {
    float4 c;     // colour sum (fp32, sample order), n (int bits)
    double2 ill;  // sumIll, sumIll2
    int4 b;       // bounce sum (low 32 bits), min, max, bounce sum (high 32 bits)
};
struct AdaptRound {
    AdaptPix* state;        // launch slots (tile * 64 + lane)
    int32_t* next_act;      // the pixels still sampling after this round
    unsigned int* next_count;  // [0]: pixels carried; [1]: those likely to converge by `horizon`
    int32_t len;            // samples of this round
    int32_t horizon;        // sample count the round-length rule asks about (rt_api.cpp)
};

// One 16-byte sample record; NT: a non-temporal store. The pool kernel's records (read once,
// by the accumulate pass) go out non-temporally: Cornell writes 4.27 GB per launch instead of
// 4.78 GB for 2.62 GB of records (1.67x instead of 1.87x) at the same kernel time. The
// chunked kernel keeps plain stores: a lane writes its item's samples in turn, and spheres-500
// wrote 0.97 GB instead of 0.89 GB non-temporally (profiles/r02/recnt/).
// The finished sample's error flags for its record (SampleBuf::err_in_rec): the lane's flags
// since its previous sample (a lane runs one path at a time), which then start over; 0 and
// the flags stay in `st_err` for the launch's stats otherwise.
__device__ __forceinline__ int rec_err_bits(int err_in_rec, unsigned long long& st_err) {
    if (!err_in_rec) return 0;
    const int b = (int)((uint32_t)st_err << kRecErrShift);
    st_err = 0;
    return b;
}

template <bool NT>
__device__ __forceinline__ void rec_store(float4* p, float4 r);
// a 12-byte record (loads / stores of a 3-element vector move 12 bytes; its sizeof is 16, so
// records are addressed in floats)
typedef float RecF3 __attribute__((ext_vector_type(3), aligned(4)));
// A lane's bounce statistics over the samples it recorded (SampleBuf::rec12). The sum is 32-bit
// with a carry: a lane records ~10^4 samples per launch at the 8 GB record budget and depth goes
// up to 1e9, so a 32-bit sum can wrap; on a wrap the old sum goes to the launch's
// bounce total by one atomic (never in practice: 2^32 bounces in one lane's launch). (A 64-bit
// sum instead cost the pool kernel an extra spilled register reloaded in its trip loop: Cornell
// 13.91 -> 14.02 ms, profiles/r05/final/.)
struct LaneBounces {
    uint32_t sum = 0, mn = 0xffffffffu, mx = 0;
    __device__ void add(int b, unsigned long long* stats) {
        const uint32_t ns = sum + (uint32_t)b;
        if (ns < sum) {
            atomicAdd(stats + ST_BOUNCES * kStatStride, (unsigned long long)sum);
            sum = (uint32_t)b;
        } else {
            sum = ns;
        }
        mn = min(mn, (uint32_t)b);
        mx = max(mx, (uint32_t)b);
    }
    // into the launch's RenderStats (publish_stats): the accumulate pass adds none
    __device__ void to(PixStats& st) const {
        st.b = sum;
        st.bmin = mn == 0xffffffffu ? ~0ull : (unsigned long long)mn;
        st.bmax = mx;
    }
};
// The sample's record at index `idx` (s * stride_s + slot * stride_slot): {rgb, w} or, with
// rec12, {rgb} and w's bounce count into the lane's statistics.
template <bool NT>
__device__ __forceinline__ void rec_put(const SampleBuf& sb, size_t idx, V3 c, int w, LaneBounces& lb,
                                        unsigned long long* stats) {
    if (sb.rec12) {
        RecF3* p = reinterpret_cast<RecF3*>(reinterpret_cast<float*>(sb.rec) + 3 * idx);
        if constexpr (NT) __builtin_nontemporal_store(RecF3{c.x, c.y, c.z}, p);
        else *p = RecF3{c.x, c.y, c.z};
        lb.add(w, stats);
    } else {
        rec_store<NT>(sb.rec + idx, make_float4(c.x, c.y, c.z, __int_as_float(w)));
    }
}
template <bool NT>
__device__ __forceinline__ void rec_store(float4* p, float4 r) {
    if constexpr (NT) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(f4v{r.x, r.y, r.z, r.w}, reinterpret_cast<f4v*>(p));
    } else {
        *p = r;
    }
}

// n / d for 0 <= n < 2^31, d >= 1, through a double reciprocal (rinv = 1.0 / d)
// and one correction step: cheaper than the integer division sequence.
__device__ __forceinline__ int udiv(int n, int d, double rinv) {
    int q = (int)((double)n * rinv);
    const int r = n - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
}

__device__ __forceinline__ void item_pixel(const RtRegion& reg, int tiles_x, int mt, int l, int& i, int& j) {
    const int gt = reg.tile_group + mt * reg.tile_groups;
    const int ty = gt / tiles_x;
    i = reg.x + (gt - ty * tiles_x) * kTile + (l & (kTile - 1));
    j = reg.y + ty * kTile + (l / kTile);
}
__device__ __forceinline__ void item_pixel(const RtRegion& reg, int tiles_x, double rtx, int mt, int l, int& i,
                                           int& j) {
    const int gt = reg.tile_group + mt * reg.tile_groups;
    const int ty = udiv(gt, tiles_x, rtx);
    i = reg.x + (gt - ty * tiles_x) * kTile + (l & (kTile - 1));
    j = reg.y + ty * kTile + (l / kTile);
}
// Record slot a of the pass -> its pixel (i, j) (through the adaptive round's
// active list when there is one); false past the pass's slots or outside the region.
template <class SB>
__device__ __forceinline__ bool slot_pixel(const SB& sb, const RtRegion& reg, int tiles_x, double rtx, int endX,
                                           int endY, int a, int& i, int& j) {
    int ls = a;
    if (sb.act) {
        if (a >= sb.slots) return false;
        ls = sb.act[a];
        // Wait for this load here, on every path. Otherwise (fixed-spp launches never take this
        // branch) the wait-count pass kept its destination register pending on the paths around
        // the branch, and every later write of that register - a common temporary - waited with
        // vmcnt(0): for the sample records just stored, too.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt unchanged (gfx9 encoding)
    }
    item_pixel(reg, tiles_x, rtx, sb.tile0 + (ls >> 6), ls & 63, i, j);
    return i < endX && j < endY;
}

// The guided schedule's phase rows, copied to LDS at kernel start: an item's
// phase is per lane, and indexing the kernel-argument arrays by it costs a
// select chain per field (and SGPRs the path code then spills).
struct PhaseRow {
    int32_t s0, chunk, nch, base;
    double rnch;
    int32_t pad[2];
};
__device__ __forceinline__ void phase_table_init(const SampleBuf& sb, PhaseRow* tab) {
    const int t = threadIdx.x;
    if (t < kMaxPhases) {
        PhaseRow r;
        r.s0 = sb.s0[t];
        r.chunk = sb.chunk[t];
        r.nch = sb.nch[t];
        r.base = t < sb.n_phases ? sb.item_base[t] : 0x7fffffff;
        r.rnch = sb.rnch[t];
        r.pad[0] = r.pad[1] = 0;
        tab[t] = r;
    }
    __syncthreads();
}
// Item u of the launch -> (tile among this pass's tiles, lane-pixel l, sample range [s, s_end)).
__device__ __forceinline__ void item_decode(const SampleBuf& sb, const PhaseRow* tab, int u, int& tl, int& l, int& s,
                                            int& s_end) {
    int ph = 0;
    for (int q = 1; q < sb.n_phases; ++q) ph += u >= tab[q].base ? 1 : 0;
    const PhaseRow r = tab[ph];
    const int v = u - r.base;  // item within the phase: (tile, chunk) groups of 64
    const int q = v >> 6;
    l = v & 63;
    tl = udiv(q, r.nch, r.rnch);
    const int ch = q - tl * r.nch;
    s = r.s0 + ch * r.chunk;
    s_end = s + r.chunk;
}

// Item hand-out: every wave's first pool is static (wave w takes items
// [w * pool, (w + 1) * pool)), the global counter deals the rest from
// grid_waves * pool on - so the launch does not open with every wave's atomic
// on one word (4096 returning atomics serialise for ~50 us).
__device__ __forceinline__ void first_pool(const SampleBuf& sb, int& pool_next, int& pool_end, bool& exhausted) {
    const int gw = (int)(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
    pool_next = gw * sb.pool;
    pool_end = min(pool_next + sb.pool, sb.n_items);
    exhausted = pool_next >= sb.n_items;
}
// A wave's next item range [pool_next, pool_end) from the global counter (wave-uniform;
// exhausted when none is left). (A second counter dealing the launch's last items in
// smaller takes measured within noise of this, profiles/r03/tail/.)
__device__ __forceinline__ void take_pool(const RenderOut& out, const SampleBuf& sb, int lane, int& pool_next,
                                          int& pool_end, bool& exhausted) {
    int base = 0;
    if (lane == 0) base = (int)atomicAdd(out.tile_counter, (unsigned)sb.pool);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0, 64)) + (int)(gridDim.x * (blockDim.x / kWave)) * sb.pool;
    if (base >= sb.n_items) {
        exhausted = true;
        return;
    }
    pool_next = base;
    pool_end = min(base + sb.pool, sb.n_items);
}

// The chunked kernel's parameters as one block (the kernarg segment has this struct's layout).
// Its trip loop reads them through an opaque kernarg pointer at each use
// (scalar loads from the constant cache) instead of keeping them live across the loop, where
// the compiler ran out of SGPRs (106), spilled ~75 of them to VGPR lanes (v_writelane /
// v_readlane, VALU issue) and spilled VGPRs to scratch: SGPR spills 72-75 -> 34-40 in the
// fast-traversal builds; spheres-100k 2048^2 spp16 39.97 -> 38.55 ms, rain 11.65 -> 11.56 ms,
// spheres-500 unchanged (profiles/r03/exp5_ckopq/). The same change in the pool kernel (SGPR
// spills 97 -> 48) was within noise on Cornell ref and 1 % slower in fp32
// (profiles/r03/exp4_kopq/), so the pool kernel keeps its parameters in registers.
struct KernArgs {
    DevScene S0;
    RtRegion reg;
    RenderOut out;
    int tiles_x;
    SampleBuf sb;
};
__device__ __forceinline__ const KernArgs& kern_args() {
    KArgPtr p = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const KernArgs*)p;
}

template <class Real, bool EMIT, int INSTR, int TRAV, int LDSS>
__global__ __launch_bounds__(kBlockChunk) void pt_chunk_kernel(DevScene S0, RtRegion reg, RenderOut out,
                                                                        int tiles_x, SampleBuf sb) {
    constexpr bool COUNT = INSTR == 1;
    constexpr bool PROF = INSTR == 2;
    extern __shared__ int lds_stack[];
    const RtCamera& C0 = S0.cam;
    __shared__ PhaseRow ptab[kMaxPhases];
    phase_table_init(sb, ptab);
    const DevScene S = scene_prologue<LDSS>(S0, lds_stack);
    const int lane = threadIdx.x & (kWave - 1);
    StackT<LDSS>* stk = reinterpret_cast<StackT<LDSS>*>(lds_stack) + threadIdx.x;
    const int endX = min(reg.x + reg.width, C0.width);
    const int endY = min(reg.y + reg.height, C0.height);
    const int n_items = sb.n_items;

    uint32_t cnt[CT_WORDS];
    if (COUNT) {
#pragma unroll
        for (int k = 0; k < CT_WORDS; ++k) cnt[k] = 0;
    }
    unsigned long long st_err = 0;
    __shared__ unsigned long long prof_lds[PROF ? kProfWaves * kProfSlot : 1];
    Prof pf;
    prof_init<PROF>(pf, prof_lds, lane);

    int pool_next, pool_end;  // wave-uniform
    bool exhausted;           // wave-uniform
    first_pool(sb, pool_next, pool_end, exhausted);
    int slot = -1;                    // this lane's pixel slot (-1: idle)
    int s = 0, s_end = 0, i = 0, j = 0;
    uint32_t pix = 0;
    V3 pc = v3(0, 0, 0);  // the current item's pixel centre
    bool new_path = false;
    Path<EMIT> P;
    const double rtx = 1.0 / (double)tiles_x;
    // resumable fast traversal (product builds): per-lane walk state across iterations
    // (round 5 also parked diffuse hits until 32 / 48 lanes waited, then shaded them together:
    // 8-16 % slower - parked lanes are not walking; profiles/r05/defer_diffuse/)
    constexpr bool RS = trav_fast(TRAV) && INSTR != 1;  // (INSTR 2: timed sections)
    FastWalk<Real> W;
    bool walking = false;
    LaneBounces lb;  // SampleBuf::rec12

#define PK_SB (kern_args().sb)
#define PK_REG (kern_args().reg)
#define PK_OUT (kern_args().out)
#define PK_S (scene_view<LDSS>(kern_args().S0, lds_stack))
    while (true) {
        // hand out items to idle lanes (wave-uniform control flow); waits until
        // refill_min lanes are idle so the hand-out cost is shared
        const unsigned long long need = __ballot(slot < 0);
        const int n_need = __popcll(need);
        if (n_need != 0 && !exhausted && (n_need >= PK_SB.refill_min || __ballot(slot >= 0) == 0ull)) {
            if (pool_next >= pool_end) take_pool(PK_OUT, PK_SB, lane, pool_next, pool_end, exhausted);
            if (!exhausted) {
                const int take = min(n_need, pool_end - pool_next);
                const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                if (slot < 0 && rank < take) {
                    int tl, l, s1, e1;
                    item_decode(PK_SB, ptab, pool_next + rank, tl, l, s1, e1);
                    if (slot_pixel(PK_SB, PK_REG, tiles_x, rtx, endX, endY, tl * 64 + l, i, j)) {
                        slot = tl * 64 + l;
                        s = s1;
                        s_end = e1;
                        pix = (uint32_t)j * (uint32_t)C0.width + (uint32_t)i;
                        pc = pixel_center<Real>(cam_opaque(), i, j);
                        new_path = true;
                    }
                }
                pool_next += take;
            }
        }
        psec<PROF>(pf, PR_TILE);  // the item hand-out (wave-uniform)
        if (__ballot(slot >= 0) == 0ull) {
            if (exhausted) break;
            continue;
        }
        if constexpr (RS) {
            // the sample's radiance and bounce count to its record; next sample or idle
            auto finish_sample = [&](V3 c) {
                rec_put<false>(PK_SB, (size_t)s * PK_SB.stride_s + (size_t)slot * PK_SB.stride_slot, c,
                               P.bounces | rec_err_bits(PK_SB.err_in_rec, st_err), lb, PK_OUT.stats);
                ++s;
                if (s < s_end) new_path = true;
                else slot = -1;
            };
            const RtCamera& C = cam_opaque();
            prof_trip<PROF>(pf);
            // lanes between rays: start a path if needed, then the level's depth
            // cut-off / roulette, and the walk of its ray
            if (slot >= 0 && !walking) {
                if (new_path) {
                    path_begin<Real, EMIT>(C, P, pc, pix, (uint32_t)(PK_SB.s_base + s));
                    new_path = false;
                    psec<PROF>(pf, PR_NEWPATH);
                }
                V3 c;
                if (path_pre<Real, EMIT, PROF>(C, P, pf, c)) {
                    finish_sample(c);
                } else {
                    fast_walk_begin<Real, COUNT>(PK_S, P.o, P.d, W, cnt);
                    walking = true;
                }
            }
            psec<PROF>(pf, PR_RR);
            const bool was_walking = walking;
            fast_walk_rounds<Real, COUNT, TRAV == TRAV_FAST_DEFER, PROF, kStackStride, LDSS == 0>(
                PK_S, P.o, P.d, W, walking, stk, PK_SB.min_ready, exhausted, cnt, &pf);
            psec<PROF>(pf, PR_HIT);
            // walks that ended: the rest of the level (miss / emission / scatter / light sampling)
            if (was_walking && !walking) {
                fast_walk_resolve<Real, COUNT>(PK_S, P.o, P.d, W, cnt);
                V3 c;
                if (path_post<Real, EMIT, COUNT, PROF>(PK_S, C, P, W.best, W.best_t, cnt, st_err, pf, c))
                    finish_sample(c);
            }
            psec<PROF>(pf, PR_ACC);
        } else if (slot >= 0) {
            const RtCamera& C = cam_opaque();
            prof_trip<PROF>(pf);
            if (new_path) {
                path_begin<Real, EMIT>(C, P, pc, pix, (uint32_t)(PK_SB.s_base + s));
                new_path = false;
                psec<PROF>(pf, PR_NEWPATH);
            }
            V3 c;
            if (path_trip<Real, EMIT, COUNT, PROF, TRAV>(PK_S, C, P, stk, cnt, st_err, pf, c)) {
                rec_put<false>(PK_SB, (size_t)s * PK_SB.stride_s + (size_t)slot * PK_SB.stride_slot, c,
                               P.bounces | rec_err_bits(PK_SB.err_in_rec, st_err), lb, PK_OUT.stats);
                if (COUNT) {
                    cnt[CT_SAMPLES]++;
                    cnt[CT_BOUNCES] += (uint32_t)P.bounces;
                }
                ++s;
                if (s < s_end) new_path = true;
                else slot = -1;
                psec<PROF>(pf, PR_ACC);
            }
        }
    }
    PixStats st;
    lb.to(st);
    publish_stats(out, st, st_err, lane);
    publish_counters<COUNT, PROF>(out, cnt, pf, lane);
#undef PK_SB
#undef PK_REG
#undef PK_OUT
#undef PK_S
}

// ---------------------------------------------------------------------------
// Stage-compacted pool kernel (fixed spp, no emission stack): the chunked
// kernel's work items and per-sample records, but lanes are not tied to paths.
// Each wave keeps kPoolK path slots in LDS and two queues of slot indices:
//   A (trace): start the sample's path (getRay) or continue it, depth cut-off /
//     roulette, closest hit, miss or hit record + material scatter;
//   D (diffuse): the mixture-PDF light sampling, its value and the throughput
//     update (src/camera.ts:263-315), which about half of the hits need.
// Every trip runs ONE stage on up to 64 queued paths (ballot/mbcnt queue
// appends): D once 64 paths wait (or when it is the longer queue), A
// otherwise. So the diffuse shading runs on full waves rather than on the
// lanes whose path happens to need it in a given trip (the north star's
// persistent-wavefront work queues). D is split by the mixture's branch
// by branch: A draws the mixture uniform ahead (on a copy of the path's
// RNG state; D draws the same value again) and queues the path for the
// cosine-PDF or the light-PDF generate, so a D trip runs one of the two
// sampling branches instead of both at half the lanes. Each path's arithmetic
// and draw order are path_trip's, so every sample record - and the image - is
// bit-identical.
// ---------------------------------------------------------------------------
#ifndef RT_POOL_K
#define RT_POOL_K 152  // 56-byte slots + 2 queue bytes per wave, beside fp16 candidate columns
#endif
#ifndef RT_POOL_PROF
#define RT_POOL_PROF 0  // diagnostic variant: section timing (INSTR == 2 launches) in the pool kernel
#endif
constexpr int kPoolK = RT_POOL_K;          // path slots per wave
constexpr int kBlockPool = 1024;           // persistent workgroup size
constexpr int kPoolGroups = 3;             // 16-byte groups per slot, plus one 8-byte group (below)
static_assert(kPoolK >= kWave && kPoolK <= 256, "pool slots: one full wave, u8 queue entries");
// Per wave: slot state as [group][slot] float4, then the A queue (a ring) and the D queue
// (u8 slot indices; two stacks in one array each. D: cosine-branch paths from
// the bottom, light-branch paths from the top - together at most kPoolK entries).
// 56 bytes per slot (more slots per wave fill more trips: 64 / 80 / 96 slots ran Cornell in
// 21.7 / 17.7 / 16.1 ms, profiles/r02/poolsize/; 119 / 134 / 152 slots followed):
//   g0 {rng lo, rng hi, meta, hs}   meta = (phase + 2) | log2(item chunk) << 8 | lambert material << 11
//                                   (D only), phase: bounces so far (>= 0), PH_NEW or PH_ITEM;
//                                   hs = h | planar << 14 | front << 15 (D only) | s << 16
//   g1 {o (hit point p when queued for D), slot}
//   g2 {d (the face normal when queued for D), T.x}
//   g3 {T.y, T.z}                    (the 8-byte group)
// The item's end is the next multiple of its (power-of-two) chunk, the pixel comes from the
// slot (item_pixel), and the D stage reads the Lambertian albedo (the scatter's attenuation)
// from the material table. Host gates: spp <= 65535, depth <= 250, materials < 2^21,
// primitives < 2^14, power-of-two chunks.
constexpr size_t kPoolWaveBytes = ((size_t)kPoolK * (kPoolGroups * 16 + 8) + 2 * kPoolK + 15) / 16 * 16;
constexpr int kPoolClog2Bits = 3;  // log2(item chunk) field of the slot meta word
constexpr int kPoolMaxChunk = 1 << ((1 << kPoolClog2Bits) - 1);  // 128 samples
__device__ __forceinline__ float pool_meta(int phase, int clog2, int mat) {
    return __uint_as_float((uint32_t)((phase + 2) & 0xff) | ((uint32_t)clog2 << 8) | ((uint32_t)mat << 11));
}
__device__ __forceinline__ int meta_phase(float m) { return (int)(__float_as_uint(m) & 0xffu) - 2; }
__device__ __forceinline__ int meta_clog2(float m) { return (int)((__float_as_uint(m) >> 8) & 7u); }
__device__ __forceinline__ int meta_mat(float m) { return (int)(__float_as_uint(m) >> 11); }
__device__ __forceinline__ float pool_hs(int hf16, int s) { return __uint_as_float(((uint32_t)hf16 & 0xffffu) | ((uint32_t)s << 16)); }
__device__ __forceinline__ int hs_s(float v) { return (int)(__float_as_uint(v) >> 16); }
__device__ __forceinline__ int hs_hf(float v) { return (int)(__float_as_uint(v) & 0xffffu); }
__device__ __forceinline__ int item_end(int s, int clog2) { return ((s >> clog2) + 1) << clog2; }
constexpr size_t pool_lds_bytes() { return (size_t)(kBlockPool / kWave) * kPoolWaveBytes; }
enum : int { PH_NEW = -1, PH_ITEM = -2 };  // next sample's path to start / no work item

// Stacks in one array: the bottom one fills [0, cnt), the top one [kPoolK - cnt, kPoolK).
__device__ __forceinline__ void stack_push(uint8_t* q, bool top, int& cnt, bool want, int k) {
    const unsigned long long m = __ballot(want);
    if (want) {
        const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        q[top ? kPoolK - 1 - (cnt + r) : cnt + r] = (uint8_t)k;
    }
    cnt += __popcll(m);
}

template <class Real, int TRAV, int LDSS>
__global__ __launch_bounds__(kBlockPool) void pt_pool_kernel(DevScene S0, RtRegion reg, RenderOut out, int tiles_x,
                                                               SampleBuf sb) {
    extern __shared__ int lds_stack[];
    const RtCamera& C0 = S0.cam;
    __shared__ PhaseRow ptab[kMaxPhases];
    phase_table_init(sb, ptab);
    const DevScene S = scene_prologue<LDSS>(S0, lds_stack);
    const int lane = threadIdx.x & (kWave - 1);
    StackT<LDSS>* stk = reinterpret_cast<StackT<LDSS>*>(lds_stack) + threadIdx.x;
    char* wpool = reinterpret_cast<char*>(lds_stack) + S0.lds_pool_off + (size_t)(threadIdx.x / kWave) * kPoolWaveBytes;
    float4* G = reinterpret_cast<float4*>(wpool);  // group q of slot k: G[q * kPoolK + k]
    float2* G3 = reinterpret_cast<float2*>(wpool + (size_t)kPoolK * kPoolGroups * 16);  // the 8-byte group
    uint8_t* qa = reinterpret_cast<uint8_t*>(wpool + (size_t)kPoolK * (kPoolGroups * 16 + 8));
    uint8_t* qd = qa + kPoolK;
    const int endX = min(reg.x + reg.width, C0.width);
    const int endY = min(reg.y + reg.height, C0.height);
    const int n_items = sb.n_items;
    const double rtx = 1.0 / (double)tiles_x;
    uint32_t* cnt = nullptr;  // product build: no work counters
    unsigned long long st_err = 0;
    constexpr bool PP = RT_POOL_PROF;
    __shared__ unsigned long long prof_lds[PP ? kProfWaves * kProfSlot : 1];
    Prof pf;
    prof_init<PP>(pf, prof_lds, lane);

    for (int k = lane; k < kPoolK; k += kWave) {
        qa[k] = (uint8_t)k;
        G[k] = make_float4(0.f, 0.f, pool_meta(PH_ITEM, 0, 0), 0.f);
    }
    int a_cnt = kPoolK, d_cnt = 0;  // wave-uniform queue state
    int dl_cnt = 0;  // the D queue's light-branch stack (d_cnt: cosine-branch stack)
    // the A queue as two stacks in qa: paths to start from the bottom (an_cnt),
    // paths in flight from the top (ac_cnt); a_cnt stays their sum
    int an_cnt = kPoolK, ac_cnt = 0;
    int pool_next, pool_end;  // wave-uniform item hand-out
    bool exhausted;
    first_pool(sb, pool_next, pool_end, exhausted);

    // the sample's radiance and bounce count to its record; the slot's next phase
    // `err`: the sample's error flags (its miss without a background): in the record in
    // adaptive rounds (SampleBuf::err_in_rec), else in the launch's stats
    LaneBounces lb;  // SampleBuf::rec12
    auto record = [&](V3 c, int bounces, int slot, int& s, int s_end, unsigned long long err = 0ull) -> int {
        if (!sb.err_in_rec) st_err |= err;
        rec_put<true>(sb, (size_t)s * sb.stride_s + (size_t)slot * sb.stride_slot, c,
                           bounces | (sb.err_in_rec ? (int)((uint32_t)err << kRecErrShift) : 0), lb, out.stats);
        ++s;
        return s < s_end ? PH_NEW : PH_ITEM;
    };

    while (a_cnt + d_cnt + dl_cnt > 0) {
        // other lanes' slot and queue writes of the previous trip (one wave: LDS is in order)
        __asm__ volatile("" ::: "memory");
        prof_trip<PP>(pf);
        psec<PP>(pf, PR_ACC);  // the previous trip's records, slot stores and queue appends
        const bool dtop = dl_cnt > d_cnt;  // the longer D stack
        const int dn = dtop ? dl_cnt : d_cnt;
        const bool atop = ac_cnt > an_cnt;  // the longer A stack
        const int an = atop ? ac_cnt : an_cnt;
        if (dn >= kWave || dn > an) {
            // ---- D: diffuse shading of up to 64 queued paths ----
            const int n = min(kWave, dn);
            int k = -1, phase = 0;
            if (lane < n) k = (int)qd[dtop ? kPoolK - dl_cnt + lane : d_cnt - n + lane];
            if (dtop) dl_cnt -= n;
            else d_cnt -= n;
            if (k >= 0) {
                const float4 g0 = G[k], g1 = G[kPoolK + k], g2 = G[2 * kPoolK + k];
                const float2 g3 = G3[k];
                Path<false> P;
                P.rng = (uint64_t)__float_as_uint(g0.x) | ((uint64_t)__float_as_uint(g0.y) << 32);
                P.bounces = meta_phase(g0.z);
                P.em_n = 0;
                P.o = V3{g1.x, g1.y, g1.z};
                P.d = V3{g2.x, g2.y, g2.z};
                P.T = V3{g2.w, g3.x, g3.y};
                const int hf = hs_hf(g0.w);
                const int h = hf & 0x3fff;
                const bool planar = (hf >> 14) & 1, front = (hf >> 15) & 1;
                const V3 att = ld3(S.mats[meta_mat(g0.z)].color);  // the Lambertian scatter's attenuation
                const int clog2 = meta_clog2(g0.z), slot = __float_as_int(g1.w);
                int s = hs_s(g0.w);
                const int s_end = item_end(s, clog2);
                phase = P.bounces;
                const RtCamera& C = cam_opaque();
                const bool dterm =
                    dtop ? shade_diffuse<Real, false, false, PP, 2>(S, C, P, h, planar, front, P.o, P.d, att, cnt, pf)
                         : shade_diffuse<Real, false, false, PP, 1>(S, C, P, h, planar, front, P.o, P.d, att, cnt, pf);
                if (dterm) {
                    // mixture value cut-off: the level's emission (as computed at the hit: T is unchanged)
                    const V3 c = mulv(ld3(S.mats[S.prims[h].mat].emitted), P.T);
                    phase = record(c, P.bounces, slot, s, s_end);
                }
                G[k] = make_float4(__uint_as_float((uint32_t)P.rng), __uint_as_float((uint32_t)(P.rng >> 32)),
                                   pool_meta(phase, clog2, 0), pool_hs(0, s));
                G[2 * kPoolK + k] = make_float4(P.d.x, P.d.y, P.d.z, P.T.x);
                G3[k] = make_float2(P.T.y, P.T.z);
            }
            stack_push(qa, false, an_cnt, k >= 0 && phase < 0, k);
            stack_push(qa, true, ac_cnt, k >= 0 && phase >= 0, k);
            a_cnt = an_cnt + ac_cnt;
        } else {
            // ---- A: trace up to 64 queued paths ----
            const int n = min(kWave, an);
            int k = -1;
            if (lane < n) k = (int)qa[atop ? kPoolK - ac_cnt + lane : an_cnt - n + lane];
            if (atop) ac_cnt -= n;
            else an_cnt -= n;
            a_cnt -= n;
            float4 g0 = make_float4(0.f, 0.f, pool_meta(PH_ITEM, 0, 0), 0.f), g1 = g0, g2 = g0;
            float2 g3 = make_float2(0.f, 0.f);
            if (k >= 0) {
                g0 = G[k];
                g1 = G[kPoolK + k];
                g2 = G[2 * kPoolK + k];
                g3 = G3[k];
            }
            int phase = meta_phase(g0.z), clog2 = meta_clog2(g0.z), slot = __float_as_int(g1.w);
            int s = hs_s(g0.w);
            // work items for slots without one (the chunked kernel's guided hand-out)
            const unsigned long long need = __ballot(k >= 0 && phase == PH_ITEM);
            if (need != 0ull && !exhausted) {
                if (pool_next >= pool_end) take_pool(out, sb, lane, pool_next, pool_end, exhausted);
                if (!exhausted) {
                    const int take = min(__popcll(need), pool_end - pool_next);
                    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                    if (k >= 0 && phase == PH_ITEM && rank < take) {
                        int tl, l, s1, e1, i, j;
                        item_decode(sb, ptab, pool_next + rank, tl, l, s1, e1);
                        if (slot_pixel(sb, reg, tiles_x, rtx, endX, endY, tl * 64 + l, i, j)) {
                            slot = tl * 64 + l;
                            s = s1;
                            clog2 = __builtin_ctz((uint32_t)(e1 - s1));  // power-of-two, aligned chunks
                            phase = PH_NEW;
                        }
                    }
                    pool_next += take;
                }
            }
            const bool keep = k >= 0 && (phase != PH_ITEM || !exhausted);  // drained slots leave the pool
            bool to_d = false, d_light = false;
            if (k >= 0 && phase != PH_ITEM) {
                const RtCamera& C = cam_opaque();
                Path<false> P;
                if (phase == PH_NEW) {
                    int i, j;  // the slot's pixel (the hand-out's slot_pixel)
                    slot_pixel(sb, reg, tiles_x, rtx, endX, endY, slot, i, j);
                    path_begin<Real, false>(C, P, pixel_center<Real>(C, i, j),
                                            (uint32_t)j * (uint32_t)C.width + (uint32_t)i, (uint32_t)(sb.s_base + s));
                } else {
                    P.rng = (uint64_t)__float_as_uint(g0.x) | ((uint64_t)__float_as_uint(g0.y) << 32);
                    P.o = V3{g1.x, g1.y, g1.z};
                    P.d = V3{g2.x, g2.y, g2.z};
                    P.T = V3{g2.w, g3.x, g3.y};
                    P.bounces = phase;
                    P.em_n = 0;
                }
                V3 c;
                psec<PP>(pf, PR_NEWPATH);  // item hand-out and path starts
                bool term = path_pre<Real, false, PP>(C, P, pf, c);
                V3 att;
                int hf = 0, dmat = 0;
                unsigned long long err = 0ull;  // this sample's error flags (its miss)
                if (!term) {
                    const RayK<Real> ray = make_ray<Real>(P.o, P.d);
                    Real t;
                    int h;
                    if (PP && TRAV == TRAV_BRUTE && C.n_prims <= kBruteMaxPrims)  // section timer
                        h = closest_hit_brute_nf<Real, false>(S, C.n_prims, ray, t, lot_column(stk), cnt,
                                                              [&]() { psec<PP>(pf, PR_TILE); });
                    else
                        h = closest_hit_any<Real, false, TRAV>(S, C.n_prims, ray, t, stk, cnt);
                    psec<PP>(pf, PR_HIT);
                    if (h < 0) {
                        term = true;
                        c = miss_color<Real, false, PP>(C, P, err, pf);
                    } else {
                        V3 p, nrm, emitted, sdir;
                        bool front, planar;
                        const int kind = shade_hit<Real, false, false, PP>(S, P, h, t, cnt, pf, p, nrm, front,
                                                                              planar, emitted, att, sdir, &dmat);
                        if (kind == SC_NONE) {
                            term = true;
                            c = emitted;
                        } else {
                            ++P.bounces;
                            P.o = p;
                            if (kind == SC_SPEC) {
                                P.T = mulv(P.T, att);
                                P.d = sdir;
                            } else {
                                to_d = true;
                                P.d = nrm;  // queued for D: g2 carries the face normal
                                hf = h | (planar ? (1 << 14) : 0) | (front ? (1 << 15) : 0);
                                {  // shade_diffuse's first draw and branch, ahead
                                    uint64_t r = P.rng;
                                    const Real u0 = uniform<Real>(r);
                                    const Real rnd = S.mix_total == 1.0 ? u0 : u0 * (Real)S.mix_total;
                                    d_light = !(rnd < (Real)0.5 || C.n_lights == 0);
                                }
                            }
                        }
                    }
                }
                phase = term ? record(c, P.bounces, slot, s, item_end(s, clog2), err) : P.bounces;
                g0 = make_float4(__uint_as_float((uint32_t)P.rng), __uint_as_float((uint32_t)(P.rng >> 32)),
                                 pool_meta(phase, clog2, to_d ? dmat : 0), pool_hs(to_d ? hf : 0, s));
                g1 = make_float4(P.o.x, P.o.y, P.o.z, __int_as_float(slot));
                g2 = make_float4(P.d.x, P.d.y, P.d.z, P.T.x);
                g3 = make_float2(P.T.y, P.T.z);
            } else if (keep) {  // a slot still waiting for a work item
                g0 = make_float4(0.f, 0.f, pool_meta(PH_ITEM, 0, 0), 0.f);
            }
            if (keep) {
                G[k] = g0;
                G[kPoolK + k] = g1;
                G[2 * kPoolK + k] = g2;
                G3[k] = g3;
            }
            stack_push(qa, false, an_cnt, keep && !to_d && phase < 0, k);
            stack_push(qa, true, ac_cnt, keep && !to_d && phase >= 0, k);
            a_cnt = an_cnt + ac_cnt;
            stack_push(qd, false, d_cnt, to_d && !d_light, k);
            stack_push(qd, true, dl_cnt, to_d && d_light, k);
        }
    }
    PixStats st;
    lb.to(st);
    publish_stats(out, st, st_err, lane);
    publish_counters<false, PP>(out, cnt, pf, lane);
}


}  // namespace rt
