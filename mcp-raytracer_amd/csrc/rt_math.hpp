// JS-number / gl-matrix arithmetic model shared by the host scene builder and the
// device path tracer.
//
// The reference stores every Vec3 in a gl-matrix Float32Array
// (src/geometry/vec3.ts:3,19-25) while every scalar is a JS double. So a vector
// op is "compute in double, round each component to fp32 on store", and a
// scalar op is plain IEEE double. `Real` is the scalar type: `double` restates
// the reference exactly ("ref" precision), `float` is the fast fp32 mode where
// the round-to-fp32 steps become no-ops.
//
// Identities used to keep the ref mode cheap without changing a single bit:
//  * a+b, a-b, a*b of two fp32 values computed in double and rounded to fp32
//    equals the fp32 operation (double has > 2*24+2 bits), so vec+vec, vec-vec
//    and vec*vec (gl-matrix add/subtract/multiply) are done directly in fp32.
//  * products of two fp32 values are exact in double, so dot products only
//    round in the two additions, exactly like `a[0]*b[0] + a[1]*b[1] + a[2]*b[2]`,
//    and an fma whose product term is such a product rounds exactly as the
//    reference's separate multiply and add (dot, cross).
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rt {

using std::sqrt;

struct V3 {
    float x, y, z;
};

RT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }

// Vec3.create(x, y, z) with JS-number arguments: round each to fp32.
template <class Real>
RT_HD V3 mk(Real x, Real y, Real z) { return V3{(float)x, (float)y, (float)z}; }

// gl-matrix vec3.add / subtract / multiply (component-wise): exact as fp32 ops.
RT_HD V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD V3 mulv(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }

// Vec3.multiply(t) = vec3.scale(out, a, t): double product, fp32 store.
template <class Real>
RT_HD V3 scale(V3 a, Real t) {
    return V3{(float)((Real)a.x * t), (float)((Real)a.y * t), (float)((Real)a.z * t)};
}
// The correctly rounded restricted-domain forms below (rcp_rn / sqrt_rn) serve unit vectors and
// Vec3.divide (A/B at the round-4 build, profiles/r04/fp64/: spheres-500 path kernel 5.69 -> 5.62
// ms, rain 41.9 -> 41.2 ms, Cornell within 0.4 %).
#if defined(__HIPCC__)
// Correctly rounded double sqrt and reciprocal on a restricted domain, bit-identical there to the
// compiler's general expansions (gfx950), which are the same instruction sequences plus range
// scaling steps that are the identity on these inputs (round 4: 5 and 4 instructions fewer,
// 2 and 4 of them fp64):
//  * sqrt_rn: v_rsq_f64 then the Goldschmidt / Newton steps (h = y/2, r = 1/2 - h g, g += g r,
//    h += h r, two d = x - g^2, g += d h corrections) and the +-0 / +inf class select. The
//    general expansion first scales x < 2^-767 by 2^256 (and the root back by 2^-128): valid
//    for x >= 2^-767, 0, +inf (NaN and x < 0 give NaN either way).
//  * rcp_rn: the division sequence 1 / y with numerator 1 (div_scale leaves 2^-767 <= |y| <
//    2^1022 unscaled and sets no post-scale flag, the numerator's product 1 * r is exact,
//    div_fmas is then a plain fma and div_fixup the identity on the finite non-zero quotient):
//    v_rcp_f64, two Newton steps, one residual correction. Valid for 2^-767 <= |y| < 2^1022.
// tests/test_v8_math.py::test_device_sqrt_and_reciprocal_shortcuts_are_bit_exact checks both
// against ::sqrt and 1.0 / y on the device (rt_debug_fp64).
__device__ __forceinline__ double sqrt_rn(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return __builtin_amdgcn_class(x, 0x260) ? x : g;  // +-0, +inf
}
__device__ __forceinline__ double rcp_rn(double y) {
    const double r0 = __builtin_amdgcn_rcp(y);
    const double e0 = __builtin_fma(-y, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-y, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double e2 = __builtin_fma(-y, r2, 1.0);
    return __builtin_fma(e2, r2, r2);
}
// 2^-767 <= |y| < 2^1022: the biased exponent in [256, 2045) (one integer range test on the
// high word instead of two fp64 compares)
__device__ __forceinline__ bool rcp_rn_ok(double y) {
    const uint32_t hi = (uint32_t)(__builtin_bit_cast(uint64_t, y) >> 32);
    return ((hi >> 20) & 0x7ffu) - 256u < 1789u;
}
#endif
// RN(1 / t), the reference's division by a JS number
template <class Real>
RT_HD Real recip(Real t) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(Real) == 8)
        if (rcp_rn_ok(t)) return rcp_rn(t);
#endif
    return (Real)1 / t;
}
// RN(1 / RN(sqrt(l))) for l > 0 a sum of squares of fp32 values: l >= 2^-298 (sqrt_rn's domain),
// and below 2^300 its root is in rcp_rn's (else l is infinite, or NaN).
template <class Real>
RT_HD Real rsqrt_rn(Real l) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(Real) == 8)
        if (l < 0x1p300) return rcp_rn(sqrt_rn(l));
#endif
    return (Real)1 / sqrt(l);
}

// Vec3.divide(t) = vec3.scale(out, a, 1/t) (src/geometry/vec3.ts:126-130).
template <class Real>
RT_HD V3 divs(V3 a, Real t) { return scale<Real>(a, recip<Real>(t)); }

// Vec3.dot / lengthSquared (src/geometry/vec3.ts:132-136,152-157).
// In double each product of two fp32 values is exact, so fma(y1, y2, x1*x2) =
// RN(x1*x2 + y1*y2) is the reference's rounded sum, bit for bit (signed zeros
// and NaN/inf propagation included): 3 fp64 operations instead of 5.
template <class Real>
RT_HD Real dot(V3 a, V3 b) {
    if constexpr (sizeof(Real) == 8)
        return __builtin_fma((double)a.z, (double)b.z,
                             __builtin_fma((double)a.y, (double)b.y, (double)a.x * (double)b.x));
    else
        return (Real)a.x * (Real)b.x + (Real)a.y * (Real)b.y + (Real)a.z * (Real)b.z;
}
template <class Real>
RT_HD Real len2(V3 a) { return dot<Real>(a, a); }

// gl-matrix vec3.cross: each component formed in double, rounded to fp32.
// Each component x1*y2 - x2*y1 of exact double products = fma(x1, y2, -(x2*y1)).
template <class Real>
RT_HD Real xmul_sub(float x1, float y2, float x2, float y1) {
    if constexpr (sizeof(Real) == 8)
        return __builtin_fma((double)x1, (double)y2, -((double)x2 * (double)y1));
    else
        return (Real)x1 * (Real)y2 - (Real)x2 * (Real)y1;
}
template <class Real>
RT_HD V3 cross(V3 a, V3 b) {
    return V3{(float)xmul_sub<Real>(a.y, b.z, a.z, b.y), (float)xmul_sub<Real>(a.z, b.x, a.x, b.z),
              (float)xmul_sub<Real>(a.x, b.y, a.y, b.x)};
}

// gl-matrix 3.4.3 vec3.normalize: len = x²+y²+z²; if (len > 0) len = 1/sqrt(len).
template <class Real>
RT_HD V3 unit(V3 a) {
    Real l = dot<Real>(a, a);
    if (l > (Real)0) l = rsqrt_rn<Real>(l);
    return V3{(float)((Real)a.x * l), (float)((Real)a.y * l), (float)((Real)a.z * l)};
}

// Vec3.negate (src/geometry/vec3.ts:60-70): negation that normalises -0 to +0.
RT_HD V3 neg(V3 a) {
    V3 r{-a.x, -a.y, -a.z};
    if (r.x == 0.0f) r.x = 0.0f;
    if (r.y == 0.0f) r.y = 0.0f;
    if (r.z == 0.0f) r.z = 0.0f;
    return r;
}

// Vec3.reflect (src/geometry/vec3.ts:174-185): v - n*(2*(v·n)).
template <class Real>
RT_HD V3 reflect(V3 v, V3 n) {
    Real d = dot<Real>(v, n);
    return sub(v, scale<Real>(n, (Real)2 * d));
}

// JS Math.min / Math.max of two numbers: NaN-propagating, -0 < +0.
template <class Real>
RT_HD Real js_min(Real a, Real b) {
    if (a != a || b != b) return a + b;  // NaN
    if (a < b) return a;
    if (b < a) return b;
    return (a == (Real)0 && b == (Real)0) ? (__builtin_signbit(a) ? a : b) : a;
}
template <class Real>
RT_HD Real js_max(Real a, Real b) {
    if (a != a || b != b) return a + b;
    if (a > b) return a;
    if (b > a) return b;
    return (a == (Real)0 && b == (Real)0) ? (__builtin_signbit(a) ? b : a) : a;
}

// Ray.at(t) = origin.add(direction.multiply(t)) (src/geometry/ray.ts:25-28).
template <class Real>
RT_HD V3 ray_at(V3 o, V3 d, Real t) { return add(o, scale<Real>(d, t)); }

// splitmix64 finaliser (seeds the per-path PCG32 streams, pt_kernel.hpp rng_init).
RT_HD uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Color.illuminance (src/geometry/vec3.ts:239-242), always a JS double.
RT_HD double illuminance(V3 c) { return 0.299 * (double)c.x + 0.587 * (double)c.y + 0.114 * (double)c.z; }

}  // namespace rt
