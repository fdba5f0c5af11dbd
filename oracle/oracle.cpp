// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// A CPU restatement of df07/mcp-raytracer's per-pixel path (TypeScript, not
// runnable here: running the reference was refused in the survey session and
// that refusal binds this build). Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
// library, and only as the checker / CPU baseline.
//
// Structure deliberately mirrors the reference's object model (virtual hit /
// scatter / PDF objects, recursive BVHNode::hit, recursive rayColor), NOT the
// product's flattened GPU layout, so the two implementations are independent.
//
// Numerics ("ref" mode, Real = double): every Vec3 component is rounded to fp32
// on store (gl-matrix Float32Array, src/geometry/vec3.ts:3,19-25) and every
// scalar is an IEEE double (JS number). "fast" mode (Real = float) is the same
// algorithm with fp32 scalars, used to cross-check the GPU's fp32 kernel.
//
// Randomness: the reference draws unseeded Math.random() (call sites listed in
// SURVEY.md header). This restatement replaces it with the build's seeded
// counter RNG (PCG32 stream keyed by seed/pixel/sample) and
// consumes it in exactly the reference's draw order.
//
// Pinning: the building blocks are checked against the reference's own jest
// known-answer values (tests/test_oracle_kat.py, citing tests/**.test.ts line
// ranges). Whole-image radiance has no reference golden (the reference has no
// golden images and an unseeded RNG), so image-level parity of this oracle with
// the reference itself is statistical only. Third-party gl-matrix 3.4.3
// (package-lock.json:3694) is restated from its published source: normalize =
// a * (1/sqrt(|a|²)) when |a|² > 0, length = Math.hypot (V8 algorithm).
// Transcendentals (Math.cos/sin/tan/log10) use the C library here, which
// may differ from V8's fdlibm ports in the last ulp: parity unpinned at that
// level. Schlick's Math.pow(x, 5) is evaluated correctly rounded (R_pow5).
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace orc {

// ---------------------------------------------------------------------------
// Minimal JSON reader (independent of the product's parser)
// ---------------------------------------------------------------------------
struct J {
    enum T { NUL, BOO, NUM, STR, ARR, OBJ } t = NUL;
    bool b = false;
    double n = 0;
    std::string s;
    std::vector<J> a;
    std::vector<std::pair<std::string, J>> o;
    const J* at(const char* k) const {
        if (t != OBJ) return nullptr;
        for (auto& kv : o) if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct JReader {
    const char* p;
    const char* e;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
    [[noreturn]] void bad() { throw std::runtime_error("oracle: bad JSON"); }
    J val() {
        ws();
        if (p >= e) bad();
        J v;
        if (*p == '{') {
            ++p; v.t = J::OBJ; ws();
            if (*p == '}') { ++p; return v; }
            for (;;) {
                ws(); std::string k = str(); ws(); if (*p != ':') bad(); ++p;
                J x = val();
                bool replaced = false;
                for (auto& kv : v.o) if (kv.first == k) { kv.second = x; replaced = true; }
                if (!replaced) v.o.emplace_back(k, x);
                ws(); if (*p == ',') { ++p; continue; } if (*p == '}') { ++p; return v; } bad();
            }
        }
        if (*p == '[') {
            ++p; v.t = J::ARR; ws();
            if (*p == ']') { ++p; return v; }
            for (;;) { v.a.push_back(val()); ws(); if (*p == ',') { ++p; continue; } if (*p == ']') { ++p; return v; } bad(); }
        }
        if (*p == '"') { v.t = J::STR; v.s = str(); return v; }
        auto kw = [&](const char* w) { size_t n = strlen(w); if ((size_t)(e - p) >= n && !strncmp(p, w, n)) { p += n; return true; } return false; };
        if (kw("true")) { v.t = J::BOO; v.b = true; return v; }
        if (kw("false")) { v.t = J::BOO; return v; }
        if (kw("null")) return v;
        if (kw("NaN")) { v.t = J::NUM; v.n = NAN; return v; }
        if (kw("Infinity")) { v.t = J::NUM; v.n = INFINITY; return v; }
        if (kw("-Infinity")) { v.t = J::NUM; v.n = -INFINITY; return v; }
        char* end = nullptr;
        v.t = J::NUM; v.n = strtod(p, &end);
        if (end == p) bad();
        p = end;
        return v;
    }
    std::string str() {
        if (*p != '"') bad();
        ++p; std::string r;
        while (p < e && *p != '"') {
            if (*p == '\\') {
                ++p;
                char c = *p++;
                if (c == 'n') r += '\n'; else if (c == 't') r += '\t'; else if (c == 'u') { p += 4; r += '?'; }
                else r += c;
            } else r += *p++;
        }
        ++p;
        return r;
    }
};

J parse_json(const char* s) {
    JReader r{s, s + strlen(s)};
    return r.val();
}

double num(const J* v, double dflt) {
    if (!v) return dflt;
    if (v->t == J::NUM) return v->n;
    if (v->t == J::BOO) return v->b ? 1 : 0;
    if (v->t == J::NUL) return 0;
    return NAN;
}
bool truthy(const J* v) {
    if (!v) return false;
    if (v->t == J::NUL) return false;
    if (v->t == J::BOO) return v->b;
    if (v->t == J::NUM) return !(v->n == 0 || v->n != v->n);
    if (v->t == J::STR) return !v->s.empty();
    return true;
}

// ---------------------------------------------------------------------------
// Counters (algorithmic work, for the roofline accounting of SURVEY.md §8d)
// ---------------------------------------------------------------------------
struct Counters {
    double node_tests = 0, sphere_tests = 0, quad_tests = 0, plane_tests = 0;
    double material_fetches = 0, light_quad_evals = 0, light_sphere_evals = 0;
    double bounces = 0, diffuse_bounces = 0, samples = 0, rays = 0;
    void add(const Counters& o) {
        node_tests += o.node_tests; sphere_tests += o.sphere_tests; quad_tests += o.quad_tests;
        plane_tests += o.plane_tests; material_fetches += o.material_fetches;
        light_quad_evals += o.light_quad_evals; light_sphere_evals += o.light_sphere_evals;
        bounces += o.bounces; diffuse_bounces += o.diffuse_bounces; samples += o.samples; rays += o.rays;
    }
};
thread_local Counters* g_cnt = nullptr;
#define CNT(field) do { if (g_cnt) g_cnt->field += 1; } while (0)

// ---------------------------------------------------------------------------
// RNG: seeded replacement for Math.random
// ---------------------------------------------------------------------------
static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct Rng {
    uint64_t state;
    static Rng for_path(uint32_t seed, uint32_t pixel, uint32_t sample) {
        return Rng{splitmix64((((uint64_t)pixel << 32) | sample) ^ splitmix64(seed))};
    }
    uint32_t next_u32() {
        uint64_t old = state;
        state = old * 6364136223846793005ull + 1442695040888963407ull;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((32u - rot) & 31u));
    }
};
thread_local Rng* g_rng = nullptr;
thread_local int g_real_is_float = 0;
// Math.random() restated: [0,1). ref mode: u32 * 2^-32; fast mode: 24-bit.
static double js_random() {
    if (!g_rng) throw std::runtime_error("oracle: RNG not bound");
    uint32_t x = g_rng->next_u32();
    if (g_real_is_float) return (double)(float)((float)(x >> 8) * (1.0f / 16777216.0f));
    return (double)x * (1.0 / 4294967296.0);
}

// ---------------------------------------------------------------------------
// Math model
// ---------------------------------------------------------------------------
template <class R> static inline R jmin(R a, R b) {
    if (a != a || b != b) return a + b;
    if (a < b) return a;
    if (b < a) return b;
    return (a == 0 && b == 0) ? (std::signbit(a) ? a : b) : a;
}
template <class R> static inline R jmax(R a, R b) {
    if (a != a || b != b) return a + b;
    if (a > b) return a;
    if (b > a) return b;
    return (a == 0 && b == 0) ? (std::signbit(a) ? b : a) : a;
}
template <class R> static inline R R_sqrt(R x) { return std::sqrt(x); }
template <class R> static inline R R_cos(R x) { return std::cos(x); }
template <class R> static inline R R_sin(R x) { return std::sin(x); }
template <class R> static inline R R_pow(R x, R y) { return std::pow(x, y); }
// Schlick's Math.pow(x, 5) (src/materials/dielectric.ts:98) in ref mode:
// the correctly rounded x^5, formed in binary128 and rounded once. V8's fdlibm
// pow and glibc's pow are each within 1 ulp of it (neither is correctly
// rounded: glibc differs for ~0.1 % of arguments in [0, 1]); the product
// computes the same value by a different route (double-double).
static inline double R_pow5(double x) {
    __float128 q = (__float128)x;
    q = q * q * q * q * q;
    return (double)q;
}
static inline float R_pow5(float x) { return std::pow(x, 5.0f); }

static double hypot3_v8(double x, double y, double z) {
    double in[3] = {x, y, z}, ab[3] = {0, 0, 0};
    bool isnan_ = false; double mx = 0;
    for (int i = 0; i < 3; i++) {
        if (in[i] != in[i]) { isnan_ = true; continue; }
        ab[i] = std::fabs(in[i]); if (ab[i] > mx) mx = ab[i];
    }
    if (mx == INFINITY) return INFINITY;
    if (isnan_) return NAN;
    if (mx == 0) return 0;
    double sum = 0, c = 0;
    for (int i = 0; i < 3; i++) { double n = ab[i] / mx; double s = n * n - c; double pr = sum + s; c = (pr - sum) - s; sum = pr; }
    return std::sqrt(sum) * mx;
}

// Vec3 over a Float32Array; R is the JS-number type.
template <class R>
struct Vec3 {
    float v[3] = {0, 0, 0};
    static Vec3 create(R x, R y, R z) { Vec3 r; r.v[0] = (float)x; r.v[1] = (float)y; r.v[2] = (float)z; return r; }
    R x() const { return (R)v[0]; }
    R y() const { return (R)v[1]; }
    R z() const { return (R)v[2]; }
    Vec3 add(const Vec3& b) const { return create((R)v[0] + (R)b.v[0], (R)v[1] + (R)b.v[1], (R)v[2] + (R)b.v[2]); }
    Vec3 subtract(const Vec3& b) const { return create((R)v[0] - (R)b.v[0], (R)v[1] - (R)b.v[1], (R)v[2] - (R)b.v[2]); }
    Vec3 multiply(R t) const { return create((R)v[0] * t, (R)v[1] * t, (R)v[2] * t); }
    Vec3 multiplyVec(const Vec3& b) const { return create((R)v[0] * (R)b.v[0], (R)v[1] * (R)b.v[1], (R)v[2] * (R)b.v[2]); }
    Vec3 divide(R t) const { R inv = (R)1 / t; return create((R)v[0] * inv, (R)v[1] * inv, (R)v[2] * inv); }
    R dot(const Vec3& b) const { return (R)v[0] * (R)b.v[0] + (R)v[1] * (R)b.v[1] + (R)v[2] * (R)b.v[2]; }
    R lengthSquared() const { return (R)v[0] * (R)v[0] + (R)v[1] * (R)v[1] + (R)v[2] * (R)v[2]; }
    R length() const { return (R)hypot3_v8(v[0], v[1], v[2]); }
    Vec3 cross(const Vec3& b) const {
        R ax = v[0], ay = v[1], az = v[2], bx = b.v[0], by = b.v[1], bz = b.v[2];
        return create(ay * bz - az * by, az * bx - ax * bz, ax * by - ay * bx);
    }
    Vec3 unitVector() const {
        R x = v[0], y = v[1], z = v[2];
        R len = x * x + y * y + z * z;
        if (len > 0) len = (R)1 / R_sqrt<R>(len);
        return create((R)v[0] * len, (R)v[1] * len, (R)v[2] * len);
    }
    Vec3 negate() const {
        Vec3 r = create(-(R)v[0], -(R)v[1], -(R)v[2]);
        for (int i = 0; i < 3; i++) if (r.v[i] == 0) r.v[i] = 0;
        return r;
    }
    Vec3 reflect(const Vec3& n) const {
        R d = dot(n);
        Vec3 s = n.multiply(2 * d);
        return create((R)v[0] - (R)s.v[0], (R)v[1] - (R)s.v[1], (R)v[2] - (R)s.v[2]);
    }
    Vec3 refract(const Vec3& n, R eta) const {
        R cosTheta = jmin<R>(negate().dot(n), (R)1.0);
        Vec3 perp = add(n.multiply(cosTheta)).multiply(eta);
        Vec3 par = n.multiply(-R_sqrt<R>(std::fabs((R)1.0 - perp.lengthSquared())));
        return perp.add(par);
    }
    R illuminance() const { return (R)(0.299 * (double)v[0] + 0.587 * (double)v[1] + 0.114 * (double)v[2]); }
    static Vec3 random(R mn, R mx) {
        Vec3 r;
        for (int i = 0; i < 3; i++) r.v[i] = (float)(mn + (mx - mn) * (R)js_random());
        return r;
    }
    static Vec3 randomInUnitSphere() {
        for (;;) { Vec3 p = random(-1, 1); if (p.lengthSquared() < 1) return p; }
    }
    static Vec3 randomCosineDirection() {
        R r1 = (R)js_random(); R r2 = (R)js_random();
        R phi = 2 * (R)M_PI * r1; R s = R_sqrt<R>(r2);
        return create(R_cos<R>(phi) * s, R_sin<R>(phi) * s, R_sqrt<R>(1 - r2));
    }
    static Vec3 randomToSphere(R radius, R d2) {
        R r1 = (R)js_random(); R r2 = (R)js_random();
        R z = 1 + r2 * (R_sqrt<R>(1 - radius * radius / d2) - 1);
        R phi = 2 * (R)M_PI * r1;
        return create(R_cos<R>(phi) * R_sqrt<R>(1 - z * z), R_sin<R>(phi) * R_sqrt<R>(1 - z * z), z);
    }
    static Vec3 randomInUnitDisk() {
        for (;;) {
            R a = 2 * (R)js_random() - 1; R b = 2 * (R)js_random() - 1;
            Vec3 p = create(a, b, 0);
            if (p.lengthSquared() < 1) return p;
        }
    }
};

template <class R> struct Interval {
    R min, max;
    bool surrounds(R x) const { return min < x && x < max; }
};
template <class R> struct Ray {
    Vec3<R> origin, direction;
    Vec3<R> at(R t) const { return origin.add(direction.multiply(t)); }
};

template <class R> struct Material;

template <class R> struct HitRecord {
    Vec3<R> p, normal;
    R t;
    bool frontFace;
    const Material<R>* material;
};

// AABB (src/geometry/aabb.ts)
template <class R> struct AABB {
    Vec3<R> minimum, maximum;
    bool hit(const Ray<R>& r, Interval<R> rayT) const {
        CNT(node_tests);
        for (int a = 0; a < 3; a++) {
            R invD = (R)1.0 / (R)r.direction.v[a];
            R t0 = ((R)minimum.v[a] - (R)r.origin.v[a]) * invD;
            R t1 = ((R)maximum.v[a] - (R)r.origin.v[a]) * invD;
            if (invD < 0) { R tmp = t0; t0 = t1; t1 = tmp; }
            R tMin = t0 > rayT.min ? t0 : rayT.min;
            R tMax = t1 < rayT.max ? t1 : rayT.max;
            if (tMax <= tMin) return false;
        }
        return true;
    }
    static AABB surroundingBox(const AABB& a, const AABB& b) {
        AABB r;
        r.minimum = Vec3<R>::create(jmin<R>(a.minimum.x(), b.minimum.x()), jmin<R>(a.minimum.y(), b.minimum.y()), jmin<R>(a.minimum.z(), b.minimum.z()));
        r.maximum = Vec3<R>::create(jmax<R>(a.maximum.x(), b.maximum.x()), jmax<R>(a.maximum.y(), b.maximum.y()), jmax<R>(a.maximum.z(), b.maximum.z()));
        return r;
    }
    static AABB empty() {
        return AABB{Vec3<R>::create(INFINITY, INFINITY, INFINITY), Vec3<R>::create(-INFINITY, -INFINITY, -INFINITY)};
    }
};

template <class R> struct PDF {
    virtual ~PDF() {}
    virtual R value(const Vec3<R>& d) const = 0;
    virtual Vec3<R> generate() const = 0;
};

template <class R> struct Hittable {
    virtual ~Hittable() {}
    virtual bool hit(const Ray<R>& r, Interval<R> t, HitRecord<R>& rec) const = 0;
    virtual AABB<R> boundingBox() const = 0;
    virtual bool isPdf() const { return false; }
    virtual R pdfValue(const Vec3<R>&, const Vec3<R>&) const { return 0; }
    virtual Vec3<R> pdfRandomVec(const Vec3<R>&) const { return Vec3<R>(); }
};

// ONBasis (src/geometry/onbasis.ts:18-51)
template <class R> struct ONB {
    Vec3<R> u, v, w;
    explicit ONB(const Vec3<R>& n) {
        w = n.unitVector();
        Vec3<R> a = std::fabs((R)w.v[0]) > (R)0.9 ? Vec3<R>::create(0, 1, 0) : Vec3<R>::create(1, 0, 0);
        v = w.cross(a).unitVector();
        u = w.cross(v);
    }
    Vec3<R> local(const Vec3<R>& a) const { return u.multiply(a.x()).add(v.multiply(a.y())).add(w.multiply(a.z())); }
};

// CosinePDF (src/geometry/pdf.ts:32-51)
template <class R> struct CosinePDF : PDF<R> {
    ONB<R> uvw;
    explicit CosinePDF(const Vec3<R>& w) : uvw(w) {}
    R value(const Vec3<R>& d) const override {
        R c = d.unitVector().dot(uvw.w);
        return c <= 0 ? (R)0 : c / (R)M_PI;
    }
    Vec3<R> generate() const override { return uvw.local(Vec3<R>::randomCosineDirection()); }
};

// MixturePDF (src/geometry/pdf.ts:57-99)
template <class R> struct MixturePDF : PDF<R> {
    std::vector<const PDF<R>*> pdfs;
    std::vector<R> weights;
    R total = 0;
    MixturePDF(std::vector<const PDF<R>*> p, std::vector<R> w) : pdfs(std::move(p)), weights(std::move(w)) {
        total = 0;
        for (R x : weights) total = total + x;
    }
    R value(const Vec3<R>& d) const override {
        R sum = 0;
        for (size_t i = 0; i < pdfs.size(); i++) sum += weights[i] * pdfs[i]->value(d);
        return sum / total;
    }
    Vec3<R> generate() const override {
        R rand = (R)js_random() * total;
        R partial = 0;
        for (size_t i = 0; i < pdfs.size(); i++) {
            partial += weights[i];
            if (rand < partial) return pdfs[i]->generate();
        }
        return pdfs.back()->generate();
    }
};

// light.pdf(origin) closures (src/entities/quad.ts:166-171, sphere.ts:149-154)
template <class R> struct LightPDF : PDF<R> {
    const Hittable<R>* obj;
    Vec3<R> origin;
    R value(const Vec3<R>& d) const override { return obj->pdfValue(origin, d); }
    Vec3<R> generate() const override { return obj->pdfRandomVec(origin); }
};

template <class R> struct ScatterResult {
    bool valid = false;
    Vec3<R> attenuation;
    std::shared_ptr<PDF<R>> pdf;
    bool hasScattered = false;
    Ray<R> scattered;
    bool reflected = false;
};

// Material (src/materials/material.ts)
template <class R> struct Material {
    virtual ~Material() {}
    virtual ScatterResult<R> scatter(const Ray<R>&, const HitRecord<R>&) const { return ScatterResult<R>(); }
    virtual Vec3<R> emitted(const HitRecord<R>&) const { return Vec3<R>::create(0, 0, 0); }
};
template <class R> struct Lambertian : Material<R> {
    Vec3<R> albedo;
    ScatterResult<R> scatter(const Ray<R>&, const HitRecord<R>& rec) const override {
        ScatterResult<R> s; s.valid = true; s.attenuation = albedo; s.pdf = std::make_shared<CosinePDF<R>>(rec.normal);
        return s;
    }
};
template <class R> struct Metal : Material<R> {
    Vec3<R> albedo; R fuzz;
    ScatterResult<R> scatter(const Ray<R>& rIn, const HitRecord<R>& rec) const override {
        Vec3<R> reflected = rIn.direction.unitVector().reflect(rec.normal);
        Vec3<R> fuzzy = fuzz > 0 ? reflected.add(Vec3<R>::randomInUnitSphere().multiply(fuzz)) : reflected;
        if (fuzzy.dot(rec.normal) <= 0) return ScatterResult<R>();
        ScatterResult<R> s; s.valid = true; s.attenuation = albedo; s.hasScattered = true; s.scattered = Ray<R>{rec.p, fuzzy};
        return s;
    }
};
template <class R> struct Dielectric : Material<R> {
    R ior;
    static R reflectance(R cosine, R ratio) {
        R r0 = (1 - ratio) / (1 + ratio);
        r0 = r0 * r0;
        return r0 + (1 - r0) * R_pow5((R)(1 - cosine));
    }
    ScatterResult<R> scatter(const Ray<R>& rIn, const HitRecord<R>& rec) const override {
        Vec3<R> att = Vec3<R>::create(1.0, 1.0, 1.0);
        R ratio = rec.frontFace ? ((R)1.0 / ior) : ior;
        Vec3<R> ud = rIn.direction.unitVector();
        R cosTheta = jmin<R>(ud.negate().dot(rec.normal), (R)1.0);
        R sinTheta = R_sqrt<R>((R)1.0 - cosTheta * cosTheta);
        bool cannot = ratio * sinTheta > (R)1.0;
        Vec3<R> dir; bool refl;
        if (cannot || reflectance(cosTheta, ratio) > (R)js_random()) { dir = ud.reflect(rec.normal); refl = true; }
        else { dir = ud.refract(rec.normal, ratio); refl = false; }
        ScatterResult<R> s; s.valid = true; s.attenuation = att; s.hasScattered = true; s.scattered = Ray<R>{rec.p, dir}; s.reflected = refl;
        return s;
    }
};
template <class R> struct DiffuseLight : Material<R> {
    Vec3<R> emit;
    Vec3<R> emitted(const HitRecord<R>&) const override { return emit; }
};
template <class R> struct MixedMaterial : Material<R> {
    const Material<R>* m1; const Material<R>* m2; R weight;
    ScatterResult<R> scatter(const Ray<R>& rIn, const HitRecord<R>& rec) const override {
        if ((R)js_random() < weight) return m1->scatter(rIn, rec);
        return m2->scatter(rIn, rec);
    }
    Vec3<R> emitted(const HitRecord<R>& rec) const override {
        return m1->emitted(rec).multiply(weight).add(m2->emitted(rec).multiply((R)1.0 - weight));
    }
};
template <class R> struct LayeredMaterial : Material<R> {
    const Dielectric<R>* outer; const Material<R>* inner;
    ScatterResult<R> scatter(const Ray<R>& rIn, const HitRecord<R>& rec) const override {
        ScatterResult<R> o = outer->scatter(rIn, rec);
        if (!o.valid) return o;
        if (o.reflected) return o;
        return inner->scatter(o.scattered, rec);
    }
    Vec3<R> emitted(const HitRecord<R>& rec) const override { return inner->emitted(rec); }
};

// Sphere (src/entities/sphere.ts)
template <class R> struct Sphere : Hittable<R> {
    Vec3<R> center; R radius; const Material<R>* material; AABB<R> box;
    void init() {
        Vec3<R> rv = Vec3<R>::create(radius, radius, radius);
        box = AABB<R>{center.subtract(rv), center.add(rv)};
    }
    bool hit(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const override {
        CNT(sphere_tests);
        return hit_raw(r, rayT, rec);
    }
    bool hit_raw(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const {
        Vec3<R> oc = r.origin.subtract(center);
        R a = r.direction.lengthSquared();
        R halfB = oc.dot(r.direction);
        R c = oc.lengthSquared() - radius * radius;
        R disc = halfB * halfB - a * c;
        if (disc < 0) return false;
        R sq = R_sqrt<R>(disc);
        R root = (-halfB - sq) / a;
        if (!rayT.surrounds(root)) {
            root = (-halfB + sq) / a;
            if (!rayT.surrounds(root)) return false;
        }
        Vec3<R> p = r.at(root);
        Vec3<R> normal = p.subtract(center).divide(radius);
        bool front = r.direction.dot(normal) <= 0;
        if (!front) normal = normal.negate();
        rec.t = root; rec.p = p; rec.normal = normal; rec.frontFace = front; rec.material = material;
        return true;
    }
    AABB<R> boundingBox() const override { return box; }
    bool isPdf() const override { return true; }
    R pdfValue(const Vec3<R>& origin, const Vec3<R>& dir) const override {
        CNT(light_sphere_evals);
        HitRecord<R> rec;
        if (!hit_raw(Ray<R>{origin, dir}, Interval<R>{(R)0.001, (R)INFINITY}, rec)) return 0;
        R d2 = center.subtract(origin).lengthSquared();
        if (d2 <= radius * radius) return (R)1.0 / ((R)4.0 * (R)M_PI);
        R cosT = R_sqrt<R>(1 - radius * radius / d2);
        R solid = 2 * (R)M_PI * (1 - cosT);
        return 1 / solid;
    }
    Vec3<R> pdfRandomVec(const Vec3<R>& origin) const override {
        Vec3<R> oc = center.subtract(origin);
        R d2 = oc.lengthSquared();
        ONB<R> uvw(oc);
        return uvw.local(Vec3<R>::randomToSphere(radius, d2));
    }
};

// Plane (src/entities/plane.ts)
template <class R> struct Plane : Hittable<R> {
    Vec3<R> q, u, v, normal, inverseNormal, w; R d; const Material<R>* material; AABB<R> box;
    void init() {
        Vec3<R> cp = u.cross(v);
        normal = cp.unitVector();
        inverseNormal = normal.negate();
        d = normal.dot(q);
        R cl2 = cp.lengthSquared();
        w = cp.divide(cl2);
        const R eps = (R)1e-4;
        if (std::fabs(normal.x()) > (R)0.9999) {
            R px = d / normal.x();
            box = AABB<R>{Vec3<R>::create(px - eps, -INFINITY, -INFINITY), Vec3<R>::create(px + eps, INFINITY, INFINITY)};
        } else if (std::fabs(normal.y()) > (R)0.9999) {
            R py = d / normal.y();
            box = AABB<R>{Vec3<R>::create(-INFINITY, py - eps, -INFINITY), Vec3<R>::create(INFINITY, py + eps, INFINITY)};
        } else if (std::fabs(normal.z()) > (R)0.9999) {
            R pz = d / normal.z();
            box = AABB<R>{Vec3<R>::create(-INFINITY, -INFINITY, pz - eps), Vec3<R>::create(INFINITY, INFINITY, pz + eps)};
        } else {
            box = AABB<R>{Vec3<R>::create(-INFINITY, -INFINITY, -INFINITY), Vec3<R>::create(INFINITY, INFINITY, INFINITY)};
        }
    }
    bool intersect(const Ray<R>& r, Interval<R> rayT, R& t, R& alpha, R& beta) const {
        R denom = normal.dot(r.direction);
        if (std::fabs(denom) < (R)1e-8) return false;
        t = (d - normal.dot(r.origin)) / denom;
        if (!rayT.surrounds(t)) return false;
        Vec3<R> ip = r.at(t);
        Vec3<R> ph = ip.subtract(q);
        alpha = w.dot(ph.cross(v));
        beta = w.dot(u.cross(ph));
        return true;
    }
    bool hit(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const override {
        CNT(plane_tests);
        R t, a, b;
        if (!intersect(r, rayT, t, a, b)) return false;
        rec.t = t; rec.p = r.at(t);
        rec.frontFace = r.direction.dot(normal) <= 0;
        rec.normal = rec.frontFace ? normal : inverseNormal;
        rec.material = material;
        return true;
    }
    AABB<R> boundingBox() const override { return box; }
};

// Quad (src/entities/quad.ts)
template <class R> struct Quad : Hittable<R> {
    Plane<R> plane; Vec3<R> q, u, v; const Material<R>* material; R area; AABB<R> box;
    void init() {
        plane.q = q; plane.u = u; plane.v = v; plane.material = material; plane.init();
        area = (R)u.cross(v).length();
        Vec3<R> v1 = q, v2 = q.add(u), v3 = q.add(v), v4 = q.add(u).add(v);
        auto mn = [](R a, R b, R c, R e) { return jmin<R>(jmin<R>(jmin<R>(a, b), c), e); };
        auto mx = [](R a, R b, R c, R e) { return jmax<R>(jmax<R>(jmax<R>(a, b), c), e); };
        const R eps = (R)1e-4;
        box = AABB<R>{Vec3<R>::create(mn(v1.x(), v2.x(), v3.x(), v4.x()) - eps, mn(v1.y(), v2.y(), v3.y(), v4.y()) - eps, mn(v1.z(), v2.z(), v3.z(), v4.z()) - eps),
                      Vec3<R>::create(mx(v1.x(), v2.x(), v3.x(), v4.x()) + eps, mx(v1.y(), v2.y(), v3.y(), v4.y()) + eps, mx(v1.z(), v2.z(), v3.z(), v4.z()) + eps)};
    }
    bool hit_raw(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const {
        R t, alpha, beta;
        if (!plane.intersect(r, rayT, t, alpha, beta)) return false;
        if (alpha < 0 || alpha > 1 || beta < 0 || beta > 1) return false;
        rec.t = t; rec.p = r.at(t);
        rec.frontFace = r.direction.dot(plane.normal) <= 0;
        rec.normal = rec.frontFace ? plane.normal : plane.normal.negate();
        rec.material = material;
        return true;
    }
    bool hit(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const override {
        CNT(quad_tests);
        return hit_raw(r, rayT, rec);
    }
    AABB<R> boundingBox() const override { return box; }
    bool isPdf() const override { return true; }
    R pdfValue(const Vec3<R>& origin, const Vec3<R>& dir) const override {
        CNT(light_quad_evals);
        HitRecord<R> rec;
        if (!hit_raw(Ray<R>{origin, dir}, Interval<R>{(R)0.001, (R)INFINITY}, rec)) return 0;
        R d2 = rec.p.subtract(origin).lengthSquared();
        R cosine = std::fabs(dir.dot(rec.normal));
        return d2 / (area * cosine);
    }
    Vec3<R> pdfRandomVec(const Vec3<R>& origin) const override {
        R alpha = (R)js_random(); R beta = (R)js_random();
        Vec3<R> rp = q.add(u.multiply(alpha)).add(v.multiply(beta));
        return rp.subtract(origin).unitVector();
    }
};

// HittableList (src/geometry/hittableList.ts)
template <class R> struct HittableList : Hittable<R> {
    std::vector<const Hittable<R>*> objects;
    bool hit(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const override {
        bool any = false;
        Interval<R> iv{rayT.min, rayT.max};
        for (auto* o : objects) {
            HitRecord<R> cur;
            if (o->hit(r, iv, cur)) { iv.max = cur.t; rec = cur; any = true; }
        }
        return any;
    }
    AABB<R> boundingBox() const override {
        if (objects.empty()) return AABB<R>::empty();
        AABB<R> b = objects[0]->boundingBox();
        for (size_t i = 1; i < objects.size(); i++) b = AABB<R>::surroundingBox(b, objects[i]->boundingBox());
        return b;
    }
};

template <class R> struct EmptyHittable : Hittable<R> {
    bool hit(const Ray<R>&, Interval<R>, HitRecord<R>&) const override { return false; }
    AABB<R> boundingBox() const override { return AABB<R>::empty(); }
};

template <class R> struct Scene;

// BVHNode (src/geometry/bvh.ts)
template <class R> struct BVHNode : Hittable<R> {
    const Hittable<R>* left = nullptr; const Hittable<R>* right = nullptr; AABB<R> box;
    static bool cmp(const Hittable<R>* a, const Hittable<R>* b, int axis) {
        return a->boundingBox().minimum.v[axis] < b->boundingBox().minimum.v[axis];
    }
    BVHNode(std::vector<const Hittable<R>*> list, Scene<R>& owner, int depth);
    bool hit(const Ray<R>& r, Interval<R> rayT, HitRecord<R>& rec) const override {
        if (!box.hit(r, rayT)) return false;
        HitRecord<R> hl;
        bool l = left->hit(r, rayT, hl);
        Interval<R> ri = l ? Interval<R>{rayT.min, hl.t} : rayT;
        HitRecord<R> hr;
        bool rr = right->hit(r, ri, hr);
        if (rr) { rec = hr; return true; }
        if (l) { rec = hl; return true; }
        return false;
    }
    AABB<R> boundingBox() const override { return box; }
};

template <class R> struct Scene {
    std::vector<std::unique_ptr<Material<R>>> mats;
    std::vector<std::unique_ptr<Hittable<R>>> objs;     // scene objects (in SceneData order)
    std::vector<std::unique_ptr<Hittable<R>>> owned;    // BVH nodes, leaf lists
    EmptyHittable<R> empty;
    const Hittable<R>* world = nullptr;
    std::vector<const Hittable<R>*> lights;
    int bvh_depth = 0;
    std::map<std::string, const J*> matmap;

    const Material<R>* create_material(const J* ref) {
        const J* md = nullptr;
        if (ref && ref->t == J::STR) { auto it = matmap.find(ref->s); md = it == matmap.end() ? nullptr : it->second; }
        else if (truthy(ref)) md = ref;
        if (!md) throw std::runtime_error("Material not found");
        const J* tj = md->at("type");
        std::string type = tj && tj->t == J::STR ? tj->s : "undefined";
        auto vec = [&](const char* k) {
            const J* a = md->at(k);
            if (!a || a->t != J::ARR) throw std::runtime_error(std::string("not iterable: ") + k);
            R c[3] = {(R)NAN, (R)NAN, (R)NAN};
            for (size_t i = 0; i < 3 && i < a->a.size(); i++) c[i] = (R)num(&a->a[i], NAN);
            return Vec3<R>::create(c[0], c[1], c[2]);
        };
        if (type == "lambert") { auto m = std::make_unique<Lambertian<R>>(); m->albedo = vec("color"); mats.push_back(std::move(m)); }
        else if (type == "metal") {
            auto m = std::make_unique<Metal<R>>(); m->albedo = vec("color");
            const J* f = md->at("fuzz"); double fz = f ? num(f, 0) : 0.0;
            m->fuzz = (R)(fz < 1 ? jmax<double>(0, fz) : 1.0);
            mats.push_back(std::move(m));
        } else if (type == "glass") { auto m = std::make_unique<Dielectric<R>>(); m->ior = (R)num(md->at("ior"), NAN); mats.push_back(std::move(m)); }
        else if (type == "light") { auto m = std::make_unique<DiffuseLight<R>>(); m->emit = vec("emit"); mats.push_back(std::move(m)); }
        else if (type == "mixed") {
            auto m = std::make_unique<MixedMaterial<R>>();
            m->m1 = create_material(md->at("diff")); m->m2 = create_material(md->at("spec"));
            m->weight = (R)jmax<double>(0.0, jmin<double>(1.0, num(md->at("weight"), NAN)));
            mats.push_back(std::move(m));
        } else if (type == "layered") {
            auto m = std::make_unique<LayeredMaterial<R>>();
            const J* oref = md->at("outer");
            const J* od = nullptr;
            if (oref && oref->t == J::STR) { auto it = matmap.find(oref->s); od = it == matmap.end() ? nullptr : it->second; }
            else if (truthy(oref)) od = oref;
            if (!od) throw std::runtime_error("Material not found");
            const J* ot = od->at("type");
            if (!(ot && ot->t == J::STR && ot->s == "glass")) throw std::runtime_error("Material is not a dielectric");
            auto g = std::make_unique<Dielectric<R>>(); g->ior = (R)num(od->at("ior"), NAN);
            m->outer = g.get(); mats.push_back(std::move(g));
            m->inner = create_material(md->at("inner"));
            mats.push_back(std::move(m));
        } else throw std::runtime_error("Unknown material type: " + type);
        return mats.back().get();
    }
};

template <class R>
BVHNode<R>::BVHNode(std::vector<const Hittable<R>*> list, Scene<R>& owner, int depth) {
    owner.bvh_depth = std::max(owner.bvh_depth, depth);
    AABB<R> nb = list[0]->boundingBox();
    for (size_t i = 1; i < list.size(); i++) nb = AABB<R>::surroundingBox(nb, list[i]->boundingBox());
    double xe = (double)nb.maximum.v[0] - (double)nb.minimum.v[0];
    double ye = (double)nb.maximum.v[1] - (double)nb.minimum.v[1];
    double ze = (double)nb.maximum.v[2] - (double)nb.minimum.v[2];
    int axis = 0;
    if (ye > xe && ye > ze) axis = 1; else if (ze > xe && ze > ye) axis = 2;
    size_t span = list.size();
    if (span == 1) { left = list[0]; right = &owner.empty; }
    else if (span == 2) {
        if (cmp(list[0], list[1], axis)) { left = list[0]; right = list[1]; } else { left = list[1]; right = list[0]; }
    } else if (span <= 4) {
        auto l = std::make_unique<HittableList<R>>();
        for (auto* o : list) l->objects.push_back(o);
        left = l.get(); owner.owned.push_back(std::move(l));
        right = &owner.empty;
    } else {
        // V8 TimSort with a comparator returning -1/1 (never 0) == stable sort.
        std::stable_sort(list.begin(), list.end(), [axis](const Hittable<R>* a, const Hittable<R>* b) { return cmp(a, b, axis); });
        size_t mid = span / 2;
        auto L = std::make_unique<BVHNode<R>>(std::vector<const Hittable<R>*>(list.begin(), list.begin() + mid), owner, depth + 1);
        auto Rr = std::make_unique<BVHNode<R>>(std::vector<const Hittable<R>*>(list.begin() + mid, list.end()), owner, depth + 1);
        left = L.get(); right = Rr.get();
        owner.owned.push_back(std::move(L)); owner.owned.push_back(std::move(Rr));
    }
    box = AABB<R>::surroundingBox(left->boundingBox(), right->boundingBox());
}

struct PixelOut {
    float color[3];
    int samples; long bounces; int minB; int maxB;
};

// Camera (src/camera.ts)
template <class R> struct Camera {
    Scene<R> scene;
    int W = 0, H = 0;
    Vec3<R> center, p00, du, dv, ddu, ddv, bgTop, bgBottom;
    bool hasBg = false;
    R aperture = 0, samplesOpt = 100, depthOpt = 100, aTol = 0.05, aBatch = 10, rDepth = 3;
    bool roulette = true;
    int mode = 0;
    bool adaptive = false;
    uint32_t seed = 0x5EED;
    Vec3<R> u, v, w;

    void load(const J& sd, const J* ro) {
        if (const J* ms = sd.at("materials")) if (ms->t == J::ARR) for (auto& e : ms->a) {
            const J* id = e.at("id"); std::string k = id && id->t == J::STR ? id->s : "";
            if (id && id->t == J::NUM) { char b[64]; snprintf(b, 64, "%.17g", id->n); k = b; }
            scene.matmap[k] = e.at("material");
        }
        const J* os = sd.at("objects");
        if (!os || os->t != J::ARR || os->a.empty()) throw std::runtime_error("no objects");
        std::vector<const Hittable<R>*> objs;
        for (auto& od : os->a) {
            const Material<R>* m = scene.create_material(od.at("material"));
            const J* tj = od.at("type"); std::string t = tj && tj->t == J::STR ? tj->s : "";
            auto vec = [&](const char* k) {
                const J* a = od.at(k);
                if (!a || a->t != J::ARR) throw std::runtime_error("not iterable");
                R c[3] = {(R)NAN, (R)NAN, (R)NAN};
                for (size_t i = 0; i < 3 && i < a->a.size(); i++) c[i] = (R)num(&a->a[i], NAN);
                return Vec3<R>::create(c[0], c[1], c[2]);
            };
            if (t == "sphere") { auto s = std::make_unique<Sphere<R>>(); s->center = vec("pos"); s->radius = (R)num(od.at("r"), NAN); s->material = m; s->init(); scene.objs.push_back(std::move(s)); }
            else if (t == "plane") { auto p = std::make_unique<Plane<R>>(); p->q = vec("pos"); p->u = vec("u"); p->v = vec("v"); p->material = m; p->init(); scene.objs.push_back(std::move(p)); }
            else if (t == "quad") { auto q = std::make_unique<Quad<R>>(); q->q = vec("pos"); q->u = vec("u"); q->v = vec("v"); q->material = m; q->init(); scene.objs.push_back(std::move(q)); }
            else throw std::runtime_error("Unknown object type: " + t);
            objs.push_back(scene.objs.back().get());
        }
        auto root = std::make_unique<BVHNode<R>>(objs, scene, 1);
        scene.world = root.get();
        scene.owned.push_back(std::move(root));
        for (size_t i = 0; i < os->a.size(); i++)
            if (truthy(os->a[i].at("light")) && scene.objs[i]->isPdf()) scene.lights.push_back(scene.objs[i].get());

        const J* cd = sd.at("camera");
        if (!cd) throw std::runtime_error("no camera");
        auto cvec = [&](const J* a) {
            if (!a || a->t != J::ARR) throw std::runtime_error("camera vector missing");
            R c[3] = {(R)NAN, (R)NAN, (R)NAN};
            for (size_t i = 0; i < 3 && i < a->a.size(); i++) c[i] = (R)num(&a->a[i], NAN);
            return Vec3<R>::create(c[0], c[1], c[2]);
        };
        const J* rr = sd.at("render");
        auto opt = [&](const char* k) -> const J* { if (ro) if (const J* x = ro->at(k)) return x; if (rr) if (const J* x = rr->at(k)) return x; return nullptr; };
        double width = opt("width") ? num(opt("width"), NAN) : 400;
        double aspect = opt("aspect") ? num(opt("aspect"), NAN) : 16.0 / 9.0;
        samplesOpt = (R)(opt("samples") ? num(opt("samples"), NAN) : 100);
        depthOpt = (R)(opt("depth") ? num(opt("depth"), NAN) : 100);
        aTol = (R)(opt("aTolerance") ? num(opt("aTolerance"), NAN) : 0.05);
        aBatch = (R)(opt("aBatch") ? num(opt("aBatch"), NAN) : 10);
        roulette = opt("roulette") ? truthy(opt("roulette")) : true;
        rDepth = (R)(opt("rouletteDepth") ? num(opt("rouletteDepth"), NAN) : 3);
        if (const J* m = opt("mode")) { if (m->t == J::STR) mode = m->s == "bounces" ? 1 : (m->s == "samples" ? 2 : 0); }
        if (const J* s = opt("seed")) seed = (uint32_t)(int64_t)num(s, 0);

        // Camera arithmetic is always JS doubles; vectors fp32 (host-side, once).
        const J* vf = cd->at("vfov");
        double vfov = vf ? num(vf, NAN) : NAN;
        Vec3<double> from = Vec3<double>::create(0, 0, 0), at = from, up = from;
        auto dvec = [&](const J* a) {
            if (!a || a->t != J::ARR) throw std::runtime_error("camera vector missing");
            double c[3] = {NAN, NAN, NAN};
            for (size_t i = 0; i < 3 && i < a->a.size(); i++) c[i] = num(&a->a[i], NAN);
            return Vec3<double>::create(c[0], c[1], c[2]);
        };
        from = dvec(cd->at("from")); at = dvec(cd->at("at")); up = dvec(cd->at("up"));
        const J* ap = cd->at("aperture"); double apd = ap ? num(ap, NAN) : NAN;
        const J* fo = cd->at("focus"); double focus = fo ? num(fo, NAN) : NAN;
        const J* bg = cd->at("background");
        hasBg = truthy(bg);
        if (hasBg) { bgTop = cvec(bg->at("top")); bgBottom = cvec(bg->at("bottom")); }
        W = (int)width;
        double Hd = std::ceil(width / aspect);
        H = (int)Hd;
        double fd = (focus != 0 && focus == focus) ? focus : from.subtract(at).length();
        double theta = vfov * (M_PI / 180);
        double h = std::tan(theta / 2);
        double vh = 2 * h * fd;
        double ar = width / Hd;
        double vw = vh * ar;
        Vec3<double> ww = from.subtract(at).unitVector();
        Vec3<double> uu = up.cross(ww).unitVector();
        Vec3<double> vv = ww.cross(uu);
        Vec3<double> vpU = uu.multiply(vw), vpV = vv.multiply(-vh);
        Vec3<double> pdu = vpU.divide(width), pdv = vpV.divide(Hd);
        Vec3<double> hu = vpU.divide(2), hv = vpV.divide(2);
        Vec3<double> ul = from.subtract(ww.multiply(fd)).subtract(hu).subtract(hv);
        Vec3<double> p0 = ul.add(pdu.add(pdv).multiply(0.5));
        Vec3<double> dU = uu.multiply(apd / 2), dV = vv.multiply(apd / 2);
        auto cv = [](const Vec3<double>& s) { Vec3<R> r; r.v[0] = s.v[0]; r.v[1] = s.v[1]; r.v[2] = s.v[2]; return r; };
        center = cv(from); p00 = cv(p0); du = cv(pdu); dv = cv(pdv); ddu = cv(dU); ddv = cv(dV);
        u = cv(uu); v = cv(vv); w = cv(ww);
        aperture = (R)apd;
        adaptive = aTol > 0 && samplesOpt > 1;
    }

    Ray<R> getRay(int i, int j) const {
        Vec3<R> pc = p00.add(du.multiply((R)i)).add(dv.multiply((R)j));
        Vec3<R> ps = pc;
        if (samplesOpt > 1) {
            R px = (R)-0.5 + (R)js_random();
            R py = (R)-0.5 + (R)js_random();
            ps = pc.add(du.multiply(px)).add(dv.multiply(py));
        }
        Vec3<R> ro = center;
        Vec3<R> rd = ps.subtract(center);
        if (aperture > 0) {
            Vec3<R> d = Vec3<R>::randomInUnitDisk();
            Vec3<R> off = ddu.multiply(d.x()).add(ddv.multiply(d.y()));
            ro = center.add(off);
            rd = ps.subtract(ro);
        }
        return Ray<R>{ro, rd};
    }

    Vec3<R> rayColor(const Ray<R>& r, Vec3<R> T, int& bounces) const {
        if ((R)bounces >= depthOpt) return Vec3<R>::create(0, 0, 0);
        if (roulette && (R)bounces >= rDepth) {
            R mc = jmax<R>(jmax<R>((R)T.v[0], (R)T.v[1]), (R)T.v[2]);
            R p = jmin<R>(mc, (R)0.95);
            if ((R)js_random() > p) return Vec3<R>::create(0, 0, 0);
            T = T.divide(p);
        }
        HitRecord<R> rec;
        if (g_cnt) g_cnt->rays += 1;
        if (!scene.world->hit(r, Interval<R>{(R)0.001, (R)INFINITY}, rec)) {
            if (!hasBg) throw std::runtime_error("Cannot read properties of undefined (reading 'top')");
            Vec3<R> ud = r.direction.unitVector();
            R a = (R)0.5 * (ud.y() + (R)1.0);
            return bgTop.multiply((R)1.0 - a).add(bgBottom.multiply(a)).multiplyVec(T);
        }
        CNT(material_fetches);
        Vec3<R> emitted = rec.material->emitted(rec).multiplyVec(T);
        ScatterResult<R> sr = rec.material->scatter(r, rec);
        if (!sr.valid) return emitted;
        bounces++;
        if (sr.hasScattered) {
            Vec3<R> nt = T.multiplyVec(sr.attenuation);
            Vec3<R> sc = rayColor(sr.scattered, nt, bounces);
            return emitted.add(sc);
        }
        if (sr.pdf) {
            CNT(diffuse_bounces);
            std::vector<LightPDF<R>> lp(scene.lights.size());
            std::vector<const PDF<R>*> pdfs{sr.pdf.get()};
            std::vector<R> ws{(R)0.5};
            for (size_t k = 0; k < scene.lights.size(); k++) {
                lp[k].obj = scene.lights[k]; lp[k].origin = rec.p;
            }
            for (size_t k = 0; k < lp.size(); k++) { pdfs.push_back(&lp[k]); ws.push_back((R)0.5 / (R)lp.size()); }
            MixturePDF<R> mix(pdfs, ws);
            Vec3<R> dir = mix.generate();
            Ray<R> sc{rec.p, dir};
            R pv = mix.value(dir);
            if (pv <= (R)0.0001) return emitted;
            R spv = sr.pdf->value(dir);
            Vec3<R> brdf = sr.attenuation.multiply(spv);
            Vec3<R> nt = T.multiplyVec(brdf).divide(pv);
            Vec3<R> inc = rayColor(sc, nt, bounces);
            return emitted.add(inc);
        }
        return emitted;
    }

    bool pixelConverged(int n, double sumIll, double sumIll2) const {
        // src/camera.ts:348-368, including its NaN behaviour.
        if ((double)aTol <= 0 || (double)samplesOpt <= 1 || n < 2) return false;
        double rem = std::fmod((double)n, (double)aBatch);
        if (rem != 0 || rem != rem) return false;
        double mean = sumIll / n;
        double var = (sumIll2 - (sumIll * sumIll) / n) / (n - 1);
        if (var <= 0 || var != var) return true;
        double ci = 1.96 * std::sqrt(var) / std::sqrt((double)n);
        return ci <= (double)aTol * mean;
    }

    PixelOut renderPixel(int i, int j) const {
        Vec3<R> color = Vec3<R>::create(0, 0, 0);
        int n = 0; long bsum = 0; int mn = INT32_MAX, mx = 0;
        double sIll = 0, sIll2 = 0;
        while ((R)n < samplesOpt && !pixelConverged(n, sIll, sIll2)) {
            Rng rng = Rng::for_path(seed, (uint32_t)j * (uint32_t)W + (uint32_t)i, (uint32_t)n);
            g_rng = &rng;
            Ray<R> r = getRay(i, j);
            int b = 0;
            Vec3<R> c = rayColor(r, Vec3<R>::create(1, 1, 1), b);
            g_rng = nullptr;
            if (g_cnt) { g_cnt->samples += 1; g_cnt->bounces += b; }
            color = color.add(c);
            n++; bsum += b; mn = std::min(mn, b); mx = std::max(mx, b);
            if (adaptive) { double il = (double)c.illuminance(); sIll += il; sIll2 += il * il; }
        }
        Vec3<R> fin;
        if (mode == 1) {
            double avg = n > 0 ? (double)bsum / n : 0;
            fin = Vec3<R>::create(0, 0, (R)jmin<double>(avg / (double)depthOpt, 1.0));
        } else if (mode == 2) {
            fin = Vec3<R>::create((R)jmin<double>((double)n / (double)samplesOpt, 1.0), 0, 0);
        } else {
            fin = color.divide((R)n);
        }
        PixelOut o;
        o.color[0] = fin.v[0]; o.color[1] = fin.v[1]; o.color[2] = fin.v[2];
        o.samples = n; o.bounces = bsum; o.minB = mn; o.maxB = mx;
        return o;
    }
};

// writeColorToBuffer (src/camera.ts:455-472) into a Uint8ClampedArray.
static uint8_t to_u8(float c) {
    double r = std::sqrt((double)c);
    double v = std::floor(255.999 * r);
    if (!(v > 0)) return 0;  // NaN and negatives clamp to 0
    if (v >= 255) return 255;
    return (uint8_t)v;
}

}  // namespace orc

using namespace orc;

namespace {
thread_local std::string g_err;

template <class R>
int render_impl(const char* scene_json, const char* render_json, int rx, int ry, int rw, int rh, int row_step,
                int threads, float* radiance, uint8_t* rgb, int32_t* px_samples, int32_t* px_bounces,
                double* stats, double* counters, int* dims) {
    J sd = parse_json(scene_json);
    J ro;
    bool has_ro = render_json && render_json[0];
    if (has_ro) ro = parse_json(render_json);
    auto cam = std::make_unique<Camera<R>>();
    cam->load(sd, has_ro ? &ro : nullptr);
    if (dims) { dims[0] = cam->W; dims[1] = cam->H; dims[2] = cam->scene.bvh_depth; dims[3] = (int)cam->scene.lights.size(); }
    if (!radiance && !rgb && !stats && !counters) return 0;
    const int endX = std::min(rx + rw, cam->W), endY = std::min(ry + rh, cam->H);
    if (row_step < 1) row_step = 1;
    std::vector<int> rows;
    for (int j = ry; j < endY; j += row_step) rows.push_back(j);
    threads = std::max(1, threads);
    std::vector<Counters> cnts(threads);
    std::vector<double> st(threads * 7, 0);
    for (int t = 0; t < threads; t++) { st[t * 7 + 2] = INFINITY; st[t * 7 + 5] = INFINITY; }
    std::atomic<size_t> next{0};
    std::vector<std::string> errs(threads);
    auto worker = [&](int t) {
        g_real_is_float = std::is_same<R, float>::value ? 1 : 0;
        g_cnt = counters ? &cnts[t] : nullptr;
        try {
            for (;;) {
                size_t k = next.fetch_add(1);
                if (k >= rows.size()) break;
                int j = rows[k];
                for (int i = rx; i < endX; i++) {
                    PixelOut o = cam->renderPixel(i, j);
                    size_t off = ((size_t)j * cam->W + i);
                    if (radiance) { radiance[off * 3] = o.color[0]; radiance[off * 3 + 1] = o.color[1]; radiance[off * 3 + 2] = o.color[2]; }
                    if (rgb) { rgb[off * 3] = to_u8(o.color[0]); rgb[off * 3 + 1] = to_u8(o.color[1]); rgb[off * 3 + 2] = to_u8(o.color[2]); }
                    if (px_samples) px_samples[off] = o.samples;
                    if (px_bounces) px_bounces[off] = (int32_t)o.bounces;
                    double* s = &st[t * 7];
                    s[0] += 1; s[1] += o.samples; s[2] = std::min(s[2], (double)o.samples); s[3] = std::max(s[3], (double)o.samples);
                    s[4] += (double)o.bounces; s[5] = std::min(s[5], o.samples ? (double)o.minB : INFINITY); s[6] = std::max(s[6], (double)o.maxB);
                }
            }
        } catch (const std::exception& e) { errs[t] = e.what(); }
        g_cnt = nullptr;
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(worker, t);
    worker(0);
    for (auto& th : pool) th.join();
    for (auto& e : errs) if (!e.empty()) throw std::runtime_error(e);
    if (stats) {
        double s[7] = {0, 0, INFINITY, 0, 0, INFINITY, 0};
        for (int t = 0; t < threads; t++) {
            double* x = &st[t * 7];
            s[0] += x[0]; s[1] += x[1]; s[2] = std::min(s[2], x[2]); s[3] = std::max(s[3], x[3]);
            s[4] += x[4]; s[5] = std::min(s[5], x[5]); s[6] = std::max(s[6], x[6]);
        }
        for (int k = 0; k < 7; k++) stats[k] = s[k];
    }
    if (counters) {
        Counters c;
        for (auto& x : cnts) c.add(x);
        double v[11] = {c.node_tests, c.sphere_tests, c.quad_tests, c.plane_tests, c.material_fetches,
                        c.light_quad_evals, c.light_sphere_evals, c.bounces, c.diffuse_bounces, c.samples, c.rays};
        for (int k = 0; k < 11; k++) counters[k] = v[k];
    }
    return 0;
}

}  // namespace

extern "C" {

const char* or_last_error() { return g_err.c_str(); }

// Render a region with the oracle. real_kind 0 = ref (double scalars), 1 = fp32.
// stats[7] = {pixels, samples total, min, max, bounces total, min, max}
// counters[11] = {node_tests, sphere_tests, quad_tests, plane_tests, material_fetches,
//                 light_quad_evals, light_sphere_evals, bounces, diffuse_bounces, samples, rays}
// dims[4] = {width, height, bvh_depth, n_lights}
int or_render(const char* scene_json, const char* render_json, int rx, int ry, int rw, int rh, int row_step,
              int threads, int real_kind, float* radiance, uint8_t* rgb, int32_t* px_samples, int32_t* px_bounces,
              double* stats, double* counters, int* dims) {
    try {
        if (real_kind == 1)
            return render_impl<float>(scene_json, render_json, rx, ry, rw, rh, row_step, threads, radiance, rgb,
                                      px_samples, px_bounces, stats, counters, dims);
        return render_impl<double>(scene_json, render_json, rx, ry, rw, rh, row_step, threads, radiance, rgb,
                                   px_samples, px_bounces, stats, counters, dims);
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}

// Closest hit through the oracle's recursive BVH for a batch of rays (ref mode).
// out per ray: {hit, t, p.xyz, n.xyz, front, object_index}
int or_world_hit(const char* scene_json, int n, const float* orig, const float* dir, double tmin, double tmax,
                 double* out) {
    try {
        J sd = parse_json(scene_json);
        auto cam = std::make_unique<Camera<double>>();
        cam->load(sd, nullptr);
        for (int k = 0; k < n; k++) {
            Ray<double> r;
            for (int a = 0; a < 3; a++) { r.origin.v[a] = orig[k * 3 + a]; r.direction.v[a] = dir[k * 3 + a]; }
            HitRecord<double> rec;
            double* o = out + k * 10;
            bool h = cam->scene.world->hit(r, Interval<double>{tmin, tmax}, rec);
            o[0] = h;
            o[1] = h ? rec.t : 0;
            for (int a = 0; a < 3; a++) { o[2 + a] = h ? rec.p.v[a] : 0; o[5 + a] = h ? rec.normal.v[a] : 0; }
            o[8] = h ? rec.frontFace : 0;
            o[9] = -1;
            if (h) {
                for (size_t i = 0; i < cam->scene.objs.size(); i++) {
                    HitRecord<double> r2;
                    // identify by material pointer + t equality
                    if (cam->scene.objs[i]->hit(r, Interval<double>{tmin, tmax}, r2) && r2.t == rec.t &&
                        r2.material == rec.material) { o[9] = (double)i; break; }
                }
            }
        }
        return 0;
    } catch (const std::exception& e) { g_err = e.what(); return 1; }
}

// ---- Known-answer building blocks (ref mode) -------------------------------
static Vec3<double> V(const double* a) { return Vec3<double>::create(a[0], a[1], a[2]); }
static void put(double* o, const Vec3<double>& v) { o[0] = v.v[0]; o[1] = v.v[1]; o[2] = v.v[2]; }

// out: {hit, t, p.xyz, n.xyz, front}
int or_sphere_hit(const double* c, double r, const double* o, const double* d, double tmin, double tmax, double* out) {
    Sphere<double> s; Material<double> m; s.center = V(c); s.radius = r; s.material = &m; s.init();
    HitRecord<double> rec;
    bool h = s.hit_raw(Ray<double>{V(o), V(d)}, Interval<double>{tmin, tmax}, rec);
    out[0] = h; out[1] = h ? rec.t : 0; if (h) { put(out + 2, rec.p); put(out + 5, rec.normal); } out[8] = h ? rec.frontFace : 0;
    return h;
}
int or_quad_hit(const double* q, const double* u, const double* v, const double* o, const double* d, double tmin,
                double tmax, double* out) {
    Quad<double> s; Material<double> m; s.q = V(q); s.u = V(u); s.v = V(v); s.material = &m; s.init();
    HitRecord<double> rec;
    bool h = s.hit_raw(Ray<double>{V(o), V(d)}, Interval<double>{tmin, tmax}, rec);
    out[0] = h; out[1] = h ? rec.t : 0; if (h) { put(out + 2, rec.p); put(out + 5, rec.normal); } out[8] = h ? rec.frontFace : 0;
    return h;
}
// out: {hit, t, alpha, beta}
int or_plane_intersect(const double* q, const double* u, const double* v, const double* o, const double* d,
                       double tmin, double tmax, double* out) {
    Plane<double> p; Material<double> m; p.q = V(q); p.u = V(u); p.v = V(v); p.material = &m; p.init();
    double t = 0, a = 0, b = 0;
    bool h = p.intersect(Ray<double>{V(o), V(d)}, Interval<double>{tmin, tmax}, t, a, b);
    out[0] = h; out[1] = t; out[2] = a; out[3] = b;
    return h;
}
// box[6] of the primitive: kind 0 sphere(c,r), 1 quad(q,u,v), 2 plane(q,u,v)
int or_prim_box(int kind, const double* a, const double* b, const double* c, double r, double* box) {
    AABB<double> bx; Material<double> m;
    if (kind == 0) { Sphere<double> s; s.center = V(a); s.radius = r; s.material = &m; s.init(); bx = s.box; }
    else if (kind == 1) { Quad<double> s; s.q = V(a); s.u = V(b); s.v = V(c); s.material = &m; s.init(); bx = s.box; }
    else { Plane<double> s; s.q = V(a); s.u = V(b); s.v = V(c); s.material = &m; s.init(); bx = s.box; }
    put(box, bx.minimum); put(box + 3, bx.maximum);
    return 0;
}
int or_aabb_hit(const double* mn, const double* mx, const double* o, const double* d, double tmin, double tmax) {
    AABB<double> b{V(mn), V(mx)};
    return b.hit(Ray<double>{V(o), V(d)}, Interval<double>{tmin, tmax});
}
double or_quad_pdf_value(const double* q, const double* u, const double* v, const double* origin, const double* dir) {
    Quad<double> s; Material<double> m; s.q = V(q); s.u = V(u); s.v = V(v); s.material = &m; s.init();
    return s.pdfValue(V(origin), V(dir));
}
double or_quad_area(const double* u, const double* v) { return V(u).cross(V(v)).length(); }
double or_sphere_pdf_value(const double* c, double r, const double* origin, const double* dir) {
    Sphere<double> s; Material<double> m; s.center = V(c); s.radius = r; s.material = &m; s.init();
    return s.pdfValue(V(origin), V(dir));
}
double or_cosine_pdf_value(const double* n, const double* dir) { CosinePDF<double> p(V(n)); return p.value(V(dir)); }
double or_schlick(double cosine, double ratio) { return Dielectric<double>::reflectance(cosine, ratio); }
void or_reflect(const double* v, const double* n, double* out) { put(out, V(v).reflect(V(n))); }
void or_refract(const double* v, const double* n, double eta, double* out) { put(out, V(v).refract(V(n), eta)); }
void or_unit(const double* v, double* out) { put(out, V(v).unitVector()); }
double or_length(const double* v) { return V(v).length(); }
// ONBasis around n (src/geometry/onbasis.ts:18-51): out {u.xyz, v.xyz, w.xyz, local(a).xyz}
void or_onb(const double* n, const double* a, double* out) {
    ONB<double> b(V(n));
    put(out, b.u); put(out + 3, b.v); put(out + 6, b.w); put(out + 9, b.local(V(a)));
}
// The oracle's Math.cos / Math.sin of the cosine-PDF angle phi = 2 * PI * xi,
// xi = u / 2^32 (Vec3.randomCosineDirection, src/geometry/vec3.ts:325-337), and
// Schlick's Math.pow(xi, 5) (src/materials/dielectric.ts:98): for the V8 fixture
// (tests/golden/v8_math.npz, tests/test_v8_math.py).
void or_math_probe(int n, const uint32_t* u, double* out) {
    for (int k = 0; k < n; ++k) {
        const double xi = (double)u[k] * (1.0 / 4294967296.0);
        const double phi = 2 * M_PI * xi;
        out[3 * k] = R_cos<double>(phi);
        out[3 * k + 1] = R_sin<double>(phi);
        out[3 * k + 2] = R_pow5(xi);
    }
}
// Mixture value with fixed component values (tests/geometry/pdf.test.ts:126-156)
double or_mixture_value(int n, const double* values, const double* weights) {
    struct VP : PDF<double> { double x; double value(const Vec3<double>&) const override { return x; } Vec3<double> generate() const override { return Vec3<double>(); } };
    std::vector<VP> ps(n); std::vector<const PDF<double>*> pp; std::vector<double> ws;
    for (int i = 0; i < n; i++) { ps[i].x = values[i]; pp.push_back(&ps[i]); ws.push_back(weights[i]); }
    MixturePDF<double> m(pp, ws);
    return m.value(Vec3<double>());
}
// One Material.scatter + emitted per trial (src/materials/*.ts), at a hit at the
// origin with the given normal / front flag, incoming direction `din`. Trial k
// draws from Rng::for_path(seed, k, 0). out[k*12..]: {valid, hasScattered,
// reflected, attenuation.xyz, dir.xyz, emitted.xyz}; dir is the scattered ray's
// direction, or pdf.generate() for a PDF result (tests/materials/*.test.ts).
int or_material_probe(const char* material_json, const double* din, const double* normal, int front, uint32_t seed,
                      int n, double* out) {
    try {
        J md = parse_json(material_json);
        Scene<double> scene;
        const Material<double>* m = scene.create_material(&md);
        HitRecord<double> rec; rec.p = Vec3<double>::create(0, 0, 0); rec.normal = V(normal); rec.t = 1;
        rec.frontFace = front != 0; rec.material = m;
        Ray<double> rin{Vec3<double>::create(0, 0, 0).subtract(V(din)), V(din)};
        for (int k = 0; k < n; k++) {
            Rng rng = Rng::for_path(seed, (uint32_t)k, 0);
            g_rng = &rng;
            double* o = out + k * 12;
            ScatterResult<double> s = m->scatter(rin, rec);
            o[0] = s.valid; o[1] = s.hasScattered; o[2] = s.reflected;
            put(o + 3, s.valid ? s.attenuation : Vec3<double>());
            put(o + 6, !s.valid ? Vec3<double>() : s.hasScattered ? s.scattered.direction : s.pdf->generate());
            put(o + 9, m->emitted(rec));
            g_rng = nullptr;
        }
        return 0;
    } catch (const std::exception& e) { g_rng = nullptr; g_err = e.what(); return 1; }
}
// Camera.getRay(i, j) of sample n (src/camera.ts getRay), the RNG keyed as in a
// render (Rng::for_path(seed, j * W + i, n)): out[6] = {origin.xyz, direction.xyz}.
int or_get_ray(const char* scene_json, const char* render_json, int i, int j, int n, double* out) {
    try {
        J sd = parse_json(scene_json);
        J ro; bool has = render_json && render_json[0]; if (has) ro = parse_json(render_json);
        auto cam = std::make_unique<Camera<double>>();
        cam->load(sd, has ? &ro : nullptr);
        Rng rng = Rng::for_path(cam->seed, (uint32_t)j * (uint32_t)cam->W + (uint32_t)i, (uint32_t)n);
        g_rng = &rng;
        Ray<double> r = cam->getRay(i, j);
        g_rng = nullptr;
        put(out, r.origin); put(out + 3, r.direction);
        return 0;
    } catch (const std::exception& e) { g_rng = nullptr; g_err = e.what(); return 1; }
}
// RNG stream (for cross-checking the device RNG bit-for-bit)
void or_rng_stream(uint32_t seed, uint32_t pixel, uint32_t sample, int n, uint32_t* out) {
    Rng r = Rng::for_path(seed, pixel, sample);
    for (int i = 0; i < n; i++) out[i] = r.next_u32();
}
// Camera frame: {W, H, pixel00.xyz, du.xyz, dv.xyz, center.xyz}
int or_camera_info(const char* scene_json, const char* render_json, double* out) {
    try {
        J sd = parse_json(scene_json);
        J ro; bool has = render_json && render_json[0]; if (has) ro = parse_json(render_json);
        auto cam = std::make_unique<Camera<double>>();
        cam->load(sd, has ? &ro : nullptr);
        out[0] = cam->W; out[1] = cam->H;
        put(out + 2, cam->p00); put(out + 5, cam->du); put(out + 8, cam->dv); put(out + 11, cam->center);
        return 0;
    } catch (const std::exception& e) { g_err = e.what(); return 1; }
}

}  // extern "C"
