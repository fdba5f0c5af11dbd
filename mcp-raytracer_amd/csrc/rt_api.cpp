// C ABI of the path-tracing core (include/rt_amd.h).
//
// rt_camera = the reference's Camera object after createCameraFromSceneData:
// the host build (scene.cpp) plus lazily allocated device copies. Rendering
// follows Camera.renderRegion's contract: the caller owns the output buffer,
// only the region is written, RenderStats are returned.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <rccl/rccl.h>  // types and declarations only: librccl is dlopen'ed (Rccl below)

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/rt_amd.h"
#include "json.hpp"
#include "launch.hpp"
#include "scene.hpp"

using namespace rt;

// png.hip: the frame's PNG, encoded on the device queue `stream` (waited for).
std::vector<uint8_t> rt_png_encode_device(const uint8_t* d_rgb, int32_t w, int32_t h, hipStream_t stream);

static_assert(ST_WORDS == RT_STATS_WORDS, "rt_camera_stats_words layout");

#ifndef RT_BUILD_ID
#define RT_BUILD_ID "unhashed"
#endif

namespace {

thread_local std::string g_error;

// A/B switches for measurements: RT_AMD_LDS_SCENE=0 (no LDS-resident scene),
// RT_AMD_CHUNKED=0 (sequential-pixel kernel for fixed-spp renders).
bool env_flag(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    if (!e || !e[0]) return dflt;
    return e[0] != '0';
}
bool lds_scene_enabled() { return env_flag("RT_AMD_LDS_SCENE", true); }
int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return (e && e[0]) ? std::max(1, std::atoi(e)) : dflt;
}
// the same without the clamp to >= 1 (switches and counts where 0 means off)
int env_int0(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return (e && e[0]) ? std::atoi(e) : dflt;
}

int set_error(int code, const std::string& msg) {
    g_error = msg;
    return code;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

int device_cus(int dev) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    return cus;
}

// Pass sizing of the chunked / pool kernels. A pass hands out its items through one int32
// counter (take_pool), which may overshoot the item count by 2 x grid waves x pool before the
// last wave sees it exhausted: items must stay below kItemCap. A pass of `units` groups of
// `unit_slots` pixel slots numbers ceil64(units * unit_slots) x chunks_per_slot items
// (chunks_per_slot = the schedule's sum of nch: one item per (slot, chunk)). So each pass is
// the smallest of: the units left, the record budget, and the counter headroom - a larger
// record budget gives fewer, bounded passes instead of an error.
constexpr long kItemCap = (1l << 31) - (1l << 22);

long pass_units(long units_left, long unit_slots, long chunks_per_slot, size_t rec_bytes_per_unit, size_t budget) {
    const long by_budget = (long)(budget / std::max<size_t>(rec_bytes_per_unit, 1));
    const long by_items = (kItemCap - 1) / (std::max<long>(unit_slots, 1) * std::max<long>(chunks_per_slot, 1));
    return std::max<long>(1, std::min(units_left, std::min(by_budget, by_items)));
}

}  // namespace

// error hook for the other translation units of the library (image.cpp)
int rt_set_error_message(int code, const char* msg) { return set_error(code, msg ? msg : ""); }

// ONBasis of a hit normal (src/geometry/onbasis.ts:18-51), host side: the same
// rt_math.hpp operations as the kernel's make_onb, so the stored basis equals
// the one the kernel would build (ref: fp64 scalars, -ffp-contract=off).
template <class Real>
static RtOnb host_onb(V3 n) {
    const V3 w = unit<Real>(n);
    const V3 a = std::fabs((Real)w.x) > (Real)0.9 ? v3(0, 1, 0) : v3(1, 0, 0);
    const V3 v = unit<Real>(cross<Real>(w, a));
    const V3 u = cross<Real>(w, v);
    return RtOnb{{u.x, u.y, u.z, 0.f}, {v.x, v.y, v.z, 0.f}, {w.x, w.y, w.z, 0.f}};
}

// Per planar primitive slot: [precision ref, fp32][face front, back] bases of
// its hit normals (front: the plane normal; back: Vec3.negate of it). Covers
// slots [0, last planar slot]; empty when the scene has no quad or plane.
static std::vector<RtOnb> planar_onbs(const std::vector<RtPrim>& prims, int32_t* n_onb) {
    int32_t n = 0;
    for (size_t k = 0; k < prims.size(); ++k)
        if (prims[k].type != PRIM_SPHERE) n = (int32_t)k + 1;
    std::vector<RtOnb> t((size_t)n * 4, RtOnb{});
    for (int32_t k = 0; k < n; ++k) {
        if (prims[k].type == PRIM_SPHERE) continue;
        const V3 pn = v3(prims[k].g3[0], prims[k].g3[1], prims[k].g3[2]);
        t[k * 4 + 0] = host_onb<double>(pn);
        t[k * 4 + 1] = host_onb<double>(neg(pn));
        t[k * 4 + 2] = host_onb<float>(pn);
        t[k * 4 + 3] = host_onb<float>(neg(pn));
    }
    *n_onb = n;
    return t;
}

// The host half of a camera: the reference's Camera after createCameraFromSceneData
// (src/scenes/scenes.ts:60-104) - the flattened scene, options and mixture weights.
struct CamHost {
    SceneBuild build;
    int32_t precision = PREC_REF;
    int32_t traversal = TRAV_AUTO;
    double mix_total = 0.5, light_w = 0.0;

    // The strategy a launch actually uses: BRUTE/FAST are exact only where every
    // primitive lies inside its reference box (scene.cpp prims_inside_boxes).
    int effective_traversal(int trav) const {
        if (!build.fast_ok) return TRAV_REFERENCE;
        if (trav == TRAV_AUTO) return build.cam.n_prims <= kBruteMaxPrims ? TRAV_BRUTE : TRAV_FAST;
        return trav;
    }
};

// One device's copy of a camera: the scene blob in that device's HBM, its frame, record and
// stats buffers, events and (multi-GPU) its stream and tile-packed slabs. A camera keeps one
// per device it rendered on (rt_camera_render_multi: one per listed device entry), so moving
// between devices never re-uploads.
struct DevCtx {
    const CamHost& host;
    const SceneBuild& build;
    const int device;    // HIP device ordinal the buffers live on
    const int instance;  // >0: a further context on the same device (a device listed twice)
    bool live = false;   // scene uploaded, buffers allocated
    DevCtx(const CamHost& h, int dev, int inst) : host(h), build(h.build), device(dev), instance(inst) {}
    DevCtx(const DevCtx&) = delete;
    DevCtx& operator=(const DevCtx&) = delete;

    uint4* d_blob = nullptr;  // [tnodes][prims][mats][lights][nodes] (DevScene)
    int32_t lds_words = 0;    // [tnodes][tprims][tsph][prims] prefix, 16-byte words
    int32_t lds_words2 = 0;   // the same + [mats][lights]
    int32_t off_prims = 0, off_mats = 0, off_lights = 0, off_nodes = 0, off_tprims = 0, off_tsph = 0, off_onbs = 0;
    int32_t off_tsph2 = -1;  // leaf-order sphere records with the fp64 radius (RtLeafSph), or -1
    int32_t off_pre = 0, n_pre = 0, off_xrec = 0;
    int32_t n_onb = 0;
    int lds_max = 64 * 1024;  // dynamic LDS bytes a workgroup may use on this device
    // HIP events of the last launch, 3 per pass: path kernel start, path kernel
    // end, accumulate end (the sequential kernel: one pass, no accumulate)
    std::vector<hipEvent_t> ev;
    int n_passes = 0;
    bool ev_accum = false;
    int last_kernel = RT_KERNEL_NONE;
    unsigned long long* d_stats = nullptr;
    unsigned long long* d_counters = nullptr;
    unsigned int* d_tile = nullptr;
    uint8_t* d_rgb = nullptr;
    float* d_rad = nullptr;
    int cus = 256;

    // multi-GPU (rt_camera_render_multi): this context's stream, its tile-packed slabs, and on
    // the root context the gathered slabs of every device plus the stats words' host copy
    hipStream_t stream = nullptr;
    hipEvent_t ev_rendered = nullptr, ev_gather0 = nullptr, ev_gather1 = nullptr;
    uint8_t* d_slab = nullptr;
    float* d_rslab = nullptr;
    uint8_t* d_gather = nullptr;
    float* d_rgather = nullptr;
    size_t slab_cap = 0, rslab_cap = 0, gather_cap = 0, rgather_cap = 0;
    unsigned long long* h_words = nullptr;
    int h_words_cap = 0;

    ~DevCtx() {
        release();
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (void* p : {(void*)d_slab, (void*)d_rslab, (void*)d_gather, (void*)d_rgather})
            if (p) (void)hipFree(p);
        if (h_words) (void)hipHostFree(h_words);
        for (hipEvent_t e : {ev_rendered, ev_gather0, ev_gather1})
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
        (void)hipSetDevice(prev);
    }

    // multi-GPU buffers (grown on demand; the caller has made `device` current)
    template <class T>
    static T* grow(T* p, size_t& cap, size_t bytes, const char* what) {
        if (bytes <= cap && p) return p;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hip_check(hipMalloc(&p, std::max<size_t>(bytes, 16)), what);
        cap = bytes;
        return p;
    }
    void ensure_multi(size_t slab_bytes, size_t rslab_bytes, bool root, int n) {
        if (!stream) hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
        for (hipEvent_t* e : {&ev_rendered, &ev_gather0, &ev_gather1})
            if (!*e) hip_check(hipEventCreate(e), "hipEventCreate");
        d_slab = grow(d_slab, slab_cap, slab_bytes, "hipMalloc(slab)");
        if (rslab_bytes) d_rslab = grow(d_rslab, rslab_cap, rslab_bytes, "hipMalloc(radiance slab)");
        if (!root) return;
        d_gather = grow(d_gather, gather_cap, slab_bytes * n, "hipMalloc(gathered slabs)");
        if (rslab_bytes) d_rgather = grow(d_rgather, rgather_cap, rslab_bytes * n, "hipMalloc(gathered radiance)");
        if (h_words_cap < n) {
            if (h_words) (void)hipHostFree(h_words);
            h_words = nullptr;
            h_words_cap = 0;
            hip_check(hipHostMalloc((void**)&h_words, (size_t)n * ST_WORDS * sizeof(unsigned long long), 0),
                      "hipHostMalloc");
            h_words_cap = n;
        }
    }

    void release() {
        if (!live) return;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (void* p : {(void*)d_blob, (void*)d_stats, (void*)d_counters, (void*)d_tile, (void*)d_rgb, (void*)d_rad,
                        (void*)d_sbuf})
            if (p) (void)hipFree(p);
        // every freed pointer is reset: a later ensure_device / ensure_frame /
        // ensure_sbuf (possibly on another device) must reallocate all of them
        d_blob = nullptr;
        d_stats = nullptr;
        d_counters = nullptr;
        d_tile = nullptr;
        d_rgb = nullptr;
        d_rad = nullptr;
        d_sbuf = nullptr;
        sbuf_cap = 0;
        free_adapt_buffers();
        if (d_acount) (void)hipFree(d_acount);
        d_acount = nullptr;
        if (h_acount) (void)hipHostFree(h_acount);
        h_acount = nullptr;
        for (hipEvent_t& e : ev)
            if (e) (void)hipEventDestroy(e), e = nullptr;
        ev.clear();
        n_passes = 0;
        (void)hipSetDevice(prev);
        live = false;
    }

    // The RtExact records (scene.hpp) of a brute-force scene's primitives (empty above
    // kBruteMaxPrims: only closest_hit_brute_nf reads them)
    static std::vector<RtExact> exact_records(const std::vector<RtPrim>& prims) {
        std::vector<RtExact> out;
        if (prims.size() > (size_t)kBruteMaxPrims) return out;
        for (const RtPrim& p : prims) {
            RtExact x{};
            int32_t code = 0;
            std::memcpy(&code, &p.g4[3], sizeof code);
            x.s0 = p.s0;
            x.kind = PRE_OTHER;
            // the fp32 mode's radius / D is (float)s0; a primitive whose g0[3] is not (NaN
            // fields, say) keeps the RtPrim path
            const bool s0f_ok = (float)p.s0 == p.g0[3];
            if (p.type == PRIM_SPHERE && s0f_ok) {
                x.kind = PRE_SPHERE;
                for (int i = 0; i < 3; ++i) x.f[i] = p.g0[i];
            } else if (p.type == PRIM_QUAD && code >= 1 && code <= 6 && s0f_ok) {
                const int a = (code - 1) % 3, vflag = (code - 1) / 3;
                const int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
                if (p.g3[a] == 1.0f || p.g3[a] == -1.0f) {  // always so (a one-component unit normal)
                    x.kind = code | (p.g3[a] < 0.0f ? kExactNegNa : 0);
                    x.f[0] = p.g0[ia];
                    x.f[1] = p.g0[ib];
                    x.f[2] = p.g3[3];
                    x.f[3] = p.g2[3];
                    x.f[4] = p.g1[3];
                }
            }
            out.push_back(x);
        }
        return out;
    }

    // The RtPre records (scene.hpp) of the brute-force pre-filter pass, from the RtPrim fields:
    // spheres in pairs, axis-aligned quads in pairs of one axis code, the rest (an odd one out,
    // planar quads, planes) one per record. The pass sets each primitive's candidate bit and
    // bound by its slot, so the records' order is free; pairs come first. Sets *n_rec.
    static std::vector<RtPre> prefilter_records(const std::vector<RtPrim>& prims, int32_t* n_rec) {
        struct One {
            int kind;  // PRE_SPHERE, axis code 1..6, PRE_OTHER
            float f[6];
        };
        std::vector<RtPre> out;
        *n_rec = 0;
        if (prims.size() > (size_t)kBruteMaxPrims) {  // closest_hit_brute_nf runs up to kBruteMaxPrims
            out.resize(1);
            return out;
        }
        std::vector<One> one(prims.size());
        for (size_t k = 0; k < prims.size(); ++k) {
            const RtPrim& p = prims[k];
            One q{};
            int32_t code = 0;
            std::memcpy(&code, &p.g4[3], sizeof code);
            if (p.type == PRIM_SPHERE) {
                q.kind = PRE_SPHERE;
                for (int i = 0; i < 4; ++i) q.f[i] = p.g0[i];
            } else if (p.type == PRIM_QUAD && code >= 1 && code <= 6) {
                const int a = (code - 1) % 3, vflag = (code - 1) / 3;
                const int ia = vflag ? (a + 1) % 3 : (a + 2) % 3, ib = vflag ? (a + 2) % 3 : (a + 1) % 3;
                q.kind = code;
                const double asv = (double)p.g3[3] * (double)p.g2[3];  // w_a * v (alpha's factor)
                const double asu = (double)p.g3[3] * (double)p.g1[3];  // w_a * u (beta's factor)
                q.f[0] = (float)(p.s0 / (double)p.g3[a]);          // the plane x_a = D / n_a
                q.f[1] = (float)asv;
                q.f[2] = (float)asu;
                q.f[3] = (float)(-(double)p.g0[ia] * asv - 0.5);  // alpha - 1/2 at the quad's corner
                q.f[4] = (float)(-(double)p.g0[ib] * asu - 0.5);
                constexpr double kRelPre = 1e-5;  // pt_kernel.hpp kRel
                q.f[5] = (float)(kRelPre * std::max(std::fabs((double)p.g0[ia]), std::fabs((double)p.g0[ib])) * (1.0 + 1e-6));
            } else {
                q.kind = PRE_OTHER;
            }
            one[k] = q;
        }
        std::vector<bool> used(prims.size(), false);
        auto head = [](int kind, size_t k0, size_t k1) { return (int32_t)(kind | (int)k0 << 8 | (int)k1 << 16); };
        for (size_t k0 = 0; k0 < prims.size(); ++k0) {  // pairs of one kind (sphere / axis code)
            const int kind = one[k0].kind;
            if (used[k0] || kind == PRE_OTHER) continue;
            size_t k1 = k0 + 1;
            while (k1 < prims.size() && (used[k1] || one[k1].kind != kind)) ++k1;
            if (k1 == prims.size()) continue;
            used[k0] = used[k1] = true;
            const One &a = one[k0], &b = one[k1];
            RtPre r{};
            if (kind == PRE_SPHERE) {
                for (int i = 0; i < 4; ++i) {
                    r.f[2 * i] = a.f[i];
                    r.f[2 * i + 1] = b.f[i];
                }
                r.f[8] = a.f[3] * a.f[3];
                r.f[9] = b.f[3] * b.f[3];
                r.head = head(PRE_SPHERE2, k0, k1);
            } else {
                for (int i = 0; i < 5; ++i) {
                    r.f[2 * i] = a.f[i];
                    r.f[2 * i + 1] = b.f[i];
                }
                r.f[10] = -std::fabs(a.f[1]);
                r.f[11] = -std::fabs(b.f[1]);
                r.f[12] = -std::fabs(a.f[2]);
                r.f[13] = -std::fabs(b.f[2]);
                r.f[14] = std::max(a.f[5], b.f[5]);
                r.head = head(PRE_QUAD2 + kind, k0, k1);
            }
            out.push_back(r);
        }
        for (size_t k = 0; k < prims.size(); ++k) {  // the rest, one per record
            if (used[k]) continue;
            RtPre r{};
            for (int i = 0; i < 6; ++i) r.f[i] = one[k].f[i];
            r.head = head(one[k].kind, k, 0);
            out.push_back(r);
        }
        *n_rec = (int32_t)out.size();
        if (out.empty()) out.resize(1);  // 16-byte multiple, never empty
        return out;
    }

    template <class T>
    static void append(std::vector<char>& blob, const std::vector<T>& v, int32_t* off) {
        if ((v.size() * sizeof(T)) % 16) throw std::runtime_error("blob sections must be 16-byte multiples");
        if (off) *off = (int32_t)blob.size();
        const char* p = reinterpret_cast<const char*>(v.data());
        blob.insert(blob.end(), p, p + v.size() * sizeof(T));
    }

    // Uploads the scene on first use; the caller has made `device` current.
    void ensure_device() {
        int dev = 0;
        hip_check(hipGetDevice(&dev), "hipGetDevice");
        if (dev != device) throw std::logic_error("device context used on another device");
        if (live) return;
        std::vector<char> blob;
        append(blob, build.t4nodes, nullptr);  // the fast traversal's 4-wide tree heads the blob
        append(blob, build.tprims, &off_tprims);
        append(blob, build.tsph, &off_tsph);
        append(blob, build.prims, &off_prims);
        append(blob, exact_records(build.prims), &off_xrec);
        lds_words = (int32_t)(blob.size() / 16);
        append(blob, build.mats, &off_mats);
        append(blob, build.lights, &off_lights);
        const std::vector<RtOnb> onbs = planar_onbs(build.prims, &n_onb);
        append(blob, onbs, &off_onbs);
        lds_words2 = (int32_t)(blob.size() / 16);
        append(blob, build.nodes, &off_nodes);
        append(blob, prefilter_records(build.prims, &n_pre), &off_pre);
        off_tsph2 = -1;
        if (!build.tsph2.empty()) append(blob, build.tsph2, &off_tsph2);
        hip_check(hipMalloc(&d_blob, std::max<size_t>(blob.size(), 16)), "hipMalloc");
        if (!blob.empty()) hip_check(hipMemcpy(d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice), "hipMemcpy");
        hip_check(hipMalloc(&d_stats, ST_WORDS * kStatStride * sizeof(unsigned long long)), "hipMalloc");
        hip_check(hipMalloc(&d_counters, kCounterWords * sizeof(unsigned long long)), "hipMalloc");
        hip_check(hipMalloc(&d_tile, 64), "hipMalloc");
        live = true;
        cus = device_cus(dev);
        int smem = 0;
        if (hipDeviceGetAttribute(&smem, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && smem > 0)
            lds_max = smem;
    }

    void ensure_frame() {
        if (d_rgb) return;
        const size_t px = (size_t)build.cam.width * build.cam.height;
        hip_check(hipMalloc(&d_rgb, std::max<size_t>(px * 3, 1)), "hipMalloc");
        hip_check(hipMalloc(&d_rad, std::max<size_t>(px * 3, 1) * sizeof(float)), "hipMalloc");
    }

    // Events of pass p (created on demand on the camera's device).
    hipEvent_t pass_event(int p, int k) {
        while ((int)ev.size() < 3 * (p + 1)) {
            hipEvent_t e = nullptr;
            hip_check(hipEventCreate(&e), "hipEventCreate");
            ev.push_back(e);
        }
        return ev[3 * p + k];
    }

    // The strategy a launch actually uses: BRUTE/FAST are exact only where every
    // primitive lies inside its reference box (scene.cpp prims_inside_boxes).
    int effective_traversal(int trav) const { return host.effective_traversal(trav); }

    // Device time of the last launch from its events: path kernel(s) and accumulate passes,
    // summed per pass (never one span across both). Waits for those events.
    void times(float* path_ms, float* accum_ms) {
        *path_ms = 0.0f;
        *accum_ms = 0.0f;
        for (int p = 0; p < n_passes; ++p) {
            float a = 0.0f, b = 0.0f;
            hip_check(hipEventSynchronize(ev[3 * p + 1]), "hipEventSynchronize");
            hip_check(hipEventElapsedTime(&a, ev[3 * p], ev[3 * p + 1]), "hipEventElapsedTime");
            *path_ms += a;
            if (ev_accum) {
                hip_check(hipEventSynchronize(ev[3 * p + 2]), "hipEventSynchronize");
                hip_check(hipEventElapsedTime(&b, ev[3 * p + 1], ev[3 * p + 2]), "hipEventElapsedTime");
                *accum_ms += b;
            }
        }
    }

    DevScene dev_scene() const {
        DevScene S;
        const char* b = reinterpret_cast<const char*>(d_blob);
        S.tnodes = reinterpret_cast<const RtTNode*>(b);
        S.prims = reinterpret_cast<const RtPrim*>(b + off_prims);
        S.gprims = S.prims;
        S.gpre = reinterpret_cast<const RtPre*>(b + off_pre);
        S.n_pre = n_pre;
        S.xrec = reinterpret_cast<const RtExact*>(b + off_xrec);
        S.off_xrec = off_xrec;
        S.tprims = reinterpret_cast<const int32_t*>(b + off_tprims);
        S.off_tprims = off_tprims;
        S.tsph = reinterpret_cast<const float4*>(b + off_tsph);
        S.off_tsph = off_tsph;
        S.mats = reinterpret_cast<const RtMat*>(b + off_mats);
        S.lights = reinterpret_cast<const RtLight*>(b + off_lights);
        S.glights = S.lights;
        S.nodes = reinterpret_cast<const RtNode*>(b + off_nodes);
        S.onbs = reinterpret_cast<const RtOnb*>(b + off_onbs);
        S.n_onb = n_onb;
        S.off_onbs = off_onbs;
        S.blob = d_blob;
        S.tsph2 = nullptr;  // (set per launch: trees walked from global memory)
        S.lds_words = lds_words;
        S.off_prims = off_prims;
        S.off_mats = off_mats;
        S.off_lights = off_lights;
        S.lds_stack_bytes = 0;
        S.lds_pool_off = 0;
        S.lds_node_pad = 0;  // set per launch when the scene is LDS-resident
        S.t4_stride = (int32_t)sizeof(RtT4Node);
        S.n_top = 0;         // set per launch when the tree is walked from global memory
        S.top_lds = nullptr;
        S.nearfar = 0;       // (scene_view sets it per LDS level)
        S.troot = build.t4root;
        S.root_box = build.troot_box;
        S.cam = build.cam;
        S.mix_total = host.mix_total;
        S.light_w = host.light_w;
        return S;
    }

    // Launch one render; returns after queueing (and synchronising if asked).
    void launch(const rt_region& region, int tile_group, int tile_groups, int prec, int trav, int count,
                uint8_t* rgb, float* rad, int32_t* pxs, int32_t* pxb, int packed, hipStream_t stream) {
        const RtCamera& C = build.cam;
        if (tile_groups < 1 || tile_group < 0 || tile_group >= tile_groups)
            throw std::invalid_argument("tile_group must satisfy 0 <= tile_group < tile_groups");
        const int x0 = std::max(region.x, 0), y0 = std::max(region.y, 0);
        const int x1 = std::min(region.x + region.width, C.width);
        const int y1 = std::min(region.y + region.height, C.height);
        RtRegion reg{x0, y0, std::max(x1 - x0, 0), std::max(y1 - y0, 0), tile_group, tile_groups};
        const int tiles_x = (reg.width + kTile - 1) / kTile;
        const int tiles_y = (reg.height + kTile - 1) / kTile;
        const long total = (long)tiles_x * tiles_y;
        const long mine = total > tile_group ? (total - tile_group + tile_groups - 1) / tile_groups : 0;
        LaunchGeom g;
        g.tiles_x = std::max(tiles_x, 1);
        g.my_tiles = (int)mine;
        const long want = (mine + (kBlock / kWave) - 1) / (kBlock / kWave);
        g.grid = (int)std::max<long>(1, std::min<long>(want, (long)cus));  // one persistent workgroup per CU
        KernelVariant v{C.emissive_scatter != 0, count, effective_traversal(trav)};
        const size_t stack0 = stack_lds_bytes(C.stack_depth, v.trav, C.n_prims);        // tree in global memory
        const size_t stack1 = stack_lds_bytes(C.stack_depth, v.trav, C.n_prims, true);  // LDS-resident tree
        // LDS-resident scene: the BVH walk's data and the primitive records
        // (level 1), plus the material and light tables when they fit too
        // (level 2). The brute-force loop reads its wave-uniform primitive
        // records through scalar loads either way; LDS serves the per-lane
        // reads (hit record, materials, light sampling).
        const size_t lds_cap = (size_t)std::min(lds_max, kLdsSceneMaxBytes);
        // the LDS copy pads every 4-wide node to 144 bytes (pt_kernel.hpp t4_node: LDS bank windows)
        const int32_t node_pad =
            v.trav == TRAV_FAST && env_flag("RT_AMD_NODE_PAD", true) ? (int32_t)build.t4nodes.size() : 0;
        g.lds_level = 0;
        if (lds_scene_enabled() && v.trav != TRAV_REFERENCE) {
            if (stack1 + (size_t)(lds_words2 + node_pad) * 16 <= lds_cap && env_flag("RT_AMD_LDS_MATS", true))
                g.lds_level = 2;
            else if (v.trav == TRAV_FAST && stack1 + (size_t)(lds_words + node_pad) * 16 <= lds_cap)
                g.lds_level = 1;
        }
        // (16-bit stack entries hold node references < 2^15 and leaf codes ~(first << 3 | count) with
        // first < 2^12: always so for a tree that fits the LDS copy; checked)
        if (g.lds_level > 0 && v.trav == TRAV_FAST &&
            (build.t4nodes.size() >= (1u << 15) || build.tprims.size() >= (1u << 12)))
            g.lds_level = 0;
        const size_t stack = g.lds_level > 0 ? stack1 : stack0;
        g.lds_bytes = stack + (g.lds_level == 0 ? 0 : (size_t)((g.lds_level == 2 ? lds_words2 : lds_words) + node_pad) * 16);
        // a tree walked from global memory: its top (breadth-first prefix) in the LDS left beside the stack
        int32_t n_top = 0;
        // (round 5 also walked 8-bit quantised 64-byte nodes here, twice the nodes in the cache:
        // 2 % slower, the decode costing more than the halved loads; profiles/r05/qnodes/)
        const size_t node_lds = sizeof(RtT4Node) + 16;
        if (g.lds_level == 0 && v.trav == TRAV_FAST && lds_scene_enabled() && env_flag("RT_AMD_TOP_CACHE", true)) {
            const size_t room = lds_cap > stack ? lds_cap - stack : 0;
            n_top = (int32_t)std::min<size_t>(build.t4nodes.size(), room / node_lds);
            g.lds_bytes = stack + (size_t)n_top * node_lds;
        }
        // Deferred exact sphere tests pay where the walk is VALU-bound and leaves hold
        // several candidates: LDS-resident trees of >= 100 primitives (spheres-500
        // +4.7 %); tiny trees have ~1 candidate per ray (rain-50 -1.3 %) and trees
        // walked from global memory are bound by node fetches (spheres-100k -2.3 %;
        // profiles/r02/defer/). RT_AMD_DEFER=0/1 overrides.
        v.defer = v.trav == TRAV_FAST &&
                  env_flag("RT_AMD_DEFER", g.lds_level >= 1 && C.n_prims >= 100);
        if (g.lds_bytes + static_lds_bytes(count, false) > (size_t)lds_max)
            throw std::runtime_error("traversal stack exceeds the workgroup LDS (BVH too deep)");
        if (env_flag("RT_AMD_LAUNCH_LOG", false))
            std::fprintf(stderr,
                         "[rt launch] prims %d stack_depth %d trav %d lds_level %d lds %zu B (stack %zu, scene L1 %d / "
                         "L2 %d B) lds_max %d tiles %ld\n",
                         C.n_prims, C.stack_depth, v.trav, g.lds_level, g.lds_bytes, stack, lds_words * 16,
                         lds_words2 * 16, lds_max, mine);
        RenderOut out{rgb, rad, pxs, pxb, d_stats, d_counters, d_tile, packed ? 1 : 0};
        hip_check(launch_init_stats(d_stats, count ? d_counters : nullptr, d_tile, stream), "init_stats");
        n_passes = 0;
        last_kernel = RT_KERNEL_NONE;
        adapt_rounds = 0;
        adapt_rendered = 0;
        if (mine == 0) return;
        DevScene S = dev_scene();
        S.lds_stack_bytes = (int32_t)stack;
        S.lds_words = g.lds_level == 2 ? lds_words2 : lds_words;
        S.lds_node_pad = g.lds_level > 0 ? node_pad : 0;
        S.n_top = n_top;
        // trees walked from global memory: leaf records that carry the exact test's fp64 radius
        // (the LDSS-0 chunked kernels read them, pt_kernel.hpp leaf_test L2)
        S.tsph2 = off_tsph2 >= 0 ? reinterpret_cast<const RtLeafSph*>(reinterpret_cast<const char*>(d_blob) + off_tsph2)
                                 : nullptr;
        if (g.lds_level == 0 && v.trav == TRAV_FAST && !S.tsph2 && C.n_prims > 0)
            throw std::runtime_error("fast traversal without leaf records");
        // Fixed spp: the chunked / pool kernels (per-sample records, in-order accumulate)
        // at every size. Round 1 kept the sequential kernel for images of >= 4 tiles per
        // resident wave; with the hand-out rules above the chunked kernel is faster there
        // too (rain-50 1080p spp512: 50.7 -> 44.1 ms, profiles/r02/sched/), records and all.
        const bool chunked = env_flag("RT_AMD_CHUNKED", true);
        // Adaptive sampling runs in rounds on the chunked / pool kernels (pt_adapt_kernel
        // settles each round in sample order); RT_AMD_ADAPT_ROUNDS=0 keeps the sequential kernel.
        // Instrumented launches (count == 1) keep the sequential kernel: a round renders samples
        // past a pixel's convergence, and the work counters would count them.
        const bool rounds = C.adaptive && count != 1 && env_flag("RT_AMD_ADAPT_ROUNDS", true);
        if (C.n_samples <= 0 || !chunked || (C.adaptive && !rounds)) {
            // sequential-pixel kernel (pixelConverged needs each pixel's samples in one place)
            hip_check(hipEventRecord(pass_event(0, 0), stream), "hipEventRecord");
            hipError_t e = prec == PREC_FP32 ? launch_render_fp32(v, S, reg, out, g, nullptr, stream)
                                             : launch_render_ref(v, S, reg, out, g, nullptr, stream);
            hip_check(e, "pt_render_kernel launch");
            hip_check(hipEventRecord(pass_event(0, 1), stream), "hipEventRecord");
            n_passes = 1;
            ev_accum = false;
            last_kernel = RT_KERNEL_SEQUENTIAL;
            return;
        }
        SampleBuf sb{};

        // Stage-compacted pool kernel (pt_pool_kernel): possible for product brute-force
        // launches without an emission stack whose per-wave path pools fit in LDS beside
        // the scene; the default in both precisions since its diffuse and trace queues are
        // split by branch (Cornell 800^2 spp256 ref 16.82 ms vs chunked ~18.9 ms; fp32
        // 14.12 vs 14.23 ms, profiles/r02/asplit/). RT_AMD_POOL_KERNEL=0/1 overrides.
        S.lds_pool_off = (int32_t)((g.lds_bytes + 15) / 16 * 16);
        const bool pool_ok = !v.emit && (count == 0 || (RT_POOL_PROF && count == 2 && prec == PREC_REF)) && v.trav == TRAV_BRUTE && C.width < 65536 && C.height < 65536 &&
                 C.n_samples <= 65535 && C.depth <= 250 && build.mats.size() < (1u << 21) &&  // 56-byte slot fields
                 build.prims.size() < (1u << 14) &&
                 (size_t)S.lds_pool_off + pool_lds_bytes() + static_lds_bytes(count, true) <= (size_t)lds_max &&
                 env_flag("RT_AMD_POOL_KERNEL", true);
        // guided schedule of `nsamp` samples over `slots` pixel slots: half of the remaining
        // samples per phase, chunks halving. First-phase chunk from the samples per resident
        // lane: an item is the critical path of its pixel, so small per-launch workloads (a
        // rank's share of the image, small images) or a few very expensive pixels (rays
        // grazing a field of spheres) need short items, while large ones amortise the
        // hand-out over long items (tools/tail_probe.py sweep).
        auto schedule = [&](double slots, int nsamp) {
            v.pool = pool_ok;
            // spl: samples per resident lane of this launch.
            const double spl = slots * (double)nsamp / ((double)cus * kBlockChunk);
            // Brute-force scenes in the chunked kernel: two tile-chunks per atomic from 512 spl
            // and first items of spl / 8 (round 1, profiles/r01/sweep_b/).
            // The pool kernel (96 path slots per wave, any slot takes any item) wants wider takes
            // and shorter first items: 4 tile-chunks per atomic from 256 samples per resident
            // lane, 2 from 128, and first items of at most 8 samples (Cornell 800^2 spp256:
            // N=1 16.84 -> 16.63 ms, a rank's 1/2 share 9.18 -> 8.43 ms; tools/sched_sweep.py,
            // profiles/r02/sched/).
            // LDS-resident BVH scenes in the chunked kernel (resumable walks): 4 tile-chunks per
            // atomic from 256 samples per resident lane (2 below) and a first chunk of the
            // power-of-two floor of sqrt(spl) / 3 (spheres-500 800^2 spp64: N=1 6.62 -> 6.26 ms,
            // rank shares N=2 3.54 -> 3.27, N=4 2.04 -> 1.78, N=8 1.21 -> 1.03 ms; rain-50 1080p
            // spp512 rank shares N=2 31.5 -> 22.2 ms, N=8 7.8 -> 5.8 ms; profiles/r02/sched/).
            // Trees walked from global memory (a sample costs ~150 us of a lane at config 5) cap
            // the first chunk at 4 (config 5, 4096^2 spp1024: 9617 -> 8980 ms per frame; 2 since round 4).
            const bool bvh = v.trav == TRAV_FAST;
            // (pool kernel, re-tuned at 152 slots per wave: 8 tile-chunks per atomic from 512 spl,
            // 4 from 48, 2 from 24, first items of at most 4 samples - Cornell N=1 14.61 -> 14.43 ms,
            // 1/2 share 7.57 -> 7.40, 1/8 share 2.57 -> 2.10 ms; profiles/r02/sched/)
            // (trees walked from global memory, round 4: 8 tile-chunks per atomic from 1024 spl,
            // chunks of at most 2 samples and shading from 40 walks done, not 48 - config 5's 1/8
            // share 1070.8 -> 1045.0 ms, spheres-100k 4096^2 spp16 N=1 134.9 -> 131.4 ms;
            // profiles/r04/cfg5/)
            const bool gtree = bvh && g.lds_level == 0;
            const int pool_auto = v.pool ? (spl >= 512.0 ? 8 : spl >= 48.0 ? 4 : spl >= 24.0 ? 2 : 1)
                                 : bvh ? (gtree && spl >= 1024.0 ? 8 : spl >= 256.0 ? 4 : 2)
                                       : (v.trav == TRAV_BRUTE && spl >= 512.0 ? 2 : 1);
            sb.pool = kWave * env_int("RT_AMD_POOL", pool_auto);
            const int c_max = v.pool ? 4 : gtree ? 2 : 32;
            // (pool kernel, fixed spp, re-checked at the round-3 build: first items of spl / 64, so 4
            // samples for the whole frame and a 1/2 share, 2 for a 1/4 share, 1 for a 1/8 share -
            // Cornell 1/8 share 2.248 -> 2.051 ms, 1/4 3.998 -> 3.931 ms, N=1 and 1/2 unchanged;
            // profiles/r03/sched/. Adaptive rounds keep spl / 8.)
            const double c_target = bvh ? std::sqrt(spl) / 3.0 : (v.pool && !rounds) ? spl / 64.0 : spl / 8.0;
            int c_auto = 1;
            while (c_auto * 2 <= c_max && c_auto * 2 <= c_target) c_auto *= 2;  // pow2 floor, in [1, c_max]
            // power-of-two chunks: items are aligned to their chunk (the pool kernel derives an
            // item's end from its sample index)
            auto pow2floor = [](int x) { int p = 1; while (p * 2 <= x) p *= 2; return p; };
            int s0 = 0, c = pow2floor(std::min(env_int("RT_AMD_CHUNK", c_auto), std::max(1, nsamp / 2))), np = 0;
            if (!env_flag("RT_AMD_GUIDED", true)) {  // uniform chunks (A/B)
                c = pow2floor(std::max(1, std::min(env_int("RT_AMD_CHUNK", c_auto), nsamp)));
                const int full = nsamp / c;
                sb.s0[np] = 0; sb.chunk[np] = c; sb.nch[np] = full; ++np;
                s0 = full * c;
            }
            while (s0 < nsamp) {
                const int rem = nsamp - s0;
                if (c <= 1 || np == kMaxPhases - 1) {  // final phase: 1-sample items
                    sb.s0[np] = s0; sb.chunk[np] = 1; sb.nch[np] = rem;
                    ++np;
                    break;
                }
                const int span = (rem / 2) / c * c;
                if (span == 0) { c /= 2; continue; }
                sb.s0[np] = s0; sb.chunk[np] = c; sb.nch[np] = span / c;
                ++np;
                s0 += span;
                c /= 2;
            }
            sb.n_phases = np;
            // the pool kernel keeps log2(item chunk) in a 3-bit slot field (pool_meta): chunks
            // of more than kPoolMaxChunk samples (RT_AMD_CHUNK overrides) take the chunked kernel
            for (int p = 0; p < np; ++p)
                if (sb.chunk[p] > kPoolMaxChunk) v.pool = false;
            int covered = 0;
            for (int p = 0; p < np; ++p) {
                if (sb.s0[p] != covered) throw std::runtime_error("guided schedule: gap");
                covered += sb.chunk[p] * sb.nch[p];
            }
            if (covered != nsamp) throw std::runtime_error("guided schedule: coverage");
            for (int p = 0; p < np; ++p) sb.rnch[p] = 1.0 / (double)sb.nch[p];
            sb.refill_min = std::min(env_int("RT_AMD_REFILL", 4), kWave);
            sb.min_ready = std::min(env_int("RT_AMD_READY", gtree ? 40 : 48), kWave);
        };
        // one pass of the path kernel over sb.slots slots (items numbered phase by phase)
        int pass = 0;
        auto run_pass = [&](bool first) {
            // items come in (tile, chunk) groups of 64 (item_decode): a pass of an adaptive round
            // whose slot count is not a multiple of 64 still numbers whole groups (the slots past
            // sb.slots are skipped by slot_pixel)
            const long group_slots = ((long)sb.slots + kWave - 1) / kWave * kWave;
            long items = 0;
            for (int p = 0; p < sb.n_phases; ++p) {
                sb.item_base[p] = (int32_t)items;
                items += group_slots * sb.nch[p];
            }
            if (items >= kItemCap) throw std::runtime_error("chunked pass too large");  // pass_units keeps it below
            sb.n_items = (int32_t)items;
            if (!first) hip_check(hipMemsetAsync(d_tile, 0, 2 * sizeof(unsigned int), stream), "hipMemsetAsync");
            LaunchGeom gp = g;
            const int block = v.pool ? kBlockPool : kBlockChunk;
            gp.grid = (int)std::max<long>(1, std::min<long>(items / block + 1, (long)cus));
            DevScene Sp = S;
            if (v.pool) gp.lds_bytes = (size_t)S.lds_pool_off + pool_lds_bytes();
            // per-pass events: path kernel [0, 1), accumulate [1, 2)
            hip_check(hipEventRecord(pass_event(pass, 0), stream), "hipEventRecord");
            hipError_t e = prec == PREC_FP32 ? launch_render_fp32(v, Sp, reg, out, gp, &sb, stream)
                                             : launch_render_ref(v, Sp, reg, out, gp, &sb, stream);
            hip_check(e, "pt_chunk_kernel launch");
            hip_check(hipEventRecord(pass_event(pass, 1), stream), "hipEventRecord");
        };
        if (rounds) {
            launch_adaptive_rounds(S, reg, out, g, mine, sb, schedule, run_pass, pass, stream);
        } else {
            // fixed spp: passes over at most sbuf_budget bytes of per-sample records
            // 12-byte records where no pixel's bounce count is an output (SampleBuf::rec12)
            sb.rec12 = C.mode != MODE_BOUNCES && !out.px_bounces && env_flag("RT_AMD_REC12", true);
            const size_t rec_per_tile = (size_t)kWave * (size_t)C.n_samples * (sb.rec12 ? 12 : sizeof(float4));
            schedule((double)mine * kWave, C.n_samples);
            const long pass_tiles = pass_units(mine, kWave, chunks_per_slot(sb), rec_per_tile, sbuf_budget());
            ensure_sbuf((size_t)pass_tiles * rec_per_tile);
            sb.rec = d_sbuf;
            for (long t0 = 0; t0 < mine; t0 += pass_tiles, ++pass) {
                const long nt = std::min(pass_tiles, mine - t0);
                sb.tile0 = (int32_t)t0;
                sb.slots = (int32_t)(nt * kWave);
                // record layout: sample-major (default) or slot-major (RT_AMD_REC_SLOT_MAJOR=1, A/B)
                if (env_flag("RT_AMD_REC_SLOT_MAJOR", false)) {
                    sb.stride_s = 1;
                    sb.stride_slot = C.n_samples;
                } else {
                    sb.stride_s = sb.slots;
                    sb.stride_slot = 1;
                }
                run_pass(t0 == 0);
                hip_check(launch_accum(S, reg, out, g.tiles_x, sb, stream), "pt_accum_kernel launch");
                hip_check(hipEventRecord(pass_event(pass, 2), stream), "hipEventRecord");
            }
        }
        n_passes = pass;
        ev_accum = true;
        last_kernel = v.pool ? RT_KERNEL_POOL : RT_KERNEL_CHUNKED;
    }

    // Adaptive sampling in rounds (src/camera.ts:400-425). Round r renders samples
    // [s_base, s_base + len) of every pixel still sampling - speculatively, since a pixel
    // may converge inside the round - on the chunked / pool kernels; pt_adapt_kernel then
    // adds them to each pixel's running PixelStats in sample order with the reference's
    // convergence check after every sample, finishes converged / complete pixels and
    // compacts the rest into the next round's active list. Rounds double in length from
    // two convergence batches (aBatch) so a pixel renders at most one round past its
    // convergence; the pixel count of each round comes back to the host (one small copy).
    template <class Sched, class Pass>
    void launch_adaptive_rounds(DevScene& S, const RtRegion& reg, const RenderOut& out, const LaunchGeom& g, long mine,
                                SampleBuf& sb, Sched& schedule, Pass& run_pass, int& pass, hipStream_t stream) {
        const RtCamera& C = build.cam;
        const long slots_all = mine * kWave;
        ensure_adapt((size_t)slots_all);
        const double ab = C.a_batch;
        const int batch = (ab >= 1.0 && ab < 65536.0) ? (int)ab : std::max(1, std::min(C.n_samples, 16));
        // first round: one convergence batch, then rounds x3 (tools/adapt_sweep.py, 800^2 / 1080p,
        // profiles/r03/adapt_sweep.log: first 10 / 20 / 40 samples x growth 2 / 3 - one batch
        // wastes least on scenes whose sky converges at the first check (rain 2.59 vs 3.36 ms at
        // 20, spheres-500 5.87 vs 6.00 ms); Cornell, whose pixels converge at 10 or run to 256,
        // prefers few long rounds: 15.94 ms with growth 3 vs 16.35 with 2, 15.56 at first 40)
        int len = batch * std::max(1, (env_int("RT_AMD_ADAPT_FIRST", batch) + batch - 1) / batch);
        const int grow = env_int("RT_AMD_ADAPT_GROW", 3);
        // after a round that retired fewer than RT_AMD_ADAPT_JUMP per mille of its pixels, the rest
        // are taken to run long and the next round renders every remaining sample: Cornell (pixels
        // converge at the first check or run to spp) 15.17 -> 14.86 ms with 3 rounds; spheres-500 and
        // rain unchanged at 100; 200 cost rain 47 % (profiles/r03/exp2/)
        const int jump = env_int0("RT_AMD_ADAPT_JUMP", 100);
        // ... or after a round whose carried pixels are mostly not expected to converge within the
        // next (grown) round: fewer than RT_AMD_ADAPT_LIKELY per mille of them have a confidence
        // interval that would close by then at their current mean and variance (pt_adapt_kernel).
        // Cornell's pixels converge at the first checks or never: 474 of 530,755 carried after round
        // 1 are likely, so it runs in 2 rounds instead of 3 (14.79 -> 14.45 ms); rain's 20 % and
        // spheres-500's 11 % keep their rounds; the default scene 13.09 -> 12.96 ms path kernel
        // (profiles/r05/adaptive_likely/). 0 turns the rule off.
        const int likely_pm = env_int0("RT_AMD_ADAPT_LIKELY", 100);
        const bool trace = env_flag("RT_AMD_ADAPT_LOG", false);
        adapt_rounds = 0;
        adapt_rendered = 0;
        long n_act = slots_all;
        const int32_t* act = nullptr;  // round 0: every slot of the launch (invalid pixels skipped)
        int cur = 0;
        AdaptRound ar{};
        ar.state = d_astate;
        ar.next_count = d_acount;
        sb.stride_slot = 1;
        bool take_rest = false;
        for (int s_base = 0; n_act > 0 && s_base < C.n_samples; s_base += len, len = take_rest ? C.n_samples : len * grow) {
            len = std::min(len, C.n_samples - s_base);
            ++adapt_rounds;
            // round 0 numbers every slot of the launch's tiles; only the pixels inside the region render
            adapt_rendered += (unsigned long long)(act ? n_act : region_pixels(reg, mine)) * (unsigned long long)len;
            if (trace) std::fprintf(stderr, "[rt adaptive] round %d: samples [%d, %d) of %ld pixels\n", adapt_rounds,
                                    s_base, s_base + len, n_act);
            ar.len = len;
            ar.horizon = (int32_t)std::min<long>(C.n_samples, (long)s_base + len + (long)len * grow);
            ar.next_act = d_act[1 - cur];
            sb.s_base = s_base;
            sb.err_in_rec = 1;
            schedule((double)n_act, len);
            const size_t rec_per_slot = (size_t)len * sizeof(float4);
            // passes of whole 64-slot groups (items are numbered per group of 64 slots)
            const long pass_slots =
                kWave * pass_units((n_act + kWave - 1) / kWave, kWave, chunks_per_slot(sb), rec_per_slot * kWave, sbuf_budget());
            ensure_sbuf((size_t)pass_slots * rec_per_slot);
            sb.rec = d_sbuf;
            hip_check(hipMemsetAsync(d_acount, 0, 2 * sizeof(unsigned int), stream), "hipMemsetAsync");
            for (long a0 = 0; a0 < n_act; a0 += pass_slots, ++pass) {
                sb.slots = (int32_t)std::min<long>(pass_slots, n_act - a0);
                sb.stride_s = sb.slots;
                sb.act = act ? act + a0 : nullptr;
                sb.tile0 = act ? 0 : (int32_t)(a0 / kWave);
                run_pass(pass == 0);
                hip_check(launch_adapt(S, reg, out, g.tiles_x, sb, ar, stream), "pt_adapt_kernel launch");
                hip_check(hipEventRecord(pass_event(pass, 2), stream), "hipEventRecord");
            }
            hip_check(hipMemcpyAsync(h_acount, d_acount, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost, stream),
                      "hipMemcpyAsync");
            hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
            const long n_prev = n_act;
            n_act = (long)h_acount[0];
            const long n_likely = (long)h_acount[1];
            if (trace)
                std::fprintf(stderr, "[rt adaptive]   %ld carried, %ld likely to converge by sample %d\n", n_act, n_likely,
                             ar.horizon);
            act = d_act[1 - cur];
            cur = 1 - cur;
            take_rest = jump > 0 && n_act > 0 &&
                        ((double)(n_prev - n_act) < (double)jump * 1e-3 * (double)n_prev ||
                         (likely_pm > 0 && (double)n_likely < (double)likely_pm * 1e-3 * (double)n_act));
        }
    }

    // Pixels inside the region among the `mine` tiles this launch owns (tile t of the region is
    // owned iff t % tile_groups == tile_group, as the kernels' item_pixel maps them).
    static long region_pixels(const RtRegion& reg, long mine) {
        const int tiles_x = std::max((reg.width + kTile - 1) / kTile, 1);
        long n = 0;
        for (long k = 0; k < mine; ++k) {
            const long t = reg.tile_group + k * reg.tile_groups;
            const int tx = (int)(t % tiles_x), ty = (int)(t / tiles_x);
            n += (long)std::min(kTile, reg.width - tx * kTile) * std::min(kTile, reg.height - ty * kTile);
        }
        return n;
    }

    int adapt_rounds = 0;                   // rounds of the last adaptive render
    unsigned long long adapt_rendered = 0;  // samples its rounds rendered (>= the samples kept)
    // Adaptive rounds: per-slot running PixelStats, two active lists, the list counter.
    AdaptPix* d_astate = nullptr;
    int32_t* d_act[2] = {nullptr, nullptr};
    unsigned int* d_acount = nullptr;
    unsigned int* h_acount = nullptr;
    size_t adapt_cap = 0;
    void ensure_adapt(size_t slots) {
        if (!h_acount) hip_check(hipHostMalloc((void**)&h_acount, 2 * sizeof(unsigned int), 0), "hipHostMalloc");
        if (!d_acount) hip_check(hipMalloc(&d_acount, 2 * sizeof(unsigned int)), "hipMalloc");
        if (slots <= adapt_cap) return;
        free_adapt_buffers();
        hip_check(hipMalloc(&d_astate, slots * sizeof(AdaptPix)), "hipMalloc(adaptive state)");
        hip_check(hipMalloc(&d_act[0], slots * sizeof(int32_t)), "hipMalloc(active list)");
        hip_check(hipMalloc(&d_act[1], slots * sizeof(int32_t)), "hipMalloc(active list)");
        adapt_cap = slots;
    }
    void free_adapt_buffers() {
        for (void* p : {(void*)d_astate, (void*)d_act[0], (void*)d_act[1]})
            if (p) (void)hipFree(p);
        d_astate = nullptr;
        d_act[0] = d_act[1] = nullptr;
        adapt_cap = 0;
    }

    // Per-sample record buffer of the chunked kernel (grown on demand, kept).
    float4* d_sbuf = nullptr;
    size_t sbuf_cap = 0;
    void ensure_sbuf(size_t bytes) {
        if (bytes <= sbuf_cap) return;
        if (d_sbuf) (void)hipFree(d_sbuf);
        d_sbuf = nullptr;
        sbuf_cap = 0;
        hip_check(hipMalloc(&d_sbuf, bytes), "hipMalloc(sample buffer)");
        sbuf_cap = bytes;
    }
    static long chunks_per_slot(const SampleBuf& sb) {
        long n = 0;
        for (int p = 0; p < sb.n_phases; ++p) n += sb.nch[p];
        return n;
    }
    static size_t sbuf_budget() {
        const char* e = std::getenv("RT_AMD_SBUF_MB");
        const long mb = e ? std::atol(e) : 8192;
        return (size_t)std::max<long>(mb, 1) << 20;
    }

    void read_stats(rt_render_stats* st, uint64_t* counters, hipStream_t stream) {
        unsigned long long wl[ST_WORDS * kStatStride], w[ST_WORDS];
        hip_check(hipMemcpyAsync(wl, d_stats, sizeof wl, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
        unsigned long long c[kCounterWords];
        if (counters)
            hip_check(hipMemcpyAsync(c, d_counters, sizeof c, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        for (int k = 0; k < ST_WORDS; ++k) w[k] = wl[k * kStatStride];
        if (counters)
            for (int k = 0; k < kCounterWords; ++k) counters[k] = c[k];
        stats_from_words(w, st);
    }

    // RenderStats from the 8 stats words; the reference's thrown Errors for the error flags.
    static void stats_from_words(const unsigned long long* w, rt_render_stats* st) {
        if (w[ST_ERROR] & ERR_NO_BACKGROUND)
            throw std::runtime_error("Cannot read properties of undefined (reading 'top')");
        if (w[ST_ERROR] & ERR_EMIT_STACK)
            throw std::runtime_error("emission stack overflow: depth exceeds the emissive-scatter limit (128)");
        if (!st) return;
        st->pixels = (double)w[ST_PIXELS];
        st->samples_total = (double)w[ST_SAMPLES];
        st->samples_min = w[ST_SMIN] == ~0ull ? INFINITY : (double)w[ST_SMIN];
        st->samples_max = (double)w[ST_SMAX];
        st->samples_avg = st->pixels > 0 ? st->samples_total / st->pixels : 0.0;
        st->bounces_total = (double)w[ST_BOUNCES];
        st->bounces_min = w[ST_BMIN] == ~0ull ? INFINITY : (double)w[ST_BMIN];
        st->bounces_max = (double)w[ST_BMAX];
        st->bounces_avg = st->samples_total > 0 ? st->bounces_total / st->samples_total : 0.0;
    }
};

// RenderStats.merge (src/render-utils/renderStats.ts:42-64) over the stats words of n
// renders (row r at words + r * ST_WORDS): totals summed, minima / maxima over the renders
// (~0 = no sample: skipped by the unsigned minimum), error flags or'ed.
static void merge_stats_words(const unsigned long long* words, int n, unsigned long long* m) {
    m[ST_PIXELS] = m[ST_SAMPLES] = m[ST_BOUNCES] = m[ST_SMAX] = m[ST_BMAX] = m[ST_ERROR] = 0;
    m[ST_SMIN] = m[ST_BMIN] = ~0ull;
    for (int r = 0; r < n; ++r) {
        const unsigned long long* w = words + (size_t)r * ST_WORDS;
        m[ST_PIXELS] += w[ST_PIXELS];
        m[ST_SAMPLES] += w[ST_SAMPLES];
        m[ST_BOUNCES] += w[ST_BOUNCES];
        m[ST_SMIN] = std::min(m[ST_SMIN], w[ST_SMIN]);
        m[ST_BMIN] = std::min(m[ST_BMIN], w[ST_BMIN]);
        m[ST_SMAX] = std::max(m[ST_SMAX], w[ST_SMAX]);
        m[ST_BMAX] = std::max(m[ST_BMAX], w[ST_BMAX]);
        m[ST_ERROR] |= w[ST_ERROR];
    }
}

// The multi-GPU split of a region: its 8x8 tiles dealt round-robin over n
// devices (tile t -> entry t % n), each device's tiles packed into an equal-size slab padded
// to the largest share, plus one spare tile whose first 64 bytes carry the device's stats
// words (the gather brings them along; rt_tiles_unpack never reads that tile).
static rt_multi_plan make_multi_plan(const rt_region& region, int width, int height, int n) {
    rt_multi_plan p{};
    const int x0 = std::max(region.x, 0), y0 = std::max(region.y, 0);
    const int x1 = std::min(region.x + region.width, width), y1 = std::min(region.y + region.height, height);
    p.region = rt_region{x0, y0, std::max(x1 - x0, 0), std::max(y1 - y0, 0)};
    p.n_devices = n;
    p.tiles = (int64_t)((p.region.width + kTile - 1) / kTile) * ((p.region.height + kTile - 1) / kTile);
    p.slab_tiles = (int32_t)((p.tiles + n - 1) / n);
    p.slab_bytes_rgb = (int64_t)(p.slab_tiles + 1) * kWave * 3;
    p.slab_bytes_radiance = (int64_t)p.slab_tiles * kWave * 3 * (int64_t)sizeof(float);
    p.stats_offset = (int64_t)p.slab_tiles * kWave * 3;
    for (int g = 0; g < n && g < RT_MAX_DEVICES; ++g)
        p.group_tiles[g] = (int32_t)(p.tiles > g ? (p.tiles - g + n - 1) / n : 0);
    return p;
}

// RCCL, loaded at the first multi-GPU gather (dlopen: a process that already holds PyTorch's
// librccl.so.1 shares it; a Node host loads ROCm's). Single-process communicators over the
// listed devices (ncclCommInitAll), cached per device list for the life of the process.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::mutex mu;  // one gather at a time per process (a communicator is not re-entrant)
    std::vector<std::pair<std::vector<int>, std::vector<ncclComm_t>>> comms;

    void check(ncclResult_t r, const char* what) {
        if (r != ncclSuccess) throw HipError(std::string(what) + ": " + (error_string ? error_string(r) : "RCCL error"));
    }
    const std::vector<ncclComm_t>& comms_for(const std::vector<int>& devs) {
        for (auto& c : comms)
            if (c.first == devs) return c.second;
        std::vector<ncclComm_t> cs(devs.size(), nullptr);
        check(comm_init_all(cs.data(), (int)devs.size(), devs.data()), "ncclCommInitAll");
        comms.emplace_back(devs, std::move(cs));
        return comms.back().second;
    }
};

static Rccl& rccl() {
    static std::mutex load_mu;
    static Rccl* lib = nullptr;
    static std::string load_error;
    std::lock_guard<std::mutex> lock(load_mu);
    if (lib) return *lib;
    if (!load_error.empty()) throw HipError(load_error);
    const char* env = std::getenv("RT_AMD_RCCL_LIB");
    void* h = nullptr;
    for (const char* name : {env && env[0] ? env : "librccl.so.1", "librccl.so"})
        if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
        load_error = std::string("RCCL not loadable (librccl.so.1): ") + dlerror() +
                     " - set RT_AMD_GATHER=peer for device-to-device copies";
        throw HipError(load_error);
    }
    auto* r = new Rccl();
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) load_error = std::string("RCCL symbol missing: ") + name;
    };
    sym(r->comm_init_all, "ncclCommInitAll");
    sym(r->group_start, "ncclGroupStart");
    sym(r->group_end, "ncclGroupEnd");
    sym(r->send, "ncclSend");
    sym(r->recv, "ncclRecv");
    sym(r->error_string, "ncclGetErrorString");
    if (!load_error.empty()) {
        delete r;
        throw HipError(load_error);
    }
    lib = r;
    return *lib;
}

struct rt_camera : CamHost {
    std::mutex mu;
    std::vector<std::unique_ptr<DevCtx>> ctxs;
    DevCtx* last = nullptr;  // the context of the most recent render (queries read it)
    // the most recent rt_camera_render_multi: its device contexts, transport and plan
    std::vector<DevCtx*> multi;
    int multi_transport = -1;
    rt_multi_plan multi_plan{};

    DevCtx& ctx(int dev, int inst = 0) {
        for (auto& c : ctxs)
            if (c->device == dev && c->instance == inst) return *c;
        ctxs.emplace_back(new DevCtx(*this, dev, inst));
        return *ctxs.back();
    }
    // the context of the calling thread's current HIP device
    DevCtx& current() {
        int dev = 0;
        hip_check(hipGetDevice(&dev), "hipGetDevice");
        return ctx(dev, 0);
    }
    void release() {
        multi.clear();
        last = nullptr;
        ctxs.clear();
    }
};

// The current HIP device of the calling thread, restored when the scope ends.
struct DeviceScope {
    int prev = 0;
    DeviceScope() { (void)hipGetDevice(&prev); }
    ~DeviceScope() { (void)hipSetDevice(prev); }
};

// Single-process multi-GPU render (rt_camera_render_multi). Entry g of `devs` renders tile
// group g of n into its context's tile-packed slab on its own stream (one host thread per entry,
// so renders that wait on the host between rounds - adaptive sampling - still overlap); the
// slabs are gathered on devs[0] (RCCL send / recv in one group over xGMI, or device-to-device
// copies), unpacked into devs[0]'s full frame (rt_tiles_unpack) and the stats words merged as
// RenderStats.merge does (the reference's workers: src/raytracer.ts:60-90, 185-205;
// src/render-utils/renderWorker.ts:17-35). Returns the root context with the frame in
// d_rgb / d_rad: `outputs` queues the caller's copies on its stream before the one host
// sync, after which *merged holds the merged stats words.
static DevCtx& render_multi(rt_camera* cam, const int32_t* devices, int n, const rt_region& region, bool want_rgb,
                            bool want_rad, unsigned long long* merged, const std::function<void(DevCtx&)>& outputs) {
    int count = 0;
    hip_check(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if (n < 1 || n > RT_MAX_DEVICES || !devices)
        throw std::invalid_argument("rt_camera_render_multi: 1 <= n_devices <= RT_MAX_DEVICES devices are required");
    std::vector<int> devs(devices, devices + n);
    bool distinct = true;
    for (int g = 0; g < n; ++g) {
        if (devs[g] < 0 || devs[g] >= count)
            throw std::invalid_argument("rt_camera_render_multi: device " + std::to_string(devs[g]) + " is not visible (" +
                                        std::to_string(count) + " devices)");
        for (int h = 0; h < g; ++h) distinct = distinct && devs[h] != devs[g];
    }
    // transport: RCCL over xGMI when every entry is its own device, else device-to-device
    // copies (a device listed twice: the split rehearsed on fewer GPUs; RCCL refuses that)
    const char* ge = std::getenv("RT_AMD_GATHER");
    const std::string gs = ge ? ge : "";
    int transport = distinct ? RT_GATHER_RCCL : RT_GATHER_PEER;
    if (gs == "peer") transport = RT_GATHER_PEER;
    else if (gs == "rccl") transport = RT_GATHER_RCCL;
    else if (!gs.empty()) throw std::invalid_argument("RT_AMD_GATHER must be 'rccl' or 'peer'");
    if (transport == RT_GATHER_RCCL && !distinct)
        throw std::invalid_argument("rt_camera_render_multi: RCCL needs distinct devices (RT_AMD_GATHER=peer allows repeats)");

    const RtCamera& C = cam->build.cam;
    const rt_multi_plan plan = make_multi_plan(region, C.width, C.height, n);
    std::vector<DevCtx*> cs(n);
    for (int g = 0; g < n; ++g) {
        int inst = 0;
        for (int h = 0; h < g; ++h) inst += devs[h] == devs[g];
        cs[g] = &cam->ctx(devs[g], inst);
    }
    cam->multi = cs;
    cam->multi_transport = transport;
    cam->multi_plan = plan;
    const size_t slab_b = (size_t)plan.slab_bytes_rgb, rslab_b = want_rad ? (size_t)plan.slab_bytes_radiance : 0;
    DeviceScope scope;

    // renders: one host thread per further entry, entry 0 on the calling thread
    std::vector<std::exception_ptr> errs(n);
    auto work = [&](int g) {
        try {
            DevCtx& c = *cs[g];
            hip_check(hipSetDevice(c.device), "hipSetDevice");
            c.ensure_device();
            c.ensure_multi(slab_b, rslab_b, g == 0, n);
            if (g == 0) c.ensure_frame();
            c.launch(plan.region, g, n, cam->precision, cam->traversal, 0, c.d_slab, want_rad ? c.d_rslab : nullptr,
                     nullptr, nullptr, 1, c.stream);
            // the stats words into the slab's spare tile (rides in the gather)
            hip_check(hipMemcpy2DAsync(c.d_slab + plan.stats_offset, sizeof(unsigned long long), c.d_stats,
                                       kStatStride * sizeof(unsigned long long), sizeof(unsigned long long), ST_WORDS,
                                       hipMemcpyDeviceToDevice, c.stream),
                      "hipMemcpy2DAsync(stats)");
            hip_check(hipEventRecord(c.ev_rendered, c.stream), "hipEventRecord");
        } catch (...) {
            errs[g] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int g = 1; g < n; ++g) th.emplace_back(work, g);
    work(0);
    for (auto& t : th) t.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);

    DevCtx& root = *cs[0];
    hip_check(hipSetDevice(root.device), "hipSetDevice");
    hip_check(hipEventRecord(root.ev_gather0, root.stream), "hipEventRecord");
    if (transport == RT_GATHER_RCCL) {
        Rccl& r = rccl();
        std::lock_guard<std::mutex> lock(r.mu);
        const std::vector<ncclComm_t>& comms = r.comms_for(devs);
        // one group: entry g sends its slab(s) to rank 0, rank 0 receives slab g into row g
        // (rank 0's own slab included: a send / recv pair to itself)
        r.check(r.group_start(), "ncclGroupStart");
        for (int g = 0; g < n; ++g) {
            r.check(r.send(cs[g]->d_slab, slab_b, ncclUint8, 0, comms[g], cs[g]->stream), "ncclSend");
            if (want_rad) r.check(r.send(cs[g]->d_rslab, rslab_b / sizeof(float), ncclFloat32, 0, comms[g], cs[g]->stream),
                                  "ncclSend");
        }
        for (int g = 0; g < n; ++g) {
            r.check(r.recv(root.d_gather + (size_t)g * slab_b, slab_b, ncclUint8, g, comms[0], root.stream), "ncclRecv");
            if (want_rad)
                r.check(r.recv(root.d_rgather + (size_t)g * (rslab_b / sizeof(float)), rslab_b / sizeof(float),
                               ncclFloat32, g, comms[0], root.stream),
                        "ncclRecv");
        }
        r.check(r.group_end(), "ncclGroupEnd");
    } else {
        for (int g = 0; g < n; ++g) {
            hip_check(hipStreamWaitEvent(root.stream, cs[g]->ev_rendered, 0), "hipStreamWaitEvent");
            hip_check(hipMemcpyPeerAsync(root.d_gather + (size_t)g * slab_b, root.device, cs[g]->d_slab, cs[g]->device,
                                         slab_b, root.stream),
                      "hipMemcpyPeerAsync");
            if (want_rad)
                hip_check(hipMemcpyPeerAsync(root.d_rgather + (size_t)g * (rslab_b / sizeof(float)), root.device,
                                             cs[g]->d_rslab, cs[g]->device, rslab_b, root.stream),
                          "hipMemcpyPeerAsync");
        }
        // an entry's next render must not overwrite its slab before this copy has read it
        hip_check(hipEventRecord(root.ev_rendered, root.stream), "hipEventRecord");
        for (int g = 1; g < n; ++g) {
            hip_check(hipSetDevice(cs[g]->device), "hipSetDevice");
            hip_check(hipStreamWaitEvent(cs[g]->stream, root.ev_rendered, 0), "hipStreamWaitEvent");
        }
        hip_check(hipSetDevice(root.device), "hipSetDevice");
    }
    const RtRegion reg{plan.region.x, plan.region.y, plan.region.width, plan.region.height, 0, 1};
    if (want_rgb)
        hip_check(launch_tiles_unpack(root.d_gather, n, plan.slab_tiles + 1, reg, C.width, 3, 1, root.d_rgb, root.stream),
                  "tiles_unpack_kernel");
    if (want_rad)
        hip_check(launch_tiles_unpack(root.d_rgather, n, plan.slab_tiles, reg, C.width, 3, 4, root.d_rad, root.stream),
                  "tiles_unpack_kernel");
    hip_check(hipMemcpy2DAsync(root.h_words, ST_WORDS * sizeof(unsigned long long), root.d_gather + plan.stats_offset, slab_b,
                               ST_WORDS * sizeof(unsigned long long), n, hipMemcpyDeviceToHost, root.stream),
              "hipMemcpy2DAsync(stats words)");
    hip_check(hipEventRecord(root.ev_gather1, root.stream), "hipEventRecord");
    if (outputs) outputs(root);  // the caller's copies / encode, queued before the one sync
    hip_check(hipStreamSynchronize(root.stream), "hipStreamSynchronize");
    merge_stats_words(root.h_words, n, merged);
    cam->last = &root;
    return root;
}

// Queues the copy of a region's rows of the context's full frame into the caller's host
// buffers (full-frame layout: only the region is written, as Camera.renderRegion does).
static void copy_region_to_host(DevCtx& c, const rt_region& region, uint8_t* rgb, float* radiance, hipStream_t stream) {
    const RtCamera& C = c.build.cam;
    const int x0 = std::max(region.x, 0), y0 = std::max(region.y, 0);
    const int x1 = std::min(region.x + region.width, C.width);
    const int y1 = std::min(region.y + region.height, C.height);
    if (x1 <= x0 || y1 <= y0) return;
    const size_t pitch = (size_t)C.width * 3;
    const size_t off = ((size_t)y0 * C.width + x0) * 3;
    const size_t w = (size_t)(x1 - x0) * 3;
    if (rgb)
        hip_check(hipMemcpy2DAsync(rgb + off, pitch, c.d_rgb + off, pitch, w, y1 - y0, hipMemcpyDeviceToHost, stream),
                  "hipMemcpy2DAsync");
    if (radiance)
        hip_check(hipMemcpy2DAsync(radiance + off, pitch * sizeof(float), c.d_rad + off, pitch * sizeof(float),
                                   w * sizeof(float), y1 - y0, hipMemcpyDeviceToHost, stream),
                  "hipMemcpy2DAsync");
}

// The frame's PNG: encoded on the device from the context's u8 frame (png.hip), malloc'ed.
static void png_out(DevCtx& c, hipStream_t stream, uint8_t** out, size_t* out_len) {
    const RtCamera& C = c.build.cam;
    const std::vector<uint8_t> png = rt_png_encode_device(c.d_rgb, C.width, C.height, stream);
    uint8_t* b = (uint8_t*)std::malloc(png.size());
    if (!b) throw std::runtime_error("out of memory");
    std::memcpy(b, png.data(), png.size());
    *out = b;
    *out_len = png.size();
}

extern "C" {

int rt_version(void) { return RT_AMD_VERSION; }

const char* rt_last_error(void) { return g_error.c_str(); }

void rt_free(void* p) { std::free(p); }

int rt_generate_scene_data(const char* type, const char* options_json, char** out_json) {
    try {
        if (!type || !out_json) return set_error(RT_ERR_INVALID, "type and out_json are required");
        rtj::Value opts;
        const rtj::Value* optp = nullptr;
        if (options_json && options_json[0]) {
            opts = rtj::parse(options_json, std::strlen(options_json));
            if (!opts.is_null()) optp = &opts;
        }
        const std::string s = rtj::dump(generate_scene_data(type, optp));
        char* buf = (char*)std::malloc(s.size() + 1);
        if (!buf) return set_error(RT_ERR_INVALID, "out of memory");
        std::memcpy(buf, s.c_str(), s.size() + 1);
        *out_json = buf;
        return RT_OK;
    } catch (const std::exception& e) {
        return set_error(RT_ERR_INVALID, e.what());
    }
}

int rt_camera_create(const char* scene_json, const char* render_options_json, rt_camera** out) {
    try {
        if (!scene_json || !out) return set_error(RT_ERR_INVALID, "scene_json and out are required");
        const rtj::Value scene = rtj::parse(scene_json, std::strlen(scene_json));
        rtj::Value ro;
        const rtj::Value* rop = nullptr;
        if (render_options_json && render_options_json[0]) {
            ro = rtj::parse(render_options_json, std::strlen(render_options_json));
            if (!ro.is_null()) rop = &ro;
        }
        auto* cam = new rt_camera();
        try {
            cam->build = build_scene(scene, rop);
            int32_t prec = PREC_REF;
            auto pick = [&](const rtj::Value* v) {
                if (v && v->is_string()) {
                    if (v->str == "fp32") prec = PREC_FP32;
                    else if (v->str == "ref") prec = PREC_REF;
                    else throw std::runtime_error("precision must be 'ref' or 'fp32'");
                }
            };
            if (const rtj::Value* r = scene.get("render")) pick(r->get("precision"));
            if (rop) pick(rop->get("precision"));
            cam->precision = prec;
            int32_t trav = TRAV_AUTO;
            auto pick_t = [&](const rtj::Value* v) {
                if (v && v->is_string()) {
                    if (v->str == "reference") trav = TRAV_REFERENCE;
                    else if (v->str == "fast") trav = TRAV_FAST;
                    else if (v->str == "brute") trav = TRAV_BRUTE;
                    else if (v->str == "auto") trav = TRAV_AUTO;
                    else throw std::runtime_error("traversal must be 'auto', 'fast', 'brute' or 'reference'");
                }
            };
            if (const rtj::Value* r = scene.get("render")) pick_t(r->get("traversal"));
            if (rop) pick_t(rop->get("traversal"));
            cam->traversal = trav;
            if (env_flag("RT_AMD_LAUNCH_LOG", false)) {
                const SceneBuild& b = cam->build;
                std::fprintf(stderr,
                             "[rt scene] prims %zu t4nodes %zu (%zu B) tnodes %zu tprims %zu B tsph %zu B prims %zu B "
                             "mats %zu B lights %zu B nodes %zu stack_depth %d\n",
                             b.prims.size(), b.t4nodes.size(), b.t4nodes.size() * sizeof(b.t4nodes[0]), b.tnodes.size(),
                             b.tprims.size() * 4, b.tsph.size() * 16, b.prims.size() * sizeof(RtPrim),
                             b.mats.size() * sizeof(RtMat), b.lights.size() * sizeof(RtLight), b.nodes.size(),
                             b.cam.stack_depth);
            }
            // MixturePDF([cosine, ...lights], [0.5, ...0.5/nL]).totalWeight (pdf.ts:48-52)
            const int nl = cam->build.cam.n_lights;
            cam->light_w = nl > 0 ? 0.5 / (double)nl : 0.0;
            double total = 0.0;
            total += 0.5;
            for (int k = 0; k < nl; ++k) total += cam->light_w;
            cam->mix_total = total;
        } catch (...) {
            delete cam;
            throw;
        }
        *out = cam;
        return RT_OK;
    } catch (const std::exception& e) {
        return set_error(RT_ERR_INVALID, e.what());
    }
}

void rt_camera_destroy(rt_camera* cam) { delete cam; }

int rt_camera_get_info(const rt_camera* cam, rt_camera_info* info) {
    if (!cam || !info) return set_error(RT_ERR_INVALID, "null argument");
    const RtCamera& C = cam->build.cam;
    info->width = C.width;
    info->height = C.height;
    info->channels = 3;
    info->n_objects = C.n_prims;
    info->n_nodes = C.n_nodes;
    info->n_lights = C.n_lights;
    info->n_materials = C.n_mats;
    info->bvh_depth = cam->build.bvh_depth;
    info->samples_loop = C.n_samples;
    info->depth = C.depth;
    info->roulette = C.roulette;
    info->roulette_depth = C.roulette_depth;
    info->mode = C.mode;
    info->adaptive = C.adaptive;
    info->precision = cam->precision;
    // effective traversal: fast/brute only where provably exact (scene.cpp prims_inside_boxes)
    info->traversal = cam->effective_traversal(cam->traversal);
    info->seed = C.seed;
    info->samples = C.samples;
    info->aperture = C.aperture;
    info->a_tolerance = C.a_tolerance;
    info->a_batch = C.a_batch;
    return RT_OK;
}

int rt_camera_set_precision(rt_camera* cam, int32_t precision) {
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    if (precision != PREC_REF && precision != PREC_FP32) return set_error(RT_ERR_INVALID, "bad precision");
    cam->precision = precision;
    return RT_OK;
}

int rt_camera_render_region(rt_camera* cam, const rt_region* region, uint8_t* rgb, float* radiance,
                            rt_render_stats* stats) {
    if (!cam || !region) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        DevCtx& c = cam->current();
        c.ensure_device();
        c.ensure_frame();
        const hipStream_t stream = nullptr;
        cam->last = &c;
        cam->multi.clear();
        c.launch(*region, 0, 1, cam->precision, cam->traversal, 0, rgb ? c.d_rgb : nullptr,
                 radiance ? c.d_rad : nullptr, nullptr, nullptr, 0, stream);
        c.read_stats(stats, nullptr, stream);
        copy_region_to_host(c, *region, rgb, radiance, stream);
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        return RT_OK;
    } catch (const HipError& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_RENDER, e.what());
    }
}

int rt_camera_render(rt_camera* cam, uint8_t* rgb, float* radiance, rt_render_stats* stats) {
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    rt_region r{0, 0, cam->build.cam.width, cam->build.cam.height};
    return rt_camera_render_region(cam, &r, rgb, radiance, stats);
}

int rt_camera_render_png(rt_camera* cam, int32_t bands, rt_render_stats* stats, uint8_t** out, size_t* out_len) {
    if (!cam || !out || !out_len) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        DevCtx& c = cam->current();
        c.ensure_device();
        c.ensure_frame();
        const RtCamera& C = cam->build.cam;
        const hipStream_t stream = nullptr;
        // The reference renders divideIntoRegions' ceil(H / count)-row bands on `count` workers
        // (src/raytracer.ts:60-90, 185-205) and merges their RenderStats (renderStats.ts:42-64).
        // Neither the image nor the merged stats depend on the split (the path RNG is keyed by
        // pixel and sample; merge sums totals and takes minima / maxima), so the device renders
        // the whole frame in one launch whatever `bands` says - one launch and one stats read
        // instead of `bands` small ones, each waiting for the GPU.
        (void)bands;
        const rt_region r{0, 0, C.width, C.height};
        cam->last = &c;
        cam->multi.clear();
        c.launch(r, 0, 1, cam->precision, cam->traversal, 0, c.d_rgb, nullptr, nullptr, nullptr, 0, stream);
        rt_render_stats m;
        c.read_stats(&m, nullptr, stream);
        if (stats) *stats = m;
        png_out(c, stream, out, out_len);
        return RT_OK;
    } catch (const HipError& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_RENDER, e.what());
    }
}

int rt_camera_render_device(rt_camera* cam, const rt_launch* L, rt_render_stats* stats, uint64_t* work_counters) {
    if (!cam || !L) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        DevCtx& c = cam->current();
        c.ensure_device();
        const hipStream_t stream = (hipStream_t)L->stream;
        const int prec = L->precision < 0 ? cam->precision : L->precision;
        const int trav = L->traversal < 0 ? cam->traversal : L->traversal;
        if (L->count_work < 0 || L->count_work > 2) throw std::invalid_argument("count_work must be 0, 1 or 2");
        cam->last = &c;
        cam->multi.clear();
        c.launch(L->region, L->tile_group, L->tile_groups, prec, trav, L->count_work, L->rgb, L->radiance,
                 L->px_samples, L->px_bounces, L->packed_tiles, stream);
        if (L->synchronize) c.read_stats(stats, L->count_work ? work_counters : nullptr, stream);
        return RT_OK;
    } catch (const HipError& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_RENDER, e.what());
    }
}

int rt_camera_export(const rt_camera* cam, void* nodes, void* prims, void* materials, void* lights,
                     int32_t* prim_object) {
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    const SceneBuild& b = cam->build;
    if (nodes) std::memcpy(nodes, b.nodes.data(), b.nodes.size() * sizeof(RtNode));
    if (prims) std::memcpy(prims, b.prims.data(), b.prims.size() * sizeof(RtPrim));
    if (materials) std::memcpy(materials, b.mats.data(), b.mats.size() * sizeof(RtMat));
    if (lights) std::memcpy(lights, b.lights.data(), b.lights.size() * sizeof(RtLight));
    if (prim_object) std::memcpy(prim_object, b.prim_object.data(), b.prim_object.size() * sizeof(int32_t));
    return RT_OK;
}

int rt_debug_world_hit(rt_camera* cam, int32_t traversal, int32_t n, const float* orig, const float* dir,
                       double* out) {
    if (!cam || n < 0 || (n > 0 && (!orig || !dir || !out))) return set_error(RT_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lock(cam->mu);
    float* d_o = nullptr;
    float* d_d = nullptr;
    double* d_out = nullptr;
    try {
        DevCtx& c = cam->current();
        c.ensure_device();
        if (n == 0) return RT_OK;
        hip_check(hipMalloc(&d_o, (size_t)n * 3 * sizeof(float)), "hipMalloc");
        hip_check(hipMalloc(&d_d, (size_t)n * 3 * sizeof(float)), "hipMalloc");
        hip_check(hipMalloc(&d_out, (size_t)n * 10 * sizeof(double)), "hipMalloc");
        hip_check(hipMemcpy(d_o, orig, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy");
        hip_check(hipMemcpy(d_d, dir, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy");
        const int trav = c.effective_traversal(traversal < 0 ? cam->traversal : traversal);
        hip_check(launch_world_hit_ref(c.dev_scene(), trav, n, d_o, d_d, d_out, nullptr),
                  "world_hit_kernel");
        hip_check(hipMemcpy(out, d_out, (size_t)n * 10 * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
        (void)hipFree(d_o);
        (void)hipFree(d_d);
        (void)hipFree(d_out);
        return RT_OK;
    } catch (const std::exception& e) {
        if (d_o) (void)hipFree(d_o);
        if (d_d) (void)hipFree(d_d);
        if (d_out) (void)hipFree(d_out);
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_debug_math(int32_t n, const uint32_t* u, double* out) {
    if (n < 0 || (n > 0 && (!u || !out))) return set_error(RT_ERR_INVALID, "bad arguments");
    uint32_t* d_u = nullptr;
    double* d_out = nullptr;
    try {
        if (n == 0) return RT_OK;
        hip_check(hipMalloc(&d_u, (size_t)n * sizeof(uint32_t)), "hipMalloc");
        hip_check(hipMalloc(&d_out, (size_t)n * 3 * sizeof(double)), "hipMalloc");
        hip_check(hipMemcpy(d_u, u, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice), "hipMemcpy");
        hip_check(launch_math_probe(n, d_u, d_out, nullptr), "math_probe_kernel");
        hip_check(hipMemcpy(out, d_out, (size_t)n * 3 * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
        (void)hipFree(d_u);
        (void)hipFree(d_out);
        return RT_OK;
    } catch (const std::exception& e) {
        if (d_u) (void)hipFree(d_u);
        if (d_out) (void)hipFree(d_out);
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_debug_fp64(int32_t n, const double* x, double* out) {
    if (n < 0 || (n > 0 && (!x || !out))) return set_error(RT_ERR_INVALID, "bad arguments");
    double* d_x = nullptr;
    double* d_out = nullptr;
    try {
        if (n == 0) return RT_OK;
        hip_check(hipMalloc(&d_x, (size_t)n * sizeof(double)), "hipMalloc");
        hip_check(hipMalloc(&d_out, (size_t)n * 4 * sizeof(double)), "hipMalloc");
        hip_check(hipMemcpy(d_x, x, (size_t)n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
        hip_check(launch_fp64_probe(n, d_x, d_out, nullptr), "fp64_probe_kernel");
        hip_check(hipMemcpy(out, d_out, (size_t)n * 4 * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
        (void)hipFree(d_x);
        (void)hipFree(d_out);
        return RT_OK;
    } catch (const std::exception& e) {
        if (d_x) (void)hipFree(d_x);
        if (d_out) (void)hipFree(d_out);
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_debug_pass_plan(int64_t units, int64_t unit_slots, int64_t chunks_per_slot, int64_t rec_bytes_per_unit,
                       int64_t budget_bytes, int64_t* pass_units_out) {
    if (units < 0 || unit_slots < 1 || chunks_per_slot < 1 || rec_bytes_per_unit < 1 || budget_bytes < 1 ||
        !pass_units_out)
        return set_error(RT_ERR_INVALID, "bad arguments");
    *pass_units_out = pass_units((long)units, (long)unit_slots, (long)chunks_per_slot, (size_t)rec_bytes_per_unit,
                                 (size_t)budget_bytes);
    return RT_OK;
}

int rt_debug_rng(uint32_t seed, uint32_t pixel, uint32_t sample, int32_t n, uint32_t* out) {
    if (n < 0 || (n > 0 && !out)) return set_error(RT_ERR_INVALID, "bad arguments");
    uint64_t s = splitmix64((((uint64_t)pixel << 32) | sample) ^ splitmix64(seed));
    for (int32_t k = 0; k < n; ++k) {
        const uint64_t old = s;
        s = old * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        out[k] = (xs >> rot) | (xs << ((32u - rot) & 31u));
    }
    return RT_OK;
}

int rt_camera_kernel_times(rt_camera* cam, float* path_ms, float* accum_ms) {
    if (!cam || !path_ms || !accum_ms) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        *path_ms = 0.0f;
        *accum_ms = 0.0f;
        if (cam->last) cam->last->times(path_ms, accum_ms);
        return RT_OK;
    } catch (const std::exception& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_camera_stats_words(rt_camera* cam, uint64_t* dst, void* stream) {
    if (!cam || !dst) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        DevCtx* c = cam->last;
        if (!c || !c->live || !c->d_stats) throw std::invalid_argument("rt_camera_stats_words: no render yet");
        // the ST_WORDS words sit kStatStride apart (one 128-B line each); dst gets them packed
        hip_check(hipMemcpy2DAsync(dst, sizeof(uint64_t), c->d_stats, kStatStride * sizeof(unsigned long long),
                                   sizeof(uint64_t), ST_WORDS, hipMemcpyDeviceToDevice, (hipStream_t)stream),
                  "hipMemcpy2DAsync(stats)");
        return RT_OK;
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_camera_adaptive_info(rt_camera* cam, int32_t* rounds, uint64_t* samples_rendered) {
    if (!cam || !rounds || !samples_rendered) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    *rounds = cam->last ? cam->last->adapt_rounds : 0;
    *samples_rendered = cam->last ? cam->last->adapt_rendered : 0;
    return RT_OK;
}

int rt_camera_pass_count(rt_camera* cam, int32_t* passes) {
    if (!cam || !passes) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    *passes = cam->last ? cam->last->n_passes : 0;
    return RT_OK;
}

int rt_camera_last_kernel(rt_camera* cam, int32_t* kernel) {
    if (!cam || !kernel) return set_error(RT_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(cam->mu);
    *kernel = cam->last ? cam->last->last_kernel : RT_KERNEL_NONE;
    return RT_OK;
}

int rt_multi_plan_region(const rt_region* region, int32_t width, int32_t height, int32_t n_devices,
                         rt_multi_plan* plan) {
    if (!region || !plan || width < 0 || height < 0 || n_devices < 1 || n_devices > RT_MAX_DEVICES)
        return set_error(RT_ERR_INVALID, "rt_multi_plan_region: bad arguments");
    *plan = make_multi_plan(*region, width, height, n_devices);
    return RT_OK;
}

// Errors of the multi-GPU entries: the reference's render errors, HIP / RCCL errors, bad arguments.
static int multi_call(rt_camera* cam, const std::function<void()>& f) {
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    std::lock_guard<std::mutex> lock(cam->mu);
    try {
        f();
        return RT_OK;
    } catch (const HipError& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_RENDER, e.what());
    }
}

int rt_camera_render_multi(rt_camera* cam, const int32_t* devices, int32_t n_devices, const rt_region* region,
                           uint8_t* rgb, float* radiance, rt_render_stats* stats) {
    if (!region) return set_error(RT_ERR_INVALID, "null region");
    return multi_call(cam, [&] {
        unsigned long long m[ST_WORDS];
        render_multi(cam, devices, n_devices, *region, rgb != nullptr, radiance != nullptr, m,
                     [&](DevCtx& root) { copy_region_to_host(root, *region, rgb, radiance, root.stream); });
        DevCtx::stats_from_words(m, stats);
    });
}

int rt_camera_render_png_multi(rt_camera* cam, const int32_t* devices, int32_t n_devices, rt_render_stats* stats,
                               uint8_t** out, size_t* out_len) {
    if (!out || !out_len) return set_error(RT_ERR_INVALID, "null argument");
    return multi_call(cam, [&] {
        const rt_region r{0, 0, cam->build.cam.width, cam->build.cam.height};
        unsigned long long m[ST_WORDS];
        DevCtx& root = render_multi(cam, devices, n_devices, r, true, false, m, nullptr);
        DevCtx::stats_from_words(m, stats);
        png_out(root, root.stream, out, out_len);
    });
}

int rt_camera_multi_info(rt_camera* cam, rt_multi_info* info) {
    if (!info) return set_error(RT_ERR_INVALID, "null argument");
    return multi_call(cam, [&] {
        *info = rt_multi_info{};
        if (cam->multi.empty()) return;
        info->n_devices = (int32_t)cam->multi.size();
        info->transport = cam->multi_transport;
        info->plan = cam->multi_plan;
        for (size_t g = 0; g < cam->multi.size(); ++g) {
            DevCtx& c = *cam->multi[g];
            info->devices[g] = c.device;
            c.times(&info->path_ms[g], &info->accum_ms[g]);
        }
        DevCtx& root = *cam->multi[0];
        hip_check(hipEventSynchronize(root.ev_gather1), "hipEventSynchronize");
        hip_check(hipEventElapsedTime(&info->gather_ms, root.ev_gather0, root.ev_gather1), "hipEventElapsedTime");
    });
}

int rt_camera_release_device(rt_camera* cam) {
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    std::lock_guard<std::mutex> lock(cam->mu);
    cam->release();
    return RT_OK;
}

const char* rt_build_id(void) { return RT_BUILD_ID; }

int rt_tiles_unpack(const void* slabs, int32_t tile_groups, int32_t slab_tiles, const rt_region* region,
                    int32_t width, int32_t height, int32_t channels, int32_t elem_bytes, void* frame, void* stream) {
    if (!region || tile_groups < 1 || slab_tiles < 0 || width < 0 || height < 0 || channels < 1 ||
        (elem_bytes != 1 && elem_bytes != 4) || (slab_tiles > 0 && (!slabs || !frame)))
        return set_error(RT_ERR_INVALID, "rt_tiles_unpack: bad arguments");
    try {
        // the region clamped to the image, as the render launch clamps it
        const int x0 = std::max(region->x, 0), y0 = std::max(region->y, 0);
        const int x1 = std::min(region->x + region->width, width), y1 = std::min(region->y + region->height, height);
        const RtRegion reg{x0, y0, std::max(x1 - x0, 0), std::max(y1 - y0, 0), 0, 1};
        const long tiles = (long)((reg.width + kTile - 1) / kTile) * ((reg.height + kTile - 1) / kTile);
        if ((long)slab_tiles * tile_groups < tiles)
            throw std::invalid_argument("rt_tiles_unpack: slabs hold fewer tiles than the region");
        hip_check(launch_tiles_unpack(slabs, tile_groups, slab_tiles, reg, width, channels, elem_bytes, frame,
                                      (hipStream_t)stream),
                  "tiles_unpack_kernel");
        return RT_OK;
    } catch (const std::invalid_argument& e) {
        return set_error(RT_ERR_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_error(RT_ERR_DEVICE, e.what());
    }
}

int rt_device_count(int32_t* count) {
    if (!count) return set_error(RT_ERR_INVALID, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}

}  // extern "C"
