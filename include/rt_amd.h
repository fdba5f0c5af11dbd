/*
 * rt_amd.h - C ABI of the MI355X path-tracing core (librt_amd.so).
 *
 * This is the drop-in boundary for df07/mcp-raytracer's hot path. The
 * reference has no FFI: its boundary is the TypeScript object model, and the
 * call site this library replaces is
 *
 *     createCameraFromSceneData(sceneData, renderOptions)   src/scenes/scenes.ts:60-104
 *     camera.renderRegion(buffer, region) -> RenderStats     src/camera.ts:388-431
 *     camera.render(buffer)                                  src/camera.ts:439-446
 *
 * called from generateImageBuffer (src/raytracer.ts:56-59) and from each render
 * worker (src/render-utils/renderWorker.ts:17-26). Scenes cross the boundary in
 * the reference's own wire format, SceneData JSON (src/scenes/sceneData.ts:8-110);
 * render options are the RenderOptions object (src/camera.ts:42-52) as JSON, plus
 * two extensions: "seed" (u32 path-RNG seed; the reference's Math.random is
 * unseeded) and "precision" ("ref" = JS-double scalars, the default; "fp32").
 *
 * Conventions: plain pointers and sizes, no torch types. Every function returns
 * 0 on success and a nonzero status on failure; rt_last_error() then holds the
 * message (thread-local), mirroring the reference's thrown Error messages.
 * Host-side functions (scene generation, camera build, info, export) run without
 * a GPU; render functions need a visible gfx950 device.
 */
#ifndef RT_AMD_H
#define RT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_AMD_VERSION 3

enum {
    RT_OK = 0,
    RT_ERR_INVALID = 1,   /* bad arguments / scene (reference throws an Error) */
    RT_ERR_DEVICE = 2,    /* HIP error */
    RT_ERR_RENDER = 3     /* error raised during rendering (e.g. miss without background) */
};

enum { RT_PRECISION_REF = 0, RT_PRECISION_FP32 = 1 };
/* Closest-hit strategy. All return the reference's closest hit bit-for-bit:
 * REFERENCE visits nodes in BVHNode.hit's order with AABB.hit's per-axis test
 * (src/geometry/bvh.ts:128-146); FAST culls with a strict slab test on padded
 * boxes, near child first, and breaks t ties by leaf order; BRUTE tests every
 * primitive in leaf order (small scenes). AUTO (default) = BRUTE up to 16
 * primitives, else FAST. FAST/BRUTE fall back to REFERENCE for scenes where a
 * primitive can be hit outside its reference box (rt_camera_info.traversal
 * reports the strategy in effect). */
enum { RT_TRAVERSAL_FAST = 0, RT_TRAVERSAL_REFERENCE = 1, RT_TRAVERSAL_BRUTE = 2, RT_TRAVERSAL_AUTO = 3 };

typedef struct rt_camera rt_camera;

/* RenderRegion (src/camera.ts:54-59) */
typedef struct {
    int32_t x, y, width, height;
} rt_region;

/* RenderStats (src/render-utils/renderStats.ts:6-19). min fields are +inf when
 * no pixel / sample was rendered, exactly as the reference's Infinity seed. */
typedef struct {
    double pixels;
    double samples_total, samples_min, samples_max, samples_avg;
    double bounces_total, bounces_min, bounces_max, bounces_avg;
} rt_render_stats;

/* Camera geometry and options after createCameraFromSceneData. */
typedef struct {
    int32_t width, height, channels;
    int32_t n_objects, n_nodes, n_lights, n_materials, bvh_depth;
    int32_t samples_loop, depth, roulette, roulette_depth, mode, adaptive, precision, traversal;
    uint32_t seed;
    double samples, aperture, a_tolerance, a_batch;
} rt_camera_info;

/* Device-resident launch (benchmarks, multi-GPU). Output pointers are DEVICE
 * pointers in full-frame layout (width*height*3, row-major, RGB) and only the
 * region's tiles are written. Tiles are 8x8 pixel blocks enumerated row-major
 * over the region; this launch renders tile t iff t % tile_groups == tile_group
 * (tile_groups = 1: the whole region). `stream` is a hipStream_t (NULL = default). */
typedef struct {
    rt_region region;
    int32_t tile_group, tile_groups;
    int32_t precision;       /* -1: the camera's precision */
    int32_t traversal;       /* -1: the camera's; else an RT_TRAVERSAL_* value */
    int32_t count_work;      /* 1: instrumented build, fills work_counters; 2: section-timing diagnostic */
    uint8_t* rgb;            /* device, may be NULL */
    float* radiance;         /* device, may be NULL */
    int32_t* px_samples;     /* device W*H, may be NULL */
    int32_t* px_bounces;     /* device W*H, may be NULL */
    void* stream;
    int32_t synchronize;     /* 1: wait and fill stats / work_counters; 0: asynchronous (an adaptive-
                              * sampling render still waits on `stream` once per round: the next
                              * round's launch is sized by the pixels left) */
    int32_t packed_tiles;    /* 0: outputs in full-frame layout; 1: tile-packed slab - the pixel
                              * of lane l (= 8*row + col inside the tile) of this launch's k-th
                              * tile at index k*64 + l (rgb/radiance 3 values per index, the
                              * px_* arrays 1); unpack with rt_tiles_unpack (multi-GPU gather) */
} rt_launch;

/* Work counters of an instrumented launch (SURVEY.md §8d algorithmic bytes). */
enum {
    RT_CT_NODE = 0, RT_CT_SPHERE, RT_CT_QUAD, RT_CT_PLANE, RT_CT_MATERIAL, RT_CT_LIGHT_QUAD,
    RT_CT_LIGHT_SPHERE, RT_CT_BOUNCES, RT_CT_DIFFUSE, RT_CT_SAMPLES, RT_CT_RAYS,
    RT_CT_EXACT,       /* primitives whose exact fp64 test ran (fast/brute strategies) */
    RT_CT_EXACT_WAVE,  /* wave-level executions of those exact tests */
    RT_CT_WORDS
};
/* count_work == 2 (diagnostic): wave-cycles (s_memtime) per path-loop section,
 * summed over waves, at work_counters[RT_CT_WORDS + RT_PR_*]; for sections
 * k < RT_PR_LOOP also the active lanes summed over the wave executions of the
 * section at [RT_CT_WORDS + RT_PR_WORDS + k] and the number of those executions
 * at [RT_CT_WORDS + RT_PR_WORDS + RT_PR_LOOP + k]. */
enum {
    RT_PR_NEWPATH = 0, RT_PR_RR, RT_PR_HIT, RT_PR_MISS, RT_PR_HITREC, RT_PR_SCATTER, RT_PR_SAMPLE, RT_PR_PDF,
    RT_PR_ACC, RT_PR_TILE,
    RT_PR_NODE, RT_PR_LEAF,  /* lane counts only (no cycles): the resumable walk's node steps and leaf tests */
    RT_PR_LOOP, RT_PR_TRIPS, RT_PR_WORDS
};
/* work_counters arrays passed to rt_camera_render_device hold this many entries. */
#define RT_COUNTER_WORDS 64

int rt_version(void);
const char* rt_last_error(void);
void rt_free(void* p);

/* generateSceneData({type, options}) (src/scenes/scenes.ts:42-50). type is
 * "default" | "spheres" | "rain" | "cornell"; options_json the *SceneOptions
 * object or NULL. *out_json is malloc'ed; release with rt_free. */
int rt_generate_scene_data(const char* type, const char* options_json, char** out_json);

/* createCameraFromSceneData (src/scenes/scenes.ts:60-104). Host only. */
int rt_camera_create(const char* scene_json, const char* render_options_json, rt_camera** out);
void rt_camera_destroy(rt_camera* cam);
int rt_camera_get_info(const rt_camera* cam, rt_camera_info* info);
int rt_camera_set_precision(rt_camera* cam, int32_t precision);

/* Camera.renderRegion (src/camera.ts:388-431). rgb: caller-owned HOST buffer of
 * width*height*3 bytes (Uint8ClampedArray layout), only the region is written.
 * radiance: optional host float buffer of width*height*3 (final pixel colour).
 * stats: optional. */
int rt_camera_render_region(rt_camera* cam, const rt_region* region, uint8_t* rgb, float* radiance,
                            rt_render_stats* stats);
/* Camera.render (src/camera.ts:439-446): the whole image. */
int rt_camera_render(rt_camera* cam, uint8_t* rgb, float* radiance, rt_render_stats* stats);

/* Device-resident render (see rt_launch). stats / work_counters (RT_COUNTER_WORDS
 * u64) are filled only when launch->synchronize is 1. */
int rt_camera_render_device(rt_camera* cam, const rt_launch* launch, rt_render_stats* stats,
                            uint64_t* work_counters);

/* Host copies of the flattened scene, for tests: sizes in bytes are
 * n_nodes*32, n_objects*96, n_materials*64, n_lights*16; prim_object gets
 * n_objects int32 (leaf slot -> SceneData.objects index). Any pointer may be NULL. */
int rt_camera_export(const rt_camera* cam, void* nodes, void* prims, void* materials, void* lights,
                     int32_t* prim_object);

/* Closest hit of n rays through the device BVH (ref precision; traversal -1 =
 * the camera's). orig/dir: host float[3*n]; out: host double[10*n] =
 * {hit, t, p.xyz, n.xyz, front, prim_slot}. */
int rt_debug_world_hit(rt_camera* cam, int32_t traversal, int32_t n, const float* orig, const float* dir,
                       double* out);

/* The device's Math.cos(phi), Math.sin(phi) (phi = 2 PI xi, the cosine-PDF angle)
 * and Math.pow(xi, 5) (Schlick) for xi = u[k] / 2^32: out = host double[3*n]. */
int rt_debug_math(int32_t n, const uint32_t* u, double* out);

/* The device's restricted-domain double square root and reciprocal beside the general
 * ones, for x = host double[n]: out = host double[4*n] = {sqrt_rn(x), sqrt(x), rcp_rn(x),
 * 1 / x} (pins rt_math.hpp sqrt_rn / rcp_rn bit for bit on their domains). */
int rt_debug_fp64(int32_t n, const double* x, double* out);

/* Pass sizing of a fixed-spp / adaptive launch (host only, no device): the units (64-slot
 * tile groups) one pass of the path kernel takes out of `units`, given each unit's slots,
 * the guided schedule's chunks per slot (items per slot), each unit's record bytes and the
 * record budget. A pass never numbers 2^31 - 2^22 or more items (the hand-out counter's
 * headroom): a budget past that gives more passes, not an error. */
int rt_debug_pass_plan(int64_t units, int64_t unit_slots, int64_t chunks_per_slot, int64_t rec_bytes_per_unit,
                       int64_t budget_bytes, int64_t* pass_units);

/* The path RNG stream (seeded Math.random replacement), host evaluation. */
int rt_debug_rng(uint32_t seed, uint32_t pixel, uint32_t sample, int32_t n, uint32_t* out);

/* Number of visible HIP devices (0 without a GPU). */
int rt_device_count(int32_t* count);

/* Device time of the most recent rt_camera_render_device / render_region call,
 * from HIP events recorded on its stream: `path_ms` = the path-tracing
 * kernel(s), `accum_ms` = the chunked mode's in-order accumulate pass (0 for the
 * sequential kernel). Waits for that call's events. */
int rt_camera_kernel_times(rt_camera* cam, float* path_ms, float* accum_ms);

/* RenderStats words of the most recent render, queued on `stream` as a
 * device-to-device copy into `dst` (DEVICE, 8 u64): pixels, samples total,
 * samples min (~0 = none), samples max, bounces total, bounces min (~0 = none),
 * bounces max, error flags. Multi-GPU ranks ship these beside their slab so rank
 * 0 can merge them as RenderStats.merge does (src/render-utils/renderStats.ts:
 * 42-64, called from src/raytracer.ts:86-89) without a host round trip. */
#define RT_STATS_WORDS 8
int rt_camera_stats_words(rt_camera* cam, uint64_t* dst, void* stream);

/* Adaptive sampling of the most recent render: the rounds it ran on the chunked /
 * pool kernels (0: not adaptive, or the sequential kernel) and the samples those
 * rounds rendered - at least RenderStats.samples.total; the excess is the
 * speculation past each pixel's convergence (src/camera.ts:400-425 loop). */
int rt_camera_adaptive_info(rt_camera* cam, int32_t* rounds, uint64_t* samples_rendered);

/* Number of chunked-kernel passes of the most recent render (0 before any; the
 * sequential kernel counts as one). Passes split the per-sample record buffer. */
int rt_camera_pass_count(rt_camera* cam, int32_t* passes);

/* Path kernel of the most recent render: RT_KERNEL_NONE before any,
 * RT_KERNEL_SEQUENTIAL (wave per 8x8 tile, adaptive sampling), RT_KERNEL_CHUNKED
 * (lane work pool + in-order accumulate) or RT_KERNEL_POOL (stage-compacted
 * path pools + in-order accumulate). Diagnostics and tests; no reference
 * counterpart (the reference has one CPU loop, src/camera.ts:388-431).
 * (Values 4 and 5 named the round-3 walker-pool and wavefront kernels, removed
 * in round 4; they are not reused.) */
enum { RT_KERNEL_NONE = 0, RT_KERNEL_SEQUENTIAL = 1, RT_KERNEL_CHUNKED = 2, RT_KERNEL_POOL = 3 };
int rt_camera_last_kernel(rt_camera* cam, int32_t* kernel);

/* Frees the camera's device resources on every device it rendered on (scene copies, frame,
 * record and slab buffers, streams, events). A camera otherwise keeps one scene copy per device
 * (the calling thread's current device for the single-device entries, each listed device for
 * rt_camera_render_multi), so moving between devices never re-uploads; the next render
 * re-creates what it needs. */
int rt_camera_release_device(rt_camera* cam);

/* Hash of the HIP/C++ sources and compiler flags this library was built from
 * (static string, never freed). */
const char* rt_build_id(void);

/* Reassembles a region's frame from tile-packed slabs (multi-GPU gather): slabs
 * holds `tile_groups` slabs of `slab_tiles` tiles each, slab r = the packed
 * output of tile_group r (rt_launch.packed_tiles); tile k of slab r is the
 * region's tile r + k*tile_groups. Writes the region's pixels of `frame`
 * (full-frame layout, width*height pixels, `channels` values of `elem_bytes`
 * bytes each: 1 = u8 RGB, 4 = f32 radiance). DEVICE pointers; queued on
 * `stream` (a hipStream_t, NULL = default). */
int rt_tiles_unpack(const void* slabs, int32_t tile_groups, int32_t slab_tiles, const rt_region* region,
                    int32_t width, int32_t height, int32_t channels, int32_t elem_bytes, void* frame, void* stream);

/* Image file encoders for the framebuffer (the reference hands its buffer to
 * sharp, src/raytracer.ts:101-110): 8-bit RGB PNG (zlib level 0-9) or binary
 * PPM (P6). rgb: host width*height*3 bytes. *out is malloc'ed (rt_free). */
int rt_encode_png(const uint8_t* rgb, int32_t width, int32_t height, int32_t level, uint8_t** out, size_t* out_len);
int rt_encode_ppm(const uint8_t* rgb, int32_t width, int32_t height, uint8_t** out, size_t* out_len);

/* PNG of a DEVICE-resident u8 RGB frame (width*height*3), encoded on the GPU:
 * per-row PNG filter (libpng's min-sum choice), the filtered stream cut into
 * 4 KiB segments, each one deflate block with its own dynamic Huffman code
 * (run matches at distance 1 / 3) ended by a sync flush, plus its Adler-32 and
 * CRC-32; the host only combines those words and writes the chunk headers.
 * Queued on `stream` (hipStream_t, NULL = default) and waited for; *out is
 * malloc'ed (rt_free). Replaces sharp(...).png().toBuffer() (src/raytracer.ts:
 * 101-110) without the frame crossing PCIe uncompressed. */
int rt_encode_png_device(const uint8_t* d_rgb, int32_t width, int32_t height, void* stream, uint8_t** out,
                         size_t* out_len);

/* The same encoder run on the host, byte-identical to rt_encode_png_device
 * (tests: the CPU pin of the device encoder's bytes). rgb: HOST pointer. */
int rt_debug_png_host(const uint8_t* rgb, int32_t width, int32_t height, uint8_t** out, size_t* out_len);

/* generateImageBuffer's core (src/raytracer.ts:39-113): renders the whole frame
 * on the device, writes its RenderStats into *stats (may be NULL) and returns the
 * PNG encoded on the device (rt_encode_png_device). `bands` is the reference's worker
 * count (divideIntoRegions, src/raytracer.ts:185-205): neither the image nor the
 * merged stats (RenderStats.merge) depend on it, so the frame is one launch.
 * *out is malloc'ed (rt_free). */
int rt_camera_render_png(rt_camera* cam, int32_t bands, rt_render_stats* stats, uint8_t** out, size_t* out_len);

/* ---- Single-process multi-GPU (SURVEY.md §8b "rt_render_multi", §8e) ----------------------
 * The reference's parallel path is one process driving N workers over bands of one buffer
 * (src/raytracer.ts:60-90 generateImageBuffer with parallel workers, 185-205
 * divideIntoRegions; src/render-utils/renderWorker.ts:17-35 each worker's renderRegion,
 * merged with RenderStats.merge, src/render-utils/renderStats.ts:42-64). Here one call drives
 * N GPUs: the region's 8x8 tiles are dealt round-robin (tile t -> devices[t % n]); every
 * listed device renders its tiles into a tile-packed slab on its own stream (one host thread
 * per device, the camera's scene uploaded once per device and kept); the slabs - each with the
 * device's RenderStats words in a spare tile - are gathered on devices[0] over RCCL (one
 * ncclSend / ncclRecv group on single-process communicators, ncclCommInitAll, i.e. xGMI
 * between MI355X GPUs), unpacked into the full frame by rt_tiles_unpack and the stats merged
 * as RenderStats.merge does. The path RNG is keyed by (pixel, sample): the image and the
 * merged stats equal a single-device render bit for bit, for any n. A device may be listed
 * more than once (the split rehearsed on fewer GPUs); the gather then uses device-to-device
 * copies (RT_GATHER_PEER), since RCCL needs distinct devices. The environment variable
 * RT_AMD_GATHER=rccl|peer forces the transport. */
#define RT_MAX_DEVICES 16
enum { RT_GATHER_RCCL = 0, RT_GATHER_PEER = 1 };

/* The split of a region over n devices (host only). */
typedef struct {
    rt_region region;          /* the region clamped to the image */
    int32_t n_devices;
    int32_t slab_tiles;        /* tiles per slab: the largest share, ceil(tiles / n) */
    int64_t tiles;             /* 8x8 tiles of the region, row-major */
    int64_t slab_bytes_rgb;    /* u8 slab: (slab_tiles + 1) * 64 * 3 (the spare tile carries the stats words) */
    int64_t slab_bytes_radiance; /* f32 slab: slab_tiles * 64 * 3 * 4 */
    int64_t stats_offset;      /* byte offset of the 8 stats words in a u8 slab */
    int32_t group_tiles[RT_MAX_DEVICES]; /* tiles device entry g renders */
} rt_multi_plan;
int rt_multi_plan_region(const rt_region* region, int32_t width, int32_t height, int32_t n_devices,
                         rt_multi_plan* plan);

/* Camera.renderRegion over n_devices GPUs (see above). rgb / radiance: caller-owned HOST
 * buffers in full-frame layout as rt_camera_render_region (only the region is written; either
 * may be NULL); stats: the merged RenderStats (may be NULL). */
int rt_camera_render_multi(rt_camera* cam, const int32_t* devices, int32_t n_devices, const rt_region* region,
                           uint8_t* rgb, float* radiance, rt_render_stats* stats);

/* generateImageBuffer over n_devices GPUs: the whole frame as rt_camera_render_multi, then its
 * PNG encoded on devices[0] (rt_encode_png_device). *out is malloc'ed (rt_free). */
int rt_camera_render_png_multi(rt_camera* cam, const int32_t* devices, int32_t n_devices, rt_render_stats* stats,
                               uint8_t** out, size_t* out_len);

/* The most recent rt_camera_render_multi / _png_multi of this camera (n_devices = 0 when a
 * single-device render came after it): devices, transport, plan, each device's path-kernel and
 * accumulate time (HIP events on its stream) and gather_ms = devices[0]'s time from the end of
 * its own render to the assembled frame (waiting for the slowest device, the gather, the unpack
 * and the stats words' copy). Waits for those events. */
typedef struct {
    int32_t n_devices;
    int32_t transport;         /* RT_GATHER_* */
    int32_t devices[RT_MAX_DEVICES];
    float path_ms[RT_MAX_DEVICES];
    float accum_ms[RT_MAX_DEVICES];
    float gather_ms;
    rt_multi_plan plan;
} rt_multi_info;
int rt_camera_multi_info(rt_camera* cam, rt_multi_info* info);

#ifdef __cplusplus
}
#endif

#endif /* RT_AMD_H */
