// Flattened, device-resident form of the reference's Camera + world.
//
// The reference builds an object graph per render (createCameraFromSceneData,
// src/scenes/scenes.ts:60-104): Sphere/Plane/Quad objects (src/entities/*),
// Material objects (src/materials/*), a recursive BVHNode tree
// (src/geometry/bvh.ts:34-102) and a Camera (src/camera.ts:107-166). Here the
// same data is laid out as flat arrays that one HIP kernel reads:
//
//   RtNode  32 B  BVH node in depth-first order, box + (left,right) or leaf range
//   RtPrim  96 B  sphere / quad / plane, in leaf order, with its precomputed
//                 plane frame (normal, D, w) exactly as Plane's constructor does
//   RtMat   64 B  material table, nested materials by index, precomputed emission
//   RtLight 16 B  light list (prim index + quad area), in object order
//   RtCamera      frame vectors + render options
//
// Every fp32 field is produced by the same fp64-compute / fp32-store sequence
// the reference runs, so the device sees bit-identical inputs.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "json.hpp"
#include "rt_math.hpp"

namespace rt {

enum PrimType : int32_t { PRIM_SPHERE = 0, PRIM_QUAD = 1, PRIM_PLANE = 2 };
enum MatType : int32_t {
    MAT_LAMBERT = 0,
    MAT_METAL = 1,
    MAT_GLASS = 2,
    MAT_LIGHT = 3,
    MAT_MIXED = 4,
    MAT_LAYERED = 5,
};
enum RenderMode : int32_t { MODE_DEFAULT = 0, MODE_BOUNCES = 1, MODE_SAMPLES = 2 };

struct alignas(16) RtNode {
    float bmin[3];
    int32_t a;  // interior: left child node; leaf: first prim
    float bmax[3];
    int32_t b;  // interior: right child node (>= 0); leaf: -count (< 0)
};
static_assert(sizeof(RtNode) == 32, "RtNode must be 32 bytes");

// Fast-traversal node: the boxes of BOTH children live in the parent, so one
// 64-byte fetch tests two children. box[k] uses the RtNode box layout (padded
// fnodes boxes) and box[k].a is the child reference: >= 0 another RtTNode,
// < 0 a leaf ~((first_prim << 3) | count).
struct alignas(16) RtTNode {
    RtNode box[2];
};
static_assert(sizeof(RtTNode) == 64, "RtTNode must be 64 bytes");

// 4-wide fast-traversal node (the binary children-in-parent tree collapsed): four children's boxes as [axis][child]
// rows (one ds_read_b128 per row) and their references (node index, leaf code
// as in RtTNode, or kTravDone for an empty slot).
struct alignas(16) RtT4Node {
    float bmin[3][4];
    float bmax[3][4];
    int32_t ref[4];
    int32_t pad[4];
};
static_assert(sizeof(RtT4Node) == 128, "RtT4Node must be 128 bytes");
constexpr int32_t kT4Empty = (int32_t)0x80000000;  // empty child slot (= kTravDone)

// Leaf-order sphere record for trees walked from global memory (tsph2, per tprims entry): the
// fp32 pre-filter's {centre, fp32 radius}, the exact test's fp64 radius (the JS double) and the
// leaf slot - the exact Sphere.hit needs no dependent RtPrim load. Non-spheres: NaN centre.
struct alignas(16) RtLeafSph {
    float c[3];
    float r32;
    double r64;
    int32_t slot;
    int32_t pad;
};
static_assert(sizeof(RtLeafSph) == 32, "RtLeafSph must be 32 bytes");

struct alignas(16) RtPrim {
    int32_t type;
    int32_t mat;
    double s0;     // sphere: radius (JS double); quad/plane: D = normal·Q (double)
    float g0[4];   // sphere: center.xyz, (float)radius | quad/plane: Q.xyz, (float)D
    float g1[4];   // quad/plane: u.xyz, axis quad: u's nonzero component
    float g2[4];   // quad/plane: v.xyz, axis quad: v's nonzero component
    float g3[4];   // quad/plane: normal.xyz, axis quad: +-w[a]
    float g4[4];   // quad/plane: w.xyz, quad: axis code (int bits, 0 = general; scene.cpp encode_axis_quad)
};
static_assert(sizeof(RtPrim) == 96, "RtPrim must be 96 bytes");

struct alignas(16) RtMat {
    int32_t type;
    int32_t c0;      // mixed: material1 | layered: outer dielectric
    int32_t c1;      // mixed: material2 | layered: inner
    int32_t pad0;
    float color[4];    // lambert/metal albedo, light emit
    float emitted[4];  // Material.emitted(rec) (constant per material), fp32
    double p0;         // metal: clamped fuzz | glass: ior | mixed: clamped weight
    double pad1;
};
static_assert(sizeof(RtMat) == 64, "RtMat must be 64 bytes");

// Compact brute-force pre-filter record: everything the fp32 pre-filter of one primitive, or of
// a PAIR of primitives evaluated together in packed fp32 (v_pk_fma_f32: two spheres, or two
// axis-aligned quads of one axis code, which share every ray operand), reads in one 64-byte
// scalar load (the full RtPrim takes two dependent loads for a quad: its type, then its axis
// code). head = kind | k0 << 8 | k1 << 16 (the primitives' slots; k1 only for pairs), last so
// that the pairs' floats sit in aligned SGPR pairs.
//   PRE_SPHERE {cx, cy, cz, r}; 1..6 = axis code {x_a of the plane (D / n[a]), sv = +-w[a]*v[iv],
//   su = +-w[a]*u[iu], -Q[ia]*sv - 1/2, -Q[ib]*su - 1/2, kRel max(|Q[ia]|, |Q[ib]|)};
//   PRE_OTHER: read the RtPrim;
//   PRE_SPHERE2 {cx0, cx1, cy0, cy1, cz0, cz1, r0, r1, r0^2, r1^2};
//   PRE_QUAD2 + code {x_a, sv, su, -Q[ia]*sv - 1/2, -Q[ib]*su - 1/2, -|sv|, -|su|} as element pairs,
//   then max(kRel max(|Q[ia]|, |Q[ib]|)) of the two.
// (scene.cpp encode_axis_quad, rt_api.cpp prefilter_records)
enum : int32_t { PRE_SPHERE = 0, PRE_OTHER = 7, PRE_SPHERE2 = 8, PRE_QUAD2 = 8 /* + code 1..6 */ };
struct alignas(16) RtPre {
    float f[15];
    int32_t head;
};
static_assert(sizeof(RtPre) == 64, "RtPre must be 64 bytes");

// Exact-test record of a brute-force primitive (slot order; in the LDS copy beside the RtPrims):
// every field the nearest-first pass's exact test reads, in two 16-byte loads issued together
// (through the RtPrim they were five dependent LDS round trips: type, axis code, then the
// type's fields). s0: the radius / D (the JS double; the fp32 mode's value is (float)s0 =
// RtPrim g0[3]). kind as RtPre: PRE_SPHERE {centre xyz}, axis code 1..6 {Q[ia], Q[ib], +-w[a],
// v[iv], u[iu]} (the RtPrim fields aquad_t_c reads; its n[a] is +-1 exactly, the sign in bit 3
// of kind), PRE_OTHER (read the RtPrim).
struct alignas(16) RtExact {
    double s0;
    float f[5];
    int32_t kind;
};
static_assert(sizeof(RtExact) == 32, "RtExact must be 32 bytes");
constexpr int32_t kExactNegNa = 8;  // RtExact::kind flag: n[a] = -1

struct alignas(16) RtLight {
    int32_t prim;
    int32_t type;
    double area;  // quad: |u x v| via Math.hypot (double); sphere: unused
};
static_assert(sizeof(RtLight) == 16, "RtLight must be 16 bytes");

// Orthonormal basis (ONBasis, src/geometry/onbasis.ts:18-51) of a planar
// primitive's hit normal, precomputed per face (0: front = the plane normal,
// 1: back = its negation) and per precision (0: ref, 1: fp32): a diffuse bounce
// on a quad or plane reads it instead of rebuilding it (two normalisations).
struct alignas(16) RtOnb {
    float u[4], v[4], w[4];
};
static_assert(sizeof(RtOnb) == 48, "RtOnb must be 48 bytes");

struct RtCamera {
    float pixel00[4];
    float du[4];
    float dv[4];
    float center[4];
    float ddu[4];  // defocusDiskU
    float ddv[4];  // defocusDiskV
    float bg_top[4];
    float bg_bottom[4];
    double aperture;
    double samples;       // RenderOptions.samples (JS number)
    double a_tolerance;
    double a_batch;
    double depth_raw;     // RenderOptions.depth as given (RenderMode.Bounces normalisation)
    int32_t width;
    int32_t height;
    int32_t n_samples;    // loop count implied by `samples` (ceil, >= 0)
    int32_t depth;        // bounces >= depth <=> bounces >= this (ceil of JS depth)
    int32_t roulette;     // truthiness of RenderOptions.roulette
    int32_t roulette_depth;
    int32_t mode;         // RenderMode
    int32_t adaptive;     // useAdaptiveSampling (src/camera.ts:165)
    int32_t n_lights;
    int32_t has_background;
    int32_t emissive_scatter;  // some scattering material also emits (needs the emission stack)
    int32_t n_nodes;
    int32_t n_prims;
    int32_t n_mats;
    uint32_t seed;
    uint64_t seed_mix;    // splitmix64(seed): per-path RNG keys derive from it
    int32_t stack_depth;  // BVH traversal stack entries needed (tree depth + 1)
};

// Per-launch render request (the reference's RenderRegion plus the build's RNG seed
// and multi-GPU tile interleave). Tiles are 8x8 pixel blocks enumerated row-major
// inside the region; this launch renders tiles t with t % tile_groups == tile_group.
struct RtRegion {
    int32_t x, y, width, height;
    int32_t tile_group, tile_groups;
};

// Host-side build product. Owned by rt_camera; uploaded to the device lazily.
struct SceneBuild {
    std::vector<RtNode> nodes;
    std::vector<RtNode> fnodes;  // same tree, boxes for the fast traversal (padded / reject-marked)
    std::vector<RtTNode> tnodes; // fast-traversal tree, children-in-parent (SAH, or the reference tree)
    std::vector<int32_t> tprims; // its leaves' primitive slots (padded to a multiple of 4)
    std::vector<float> tsph;     // per tprims entry: sphere {centre, fp32 radius}, NaNs for other types
    std::vector<RtLeafSph> tsph2; // per tprims entry: the same + fp64 radius + slot (trees walked from global memory)
    std::vector<RtT4Node> t4nodes; // the same tree collapsed to 4-wide nodes (the device walks these)
    int32_t t4root = 0;          // its root reference
    int t4depth = 0;             // its depth in 4-wide nodes
    int32_t troot = 0;           // reference of the root (TNode index or leaf code)
    int tdepth = 0;              // its depth (root = 1)
    RtNode troot_box{};          // its root box (padded)
    std::vector<RtPrim> prims;
    std::vector<RtMat> mats;
    std::vector<RtLight> lights;
    RtCamera cam{};
    int bvh_depth = 0;
    // Every primitive lies inside its own reference box (no negative / NaN
    // sphere radius, no slightly tilted plane given a thin axis box), so a
    // conservative culling test returns the reference's hit: fast traversal OK.
    bool fast_ok = true;
    std::vector<int32_t> prim_object;  // prim slot -> index in SceneData.objects
};

// createCameraFromSceneData(sceneData, renderOptions) restated
// (src/scenes/scenes.ts:60-104). Throws std::runtime_error with the reference's
// error message where the reference throws.
SceneBuild build_scene(const rtj::Value& scene_data, const rtj::Value* render_options);

// Scene generators (src/scenes/scenes-*.ts). `type` in {default, spheres, rain,
// cornell}; options as the reference's *SceneOptions object (may be null).
rtj::Value generate_scene_data(const std::string& type, const rtj::Value* options);

// Math.hypot as implemented by V8 (Kahan-summed, max-normalised).
double v8_hypot3(double x, double y, double z);

// mulberry32 SeededRandom.next() with JS double seed arithmetic
// (src/scenes/scenes-utils.ts:8-23).
struct SeededRandom {
    double seed;
    explicit SeededRandom(double s) : seed(s) {}
    double next();
};

}  // namespace rt
