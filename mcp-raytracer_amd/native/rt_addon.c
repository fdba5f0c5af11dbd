/* N-API addon: the binding df07/mcp-raytracer's TypeScript host loads instead of
 * building its object-model Camera.
 *
 * Replaces, one-for-one:
 *   createCameraFromSceneData(sceneData, renderOptions)  src/scenes/scenes.ts:60-104
 *   camera.renderRegion(buffer, region) -> RenderStats  src/camera.ts:388-431
 *   generateSceneData(sceneConfig)                      src/scenes/scenes.ts:42-50
 *   the parallel workers of generateImageBuffer         src/raytracer.ts:60-90,185-205
 *     (renderRegionMulti, renderPng's gpus: N GPUs from one call, rt_camera_render_multi)
 * through include/rt_amd.h. Errors are thrown as JS Errors carrying the same
 * messages the reference throws (rt_last_error()).
 *
 * Built in-tree against Node's node_api.h (raytracer_amd/_build.py build_addon),
 * linked to librt_amd.so next to it (rpath $ORIGIN). */
#include <node_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rt_amd.h"

#define CHECK_NAPI(env, call)                                      \
    do {                                                           \
        if ((call) != napi_ok) {                                   \
            napi_throw_error((env), NULL, "N-API call failed: " #call); \
            return NULL;                                           \
        }                                                          \
    } while (0)

static napi_value throw_rt(napi_env env) {
    napi_throw_error(env, NULL, rt_last_error());
    return NULL;
}

/* UTF-8 copy of a JS string argument (caller frees); NULL for undefined/null. */
static char* get_string(napi_env env, napi_value v) {
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok || t == napi_undefined || t == napi_null) return NULL;
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) return NULL;
    char* s = (char*)malloc(n + 1);
    if (!s) return NULL;
    napi_get_value_string_utf8(env, v, s, n + 1, &n);
    return s;
}

static void finalize_camera(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    rt_camera_destroy((rt_camera*)data);
}

/* generateSceneData(type: string, optionsJson?: string) -> string (SceneData JSON) */
static napi_value GenerateSceneData(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* type = argc > 0 ? get_string(env, argv[0]) : NULL;
    char* opts = argc > 1 ? get_string(env, argv[1]) : NULL;
    char* out = NULL;
    const int rc = rt_generate_scene_data(type ? type : "default", opts, &out);
    free(type);
    free(opts);
    if (rc) return throw_rt(env);
    napi_value s;
    const napi_status st = napi_create_string_utf8(env, out, NAPI_AUTO_LENGTH, &s);
    rt_free(out);
    if (st != napi_ok) return NULL;
    return s;
}

/* createCamera(sceneDataJson: string, renderOptionsJson?: string) -> External<rt_camera> */
static napi_value CreateCamera(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* scene = argc > 0 ? get_string(env, argv[0]) : NULL;
    char* opts = argc > 1 ? get_string(env, argv[1]) : NULL;
    rt_camera* cam = NULL;
    const int rc = rt_camera_create(scene ? scene : "", opts, &cam);
    free(scene);
    free(opts);
    if (rc) return throw_rt(env);
    napi_value ext;
    CHECK_NAPI(env, napi_create_external(env, cam, finalize_camera, NULL, &ext));
    return ext;
}

static rt_camera* get_camera(napi_env env, napi_value v) {
    void* p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "expected a camera created by createCamera");
        return NULL;
    }
    return (rt_camera*)p;
}

static void put_number(napi_env env, napi_value obj, const char* key, double v) {
    napi_value n;
    napi_create_double(env, v, &n);
    napi_set_named_property(env, obj, key, n);
}

/* cameraInfo(cam) -> { imageWidth, imageHeight, channels, objects, lights, traversal, precision } */
static napi_value CameraInfo(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rt_camera* cam = argc > 0 ? get_camera(env, argv[0]) : NULL;
    if (!cam) return NULL;
    rt_camera_info ci;
    if (rt_camera_get_info(cam, &ci)) return throw_rt(env);
    napi_value o;
    CHECK_NAPI(env, napi_create_object(env, &o));
    put_number(env, o, "imageWidth", ci.width);
    put_number(env, o, "imageHeight", ci.height);
    put_number(env, o, "channels", ci.channels);
    put_number(env, o, "objects", ci.n_objects);
    put_number(env, o, "lights", ci.n_lights);
    put_number(env, o, "traversal", ci.traversal);
    put_number(env, o, "precision", ci.precision);
    return o;
}

static int get_int_prop(napi_env env, napi_value obj, const char* key, int32_t* out) {
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return 0;
    double d = 0;
    if (napi_get_value_double(env, v, &d) != napi_ok) return 0;
    *out = (int32_t)d;
    return 1;
}

/* renderRegion(cam, buffer: Uint8ClampedArray | Uint8Array (width*height*3, may be
 * SharedArrayBuffer-backed), region: {x, y, width, height}) -> RenderStats
 * (src/render-utils/renderStats.ts:6-19 shape). Only the region is written. */
static napi_value stats_object(napi_env env, const rt_render_stats* s);

static napi_value RenderRegion(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 3) {
        napi_throw_type_error(env, NULL, "renderRegion(camera, buffer, region)");
        return NULL;
    }
    rt_camera* cam = get_camera(env, argv[0]);
    if (!cam) return NULL;
    bool is_ta = false;
    CHECK_NAPI(env, napi_is_typedarray(env, argv[1], &is_ta));
    if (!is_ta) {
        napi_throw_type_error(env, NULL, "buffer must be a Uint8ClampedArray");
        return NULL;
    }
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void* data = NULL;
    napi_value ab;
    CHECK_NAPI(env, napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &ab, &off));
    if (tt != napi_uint8_clamped_array && tt != napi_uint8_array) {
        napi_throw_type_error(env, NULL, "buffer must be a Uint8ClampedArray");
        return NULL;
    }
    rt_camera_info ci;
    if (rt_camera_get_info(cam, &ci)) return throw_rt(env);
    if (len < (size_t)ci.width * (size_t)ci.height * 3u) {
        napi_throw_range_error(env, NULL, "buffer is smaller than width*height*3");
        return NULL;
    }
    rt_region r;
    if (!get_int_prop(env, argv[2], "x", &r.x) || !get_int_prop(env, argv[2], "y", &r.y) ||
        !get_int_prop(env, argv[2], "width", &r.width) || !get_int_prop(env, argv[2], "height", &r.height)) {
        napi_throw_type_error(env, NULL, "region must be {x, y, width, height}");
        return NULL;
    }
    rt_render_stats s;
    if (rt_camera_render_region(cam, &r, (uint8_t*)data, NULL, &s)) return throw_rt(env);
    return stats_object(env, &s);
}

/* Device ordinals from a JS array of numbers, or 0..n-1 from a number n. Returns the count
 * (0 and a pending exception on a bad argument). */
static int32_t get_devices(napi_env env, napi_value v, int32_t* devs) {
    bool is_arr = false;
    if (napi_is_array(env, v, &is_arr) != napi_ok) return 0;
    if (!is_arr) {
        int32_t n = 0;
        if (napi_get_value_int32(env, v, &n) != napi_ok || n < 1 || n > RT_MAX_DEVICES) {
            napi_throw_range_error(env, NULL, "gpus must be 1..16 or an array of device ordinals");
            return 0;
        }
        for (int32_t g = 0; g < n; ++g) devs[g] = g;
        return n;
    }
    uint32_t n = 0;
    napi_get_array_length(env, v, &n);
    if (n < 1 || n > RT_MAX_DEVICES) {
        napi_throw_range_error(env, NULL, "devices must list 1..16 device ordinals");
        return 0;
    }
    for (uint32_t g = 0; g < n; ++g) {
        napi_value e;
        if (napi_get_element(env, v, g, &e) != napi_ok || napi_get_value_int32(env, e, &devs[g]) != napi_ok) {
            napi_throw_type_error(env, NULL, "devices must be numbers");
            return 0;
        }
    }
    return (int32_t)n;
}

/* renderRegionMulti(cam, buffer, region, gpus: number | number[]) -> RenderStats: renderRegion
 * over several GPUs from this one process (rt_camera_render_multi) - the reference's worker
 * fan-out (src/raytracer.ts:60-90, renderWorker.ts:17-35) with one call: tiles dealt over the
 * devices, gathered on the first over RCCL, stats merged as RenderStats.merge. */
static napi_value RenderRegionMulti(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 4) {
        napi_throw_type_error(env, NULL, "renderRegionMulti(camera, buffer, region, gpus)");
        return NULL;
    }
    rt_camera* cam = get_camera(env, argv[0]);
    if (!cam) return NULL;
    bool is_ta = false;
    CHECK_NAPI(env, napi_is_typedarray(env, argv[1], &is_ta));
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void* data = NULL;
    napi_value ab;
    if (is_ta) CHECK_NAPI(env, napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &ab, &off));
    if (!is_ta || (tt != napi_uint8_clamped_array && tt != napi_uint8_array)) {
        napi_throw_type_error(env, NULL, "buffer must be a Uint8ClampedArray");
        return NULL;
    }
    rt_camera_info ci;
    if (rt_camera_get_info(cam, &ci)) return throw_rt(env);
    if (len < (size_t)ci.width * (size_t)ci.height * 3u) {
        napi_throw_range_error(env, NULL, "buffer is smaller than width*height*3");
        return NULL;
    }
    rt_region r;
    if (!get_int_prop(env, argv[2], "x", &r.x) || !get_int_prop(env, argv[2], "y", &r.y) ||
        !get_int_prop(env, argv[2], "width", &r.width) || !get_int_prop(env, argv[2], "height", &r.height)) {
        napi_throw_type_error(env, NULL, "region must be {x, y, width, height}");
        return NULL;
    }
    int32_t devs[RT_MAX_DEVICES];
    const int32_t n = get_devices(env, argv[3], devs);
    if (n == 0) return NULL;
    rt_render_stats s;
    if (rt_camera_render_multi(cam, devs, n, &r, (uint8_t*)data, NULL, &s)) return throw_rt(env);
    return stats_object(env, &s);
}

/* RenderStats as the reference's object shape (src/render-utils/renderStats.ts:6-19). */
static napi_value stats_object(napi_env env, const rt_render_stats* sp) {
    const rt_render_stats s = *sp;
    napi_value out, sm, bo;
    CHECK_NAPI(env, napi_create_object(env, &out));
    CHECK_NAPI(env, napi_create_object(env, &sm));
    CHECK_NAPI(env, napi_create_object(env, &bo));
    put_number(env, out, "pixels", s.pixels);
    put_number(env, sm, "total", s.samples_total);
    put_number(env, sm, "min", s.samples_min);
    put_number(env, sm, "max", s.samples_max);
    put_number(env, sm, "avg", s.samples_avg);
    put_number(env, bo, "total", s.bounces_total);
    put_number(env, bo, "min", s.bounces_min);
    put_number(env, bo, "max", s.bounces_max);
    put_number(env, bo, "avg", s.bounces_avg);
    napi_set_named_property(env, out, "samples", sm);
    napi_set_named_property(env, out, "bounces", bo);
    return out;
}

static void finalize_free(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    rt_free(data);
}

/* encodePng(pixels: Uint8ClampedArray | Uint8Array (width*height*3), width, height) -> Buffer
 * (rt_encode_png: 8-bit RGB PNG): the step generateImageBuffer hands to sharp
 * (src/raytracer.ts:101-110). */
static napi_value EncodePng(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bool is_ta = false;
    if (argc < 3 || napi_is_typedarray(env, argv[0], &is_ta) != napi_ok || !is_ta) {
        napi_throw_type_error(env, NULL, "encodePng(pixels: Uint8ClampedArray, width, height)");
        return NULL;
    }
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void* data = NULL;
    napi_value ab;
    CHECK_NAPI(env, napi_get_typedarray_info(env, argv[0], &tt, &len, &data, &ab, &off));
    int32_t w = 0, h = 0;
    CHECK_NAPI(env, napi_get_value_int32(env, argv[1], &w));
    CHECK_NAPI(env, napi_get_value_int32(env, argv[2], &h));
    if ((tt != napi_uint8_clamped_array && tt != napi_uint8_array) || w <= 0 || h <= 0 ||
        len < (size_t)w * (size_t)h * 3u) {
        napi_throw_range_error(env, NULL, "pixels must hold width*height*3 bytes");
        return NULL;
    }
    uint8_t* png = NULL;
    size_t n = 0;
    if (rt_encode_png((const uint8_t*)data, w, h, 6, &png, &n)) return throw_rt(env);
    napi_value buf;
    CHECK_NAPI(env, napi_create_external_buffer(env, n, png, finalize_free, NULL, &buf));
    return buf;
}

/* renderPng(camera, bands, gpus?) -> {png: Buffer, stats}: generateImageBuffer's core
 * (src/raytracer.ts:39-113) on the device - `bands` is the reference's worker split
 * (the frame and its merged stats do not depend on it: one launch), the PNG encoded on
 * the GPU (rt_camera_render_png) so only the compressed file crosses PCIe. `gpus` (a count
 * or an array of device ordinals) renders the frame over several GPUs of this process
 * (rt_camera_render_png_multi). */
static napi_value RenderPng(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 1) {
        napi_throw_type_error(env, NULL, "renderPng(camera, bands, gpus?)");
        return NULL;
    }
    rt_camera* cam = get_camera(env, argv[0]);
    if (!cam) return NULL;
    int32_t bands = 1;
    if (argc > 1) CHECK_NAPI(env, napi_get_value_int32(env, argv[1], &bands));
    int32_t devs[RT_MAX_DEVICES];
    int32_t ndev = 0;
    if (argc > 2) {
        napi_valuetype t;
        CHECK_NAPI(env, napi_typeof(env, argv[2], &t));
        if (t != napi_undefined && t != napi_null && (ndev = get_devices(env, argv[2], devs)) == 0) return NULL;
    }
    uint8_t* png = NULL;
    size_t n = 0;
    rt_render_stats s;
    if (ndev > 0 ? rt_camera_render_png_multi(cam, devs, ndev, &s, &png, &n)
                 : rt_camera_render_png(cam, bands, &s, &png, &n))
        return throw_rt(env);
    napi_value out, buf;
    CHECK_NAPI(env, napi_create_object(env, &out));
    CHECK_NAPI(env, napi_create_external_buffer(env, n, png, finalize_free, NULL, &buf));
    napi_set_named_property(env, out, "png", buf);
    napi_set_named_property(env, out, "stats", stats_object(env, &s));
    return out;
}

static napi_value Version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value v;
    napi_create_int32(env, rt_version(), &v);
    return v;
}

static napi_value Init(napi_env env, napi_value exports) {
    napi_property_descriptor d[] = {
        {"generateSceneData", NULL, GenerateSceneData, NULL, NULL, NULL, napi_default, NULL},
        {"createCamera", NULL, CreateCamera, NULL, NULL, NULL, napi_default, NULL},
        {"cameraInfo", NULL, CameraInfo, NULL, NULL, NULL, napi_default, NULL},
        {"renderRegion", NULL, RenderRegion, NULL, NULL, NULL, napi_default, NULL},
        {"renderRegionMulti", NULL, RenderRegionMulti, NULL, NULL, NULL, napi_default, NULL},
        {"encodePng", NULL, EncodePng, NULL, NULL, NULL, napi_default, NULL},
        {"renderPng", NULL, RenderPng, NULL, NULL, NULL, napi_default, NULL},
        {"version", NULL, Version, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
