// Host side of the drop-in: SceneData -> flat device arrays, plus the scene
// generators that produce the benchmark inputs.
//
// Each function cites the reference code it restates. Vector quantities are
// fp32 (gl-matrix Float32Array), scalars are doubles, exactly as the reference.
#include "scene.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace rt {

namespace {

using rtj::Value;

constexpr double kPI = 3.141592653589793;  // Math.PI

[[noreturn]] void fail(const std::string& msg) { throw std::runtime_error(msg); }

// ---------------------------------------------------------------------------
// JS value helpers
// ---------------------------------------------------------------------------

// ToNumber for the JSON-representable JS values we accept.
double to_number(const Value* v, double dflt) {
    if (!v) return dflt;  // property absent -> default parameter / undefined handling by caller
    switch (v->kind) {
        case Value::Number: return v->num;
        case Value::Bool: return v->b ? 1.0 : 0.0;
        case Value::Null: return 0.0;
        case Value::String: {
            const char* s = v->str.c_str();
            char* e = nullptr;
            double d = std::strtod(s, &e);
            while (e && (*e == ' ' || *e == '\t' || *e == '\n')) ++e;
            if (v->str.empty()) return 0.0;
            return (e && *e == '\0') ? d : NAN;
        }
        default: return NAN;
    }
}

bool truthy(const Value* v) {
    if (!v) return false;
    switch (v->kind) {
        case Value::Null: return false;
        case Value::Bool: return v->b;
        case Value::Number: return !(v->num == 0.0 || std::isnan(v->num));
        case Value::String: return !v->str.empty();
        default: return true;
    }
}

std::string js_string(const Value* v) {
    if (!v) return "undefined";
    switch (v->kind) {
        case Value::Null: return "null";
        case Value::Bool: return v->b ? "true" : "false";
        case Value::String: return v->str;
        case Value::Number: { std::string s; rtj::dump_number(s, v->num); return s; }
        case Value::Object: return "[object Object]";
        case Value::Array: {
            std::string s;
            for (size_t i = 0; i < v->arr.size(); ++i) { if (i) s += ","; s += js_string(&v->arr[i]); }
            return s;
        }
    }
    return "";
}

// Vec3.create(...array): spread of a 3-array into Float32Array stores
// (missing entries are undefined -> NaN). Non-iterables throw a TypeError.
V3 vec_from(const Value* v, const char* what) {
    if (!v || !v->is_array()) fail(std::string(what) + " is not iterable");
    double c[3] = {NAN, NAN, NAN};
    for (size_t i = 0; i < 3 && i < v->arr.size(); ++i) c[i] = to_number(&v->arr[i], NAN);
    return mk<double>(c[0], c[1], c[2]);
}

}  // namespace

// ---------------------------------------------------------------------------
// V8 Math.hypot (used by gl-matrix vec3.length)
// ---------------------------------------------------------------------------
double v8_hypot3(double x, double y, double z) {
    double vals[3] = {x, y, z};
    double absv[3] = {0, 0, 0};
    bool nan = false;
    double mx = 0;
    for (int i = 0; i < 3; ++i) {
        if (std::isnan(vals[i])) { nan = true; continue; }
        absv[i] = std::fabs(vals[i]);
        if (absv[i] > mx) mx = absv[i];
    }
    if (mx == INFINITY) return INFINITY;
    if (nan) return NAN;
    if (mx == 0) return 0;
    double sum = 0, comp = 0;
    for (int i = 0; i < 3; ++i) {
        double n = absv[i] / mx;
        double summand = n * n - comp;
        double prelim = sum + summand;
        comp = (prelim - sum) - summand;
        sum = prelim;
    }
    return std::sqrt(sum) * mx;
}

static double vlength(V3 a) { return v8_hypot3(a.x, a.y, a.z); }

// ---------------------------------------------------------------------------
// mulberry32 (src/scenes/scenes-utils.ts:8-23) with JS number semantics: the
// seed is a double that grows without wrapping; bit ops see ToInt32/ToUint32.
// ---------------------------------------------------------------------------
static int32_t js_to_int32(double d) {
    if (!std::isfinite(d)) return 0;
    double t = std::trunc(d);
    double m = std::fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    return (int32_t)(uint32_t)m;
}
static int32_t js_imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

double SeededRandom::next() {
    seed += 1831565813.0;  // 0x6D2B79F5
    int32_t t = js_to_int32(seed);
    t = js_imul(t ^ (int32_t)((uint32_t)t >> 15), t | 1);
    double s = (double)t + (double)js_imul(t ^ (int32_t)((uint32_t)t >> 7), t | 61);
    t ^= js_to_int32(s);
    uint32_t r = (uint32_t)(t ^ (int32_t)((uint32_t)t >> 14));
    return (double)r / 4294967296.0;
}

// ---------------------------------------------------------------------------
// Scene generators
// ---------------------------------------------------------------------------
namespace {

double opt_num(const Value* opts, const char* key, double dflt) {
    const Value* v = opts ? opts->get(key) : nullptr;
    return v ? to_number(v, dflt) : dflt;
}

std::vector<double> opt_vec3(const Value* opts, const char* key, std::vector<double> dflt) {
    const Value* v = opts ? opts->get(key) : nullptr;
    if (!v || !v->is_array()) return dflt;
    std::vector<double> out(3, NAN);
    for (size_t i = 0; i < 3 && i < v->arr.size(); ++i) out[i] = to_number(&v->arr[i], NAN);
    return out;
}

double default_seed() {
    // Math.floor(Math.random() * 2147483647): an unseeded scene, as in the reference.
    std::random_device rd;
    return std::floor(((double)rd() / 4294967296.0) * 2147483647.0);
}

Value material_entry(const std::string& id, Value material) {
    Value m = Value::object();
    m.set("id", Value::string(id));
    m.set("material", std::move(material));
    return m;
}

Value lambert(double r, double g, double b) {
    Value m = Value::object();
    m.set("type", Value::string("lambert"));
    m.set("color", rtj::vec3(r, g, b));
    return m;
}

Value camera_data(double vfov, double aperture, double focus, std::vector<double> from,
                  std::vector<double> at, std::vector<double> top, std::vector<double> bottom) {
    Value cam = Value::object();
    cam.set("vfov", Value::number(vfov));
    cam.set("aperture", Value::number(aperture));
    cam.set("focus", Value::number(focus));
    cam.set("from", rtj::vec3(from[0], from[1], from[2]));
    cam.set("at", rtj::vec3(at[0], at[1], at[2]));
    cam.set("up", rtj::vec3(0, 1, 0));
    Value bg = Value::object();
    bg.set("type", Value::string("gradient"));
    bg.set("top", rtj::vec3(top[0], top[1], top[2]));
    bg.set("bottom", rtj::vec3(bottom[0], bottom[1], bottom[2]));
    cam.set("background", std::move(bg));
    return cam;
}

Value metadata(const std::string& name, const std::string& desc) {
    Value md = Value::object();
    md.set("name", Value::string(name));
    md.set("description", Value::string(desc));
    md.set("version", Value::string("2.0"));
    return md;
}

std::string num_str(double v) { std::string s; rtj::dump_number(s, v); return s; }

// generateSpheresSceneData (src/scenes/scenes-spheres.ts:27-119). The overlap
// test (checkOverlap, 124-137) is the same predicate evaluated against a uniform
// grid of cell size 2r instead of the whole list, so large counts finish.
Value gen_spheres(const Value* opts) {
    const double count = opt_num(opts, "count", 10);
    const std::vector<double> centerPoint = opt_vec3(opts, "centerPoint", {0, 0, -2});
    const double distRadius = opt_num(opts, "radius", 1.25);
    const double minSphereRadius = opt_num(opts, "minSphereRadius", 0.1);
    const double maxSphereRadius = opt_num(opts, "maxSphereRadius", 0.2);
    const Value* seedv = opts ? opts->get("seed") : nullptr;
    const double seed = seedv ? to_number(seedv, 0) : default_seed();

    SeededRandom random(seed);
    const double scaleFactor = js_max<double>(minSphereRadius, 1 - std::log10(count + 1) / 4);
    const double adjustedMaxRadius = maxSphereRadius * scaleFactor;

    Value materials = Value::array();
    Value objects = Value::array();

    struct Placed { double c[3]; double r; };
    std::vector<Placed> placed;

    // Uniform grid over the placement ball for the overlap query.
    const double cell = std::max(2.0 * std::fabs(adjustedMaxRadius), 1e-9);
    const double lo[3] = {centerPoint[0] - distRadius - cell, centerPoint[1] - distRadius - cell,
                          centerPoint[2] - distRadius - cell};
    const double span = 2 * distRadius + 2 * cell;
    const bool use_grid = std::isfinite(span / cell) && span / cell < 1024 && count > 64;
    const int gdim = use_grid ? (int)std::ceil(span / cell) + 1 : 0;
    std::unordered_map<int64_t, std::vector<int>> grid;
    auto cell_of = [&](const double* c, int a) { return (int)std::floor((c[a] - lo[a]) / cell); };
    auto key_of = [&](int ix, int iy, int iz) { return ((int64_t)ix * gdim + iy) * gdim + iz; };

    auto overlaps = [&](const double* c, double radius) {
        auto test = [&](const Placed& s) {
            const double dx = c[0] - s.c[0], dy = c[1] - s.c[1], dz = c[2] - s.c[2];
            const double distance = std::sqrt(dx * dx + dy * dy + dz * dz);
            return distance < (radius + s.r);
        };
        if (!use_grid) {
            for (const Placed& s : placed) if (test(s)) return true;
            return false;
        }
        const int ix = cell_of(c, 0), iy = cell_of(c, 1), iz = cell_of(c, 2);
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dz = -1; dz <= 1; ++dz) {
                    auto it = grid.find(key_of(ix + dx, iy + dy, iz + dz));
                    if (it == grid.end()) continue;
                    for (int k : it->second) if (test(placed[k])) return true;
                }
        return false;
    };

    double attempts = 0;
    const double maxAttempts = count * 100;
    double spheresCreated = 0;
    while (spheresCreated < count && attempts < maxAttempts) {
        attempts++;
        const double radius = adjustedMaxRadius;
        // randomPointInSphere (141-157): SeededRandom.randomInUnitSphere stores fp32.
        V3 p;
        while (true) {
            double x = -1 + 2 * random.next();
            double y = -1 + 2 * random.next();
            double z = -1 + 2 * random.next();
            p = mk<double>(x, y, z);
            if (len2<double>(p) < 1) break;
        }
        const double distanceFactor = std::pow(random.next(), 1.0 / 3.0) * distRadius;
        double c[3] = {centerPoint[0] + (double)p.x * distanceFactor,
                       centerPoint[1] + (double)p.y * distanceFactor,
                       centerPoint[2] + (double)p.z * distanceFactor};
        if (overlaps(c, radius)) continue;

        const std::string materialId = "sphere-" + num_str(spheresCreated);
        // generateRandomMaterialData (162-182)
        Value mat = Value::object();
        const double materialType = random.next();
        if (materialType < 0.6) {
            double r = random.next(), g = random.next(), b = random.next();
            mat = lambert(r, g, b);
        } else if (materialType < 0.9) {
            const double fuzz = random.next() * 0.5;
            double r = random.next(), g = random.next(), b = random.next();
            mat.set("type", Value::string("metal"));
            mat.set("color", rtj::vec3(r, g, b));
            mat.set("fuzz", Value::number(fuzz));
        } else {
            const double ior = 1.3 + random.next() * 1.2;
            mat.set("type", Value::string("glass"));
            mat.set("ior", Value::number(ior));
        }
        materials.push(material_entry(materialId, std::move(mat)));

        Value obj = Value::object();
        obj.set("type", Value::string("sphere"));
        obj.set("pos", rtj::vec3(c[0], c[1], c[2]));
        obj.set("r", Value::number(radius));
        obj.set("material", Value::string(materialId));
        objects.push(std::move(obj));

        placed.push_back(Placed{{c[0], c[1], c[2]}, radius});
        if (use_grid)
            grid[key_of(cell_of(c, 0), cell_of(c, 1), cell_of(c, 2))].push_back((int)placed.size() - 1);
        spheresCreated++;
    }

    Value scene = Value::object();
    scene.set("camera", camera_data(40, 0.0, 1.0, {0, 0, 2}, centerPoint, {0.5, 0.7, 1.0}, {1.0, 1.0, 1.0}));
    scene.set("materials", std::move(materials));
    scene.set("objects", std::move(objects));
    scene.set("metadata", metadata("Random Spheres", "Scene with " + num_str(spheresCreated) +
                                                         " randomly placed spheres (seed: " + num_str(seed) + ")"));
    return scene;
}

// generateRainSceneData (src/scenes/scenes-rain.ts:19-145)
Value gen_rain(const Value* opts) {
    const double count = opt_num(opts, "count", 50);
    const double sphereRadius = opt_num(opts, "sphereRadius", 0.05);
    const double width = opt_num(opts, "width", 4);
    const double height = opt_num(opts, "height", 3);
    const double depth = opt_num(opts, "depth", 2);
    const std::vector<double> centerPoint = opt_vec3(opts, "centerPoint", {0, 0, -2});
    const double metalFuzz = opt_num(opts, "metalFuzz", 0.1);
    const bool groundSphere = opts && opts->get("groundSphere") ? truthy(opts->get("groundSphere")) : true;
    const double groundY = opt_num(opts, "groundY", -100.5);
    const double groundRadius = opt_num(opts, "groundRadius", 100);
    const Value* seedv = opts ? opts->get("seed") : nullptr;
    const double seed = seedv ? to_number(seedv, 0) : default_seed();

    SeededRandom random(seed);
    Value materials = Value::array();
    Value objects = Value::array();
    if (groundSphere) materials.push(material_entry("ground", lambert(0.1, 0.1, 0.1)));
    if (groundSphere) {
        Value g = Value::object();
        g.set("type", Value::string("sphere"));
        g.set("pos", rtj::vec3(0, groundY, 0));
        g.set("r", Value::number(groundRadius));
        g.set("material", Value::string("ground"));
        objects.push(std::move(g));
    }
    const double spd = std::ceil(std::pow(count, 1.0 / 3.0));
    const double xSpacing = width / spd, ySpacing = height / spd, zSpacing = depth / spd;
    const double totalW = spd * xSpacing, totalH = spd * ySpacing, totalD = spd * zSpacing;
    const double startX = centerPoint[0] - totalW / 2 + xSpacing / 2;
    const double startY = centerPoint[1] - totalH / 2 + ySpacing / 2;
    const double startZ = centerPoint[2] - totalD / 2 + zSpacing / 2;

    std::vector<std::array<double, 3>> positions;
    const long n = spd > 0 && std::isfinite(spd) ? (long)spd : 0;
    for (long x = 0; x < n; x++)
        for (long y = 0; y < n; y++)
            for (long z = 0; z < n; z++) {
                double px = startX + x * xSpacing + (random.next() - 0.5) * xSpacing * 0.3;
                double py = startY + y * ySpacing + (random.next() - 0.5) * ySpacing * 0.3;
                double pz = startZ + z * zSpacing + (random.next() - 0.5) * zSpacing * 0.3;
                positions.push_back({px, py, pz});
            }
    // shuffleArray: Fisher-Yates (152-158)
    for (long i = (long)positions.size() - 1; i > 0; i--) {
        long j = (long)std::floor(random.next() * (double)(i + 1));
        std::swap(positions[i], positions[j]);
    }
    const long take = std::min<long>((long)positions.size(), count > 0 ? (long)std::ceil(count) : 0);
    for (long i = 0; i < take; i++) {
        const auto& pos = positions[i];
        const double brightness = 0.7 + random.next() * 0.3;
        const double fuzz = metalFuzz * random.next();
        const std::string materialId = "rain-" + std::to_string(i);
        Value mat = Value::object();
        mat.set("type", Value::string("metal"));
        mat.set("color", rtj::vec3(brightness, brightness, brightness));
        mat.set("fuzz", Value::number(fuzz));
        materials.push(material_entry(materialId, std::move(mat)));
        Value obj = Value::object();
        obj.set("type", Value::string("sphere"));
        obj.set("pos", rtj::vec3(pos[0], pos[1], pos[2]));
        obj.set("r", Value::number(sphereRadius));
        obj.set("material", Value::string(materialId));
        objects.push(std::move(obj));
    }
    Value scene = Value::object();
    scene.set("camera", camera_data(40, 0.0, 1.0, {0, 0, 2}, centerPoint, {0.5, 0.7, 1.0}, {1.0, 1.0, 1.0}));
    scene.set("materials", std::move(materials));
    scene.set("objects", std::move(objects));
    scene.set("metadata", metadata("Rain Scene", "Scene with " + std::to_string(take) +
                                                     " metallic rain spheres (seed: " + num_str(seed) + ")"));
    return scene;
}

Value quad_obj(std::vector<double> pos, std::vector<double> u, std::vector<double> v, const char* mat) {
    Value o = Value::object();
    o.set("type", Value::string("quad"));
    o.set("pos", rtj::vec3(pos[0], pos[1], pos[2]));
    o.set("u", rtj::vec3(u[0], u[1], u[2]));
    o.set("v", rtj::vec3(v[0], v[1], v[2]));
    o.set("material", Value::string(mat));
    return o;
}

Value sphere_obj(std::vector<double> pos, double r, const char* mat) {
    Value o = Value::object();
    o.set("type", Value::string("sphere"));
    o.set("pos", rtj::vec3(pos[0], pos[1], pos[2]));
    o.set("r", Value::number(r));
    o.set("material", Value::string(mat));
    return o;
}

// generateCornellSceneData (src/scenes/scenes-cornell.ts:19-134)
Value gen_cornell(const Value* opts) {
    const Value* vv = opts ? opts->get("variant") : nullptr;
    const std::string variant = (vv && vv->is_string()) ? vv->str : "spheres";
    const bool spheres = variant == "spheres";
    const double boxSize = 2.0, halfSize = boxSize / 2;
    Value materials = Value::array();
    materials.push(material_entry("red", lambert(0.65, 0.05, 0.05)));
    materials.push(material_entry("green", lambert(0.12, 0.45, 0.15)));
    materials.push(material_entry("white", lambert(0.73, 0.73, 0.73)));
    {
        Value l = Value::object();
        l.set("type", Value::string("light"));
        l.set("emit", rtj::vec3(15, 15, 15));
        materials.push(material_entry("light", std::move(l)));
    }
    if (spheres) {
        materials.push(material_entry("sphere-white", lambert(0.6, 0.6, 0.6)));
        Value g = Value::object();
        g.set("type", Value::string("glass"));
        g.set("ior", Value::number(1.5));
        materials.push(material_entry("sphere-glass", std::move(g)));
    }
    Value objects = Value::array();
    const double h = halfSize;
    objects.push(quad_obj({-h, -h, -h}, {0, boxSize, 0}, {0, 0, boxSize}, "red"));
    objects.push(quad_obj({h, -h, h}, {0, boxSize, 0}, {0, 0, -boxSize}, "green"));
    objects.push(quad_obj({-h, -h, -h}, {boxSize, 0, 0}, {0, boxSize, 0}, "white"));
    objects.push(quad_obj({-h, -h, -h}, {boxSize, 0, 0}, {0, 0, boxSize}, "white"));
    objects.push(quad_obj({-h, h, h}, {boxSize, 0, 0}, {0, 0, -boxSize}, "white"));
    const double lightSize = boxSize * 0.3;
    {
        Value l = quad_obj({-lightSize / 2, halfSize - 0.01, -lightSize / 2}, {lightSize, 0, 0},
                           {0, 0, lightSize}, "light");
        l.set("light", Value::boolean(true));
        objects.push(std::move(l));
    }
    if (spheres) {
        const double sphereRadius = 0.3;
        objects.push(sphere_obj({-halfSize * 0.4, -halfSize + sphereRadius, -halfSize * 0.3}, sphereRadius,
                                "sphere-white"));
        objects.push(sphere_obj({halfSize * 0.4, -halfSize + sphereRadius, halfSize * 0.3}, sphereRadius,
                                "sphere-glass"));
    }
    Value scene = Value::object();
    scene.set("camera", camera_data(40, 0.0, 1.0, {0, 0, halfSize * 4}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}));
    Value render = Value::object();
    render.set("aspect", Value::number(1.0));
    render.set("roulette", Value::boolean(true));
    render.set("rouletteDepth", Value::number(5));
    scene.set("render", std::move(render));
    scene.set("materials", std::move(materials));
    scene.set("objects", std::move(objects));
    scene.set("metadata",
              metadata("Cornell Box (" + variant + ")",
                       std::string("Cornell box scene with ") + (spheres ? "two spheres inside" : "empty interior")));
    return scene;
}

// generateDefaultSceneData (src/scenes/scenes-default.ts:8-82)
Value gen_default() {
    Value materials = Value::array();
    materials.push(material_entry("ground", lambert(0.4, 0.4, 0.0)));
    materials.push(material_entry("blue", lambert(0.1, 0.1, 0.9)));
    {
        Value g = Value::object();
        g.set("type", Value::string("glass"));
        g.set("ior", Value::number(1.5));
        materials.push(material_entry("glass", std::move(g)));
    }
    auto metal = [](double r, double g, double b, double fuzz) {
        Value m = Value::object();
        m.set("type", Value::string("metal"));
        m.set("color", rtj::vec3(r, g, b));
        m.set("fuzz", Value::number(fuzz));
        return m;
    };
    materials.push(material_entry("silver", metal(0.8, 0.8, 0.8, 0.0)));
    materials.push(material_entry("gold", metal(0.8, 0.6, 0.2, 0.5)));
    {
        Value lay = Value::object();
        lay.set("type", Value::string("layered"));
        Value outer = Value::object();
        outer.set("type", Value::string("glass"));
        outer.set("ior", Value::number(1.5));
        lay.set("outer", std::move(outer));
        lay.set("inner", lambert(0.7, 0.3, 0.3));
        materials.push(material_entry("layered-paint", std::move(lay)));
    }
    {
        Value l = Value::object();
        l.set("type", Value::string("light"));
        l.set("emit", rtj::vec3(15.0, 14.0, 13.0));
        materials.push(material_entry("sun-light", std::move(l)));
    }
    Value objects = Value::array();
    {
        Value p = Value::object();
        p.set("type", Value::string("plane"));
        p.set("pos", rtj::vec3(0, 0, 0));
        p.set("u", rtj::vec3(1, 0, 0));
        p.set("v", rtj::vec3(0, 0, 1));
        p.set("material", Value::string("ground"));
        objects.push(std::move(p));
    }
    objects.push(sphere_obj({0, 0.5, -1}, 0.5, "layered-paint"));
    objects.push(sphere_obj({-1, 0.5, -1}, 0.5, "silver"));
    objects.push(sphere_obj({1, 0.5, -1}, 0.5, "gold"));
    objects.push(sphere_obj({0.5, 0.25, -0.5}, 0.25, "glass"));
    objects.push(sphere_obj({-0.5, 0.25, -0.5}, 0.25, "glass"));
    objects.push(sphere_obj({-0.5, 0.25, -0.5}, -.24, "glass"));
    objects.push(sphere_obj({-0.5, 0.25, -0.5}, 0.20, "blue"));
    {
        Value l = quad_obj({-2, 3, 0}, {1, 0, 0}, {0, -0.707, -0.707}, "sun-light");
        l.set("light", Value::boolean(true));
        objects.push(std::move(l));
    }
    {
        Value s = sphere_obj({30, 30.5, 15}, 10, "sun-light");
        s.set("light", Value::boolean(true));
        objects.push(std::move(s));
    }
    Value scene = Value::object();
    scene.set("camera", camera_data(40, 0.05, 2.8, {0, 0.75, 2}, {0, 0.5, -1}, {1, 1, 1}, {0.5, 0.7, 1.0}));
    scene.set("materials", std::move(materials));
    scene.set("objects", std::move(objects));
    scene.set("metadata", metadata("Default Scene",
                                   "A scene with various spheres demonstrating different materials including "
                                   "layered, mixed, and basic materials"));
    return scene;
}

}  // namespace

Value generate_scene_data(const std::string& type, const Value* options) {
    // generateSceneData (src/scenes/scenes.ts:42-50)
    if (type == "default") return gen_default();
    if (type == "spheres") return gen_spheres(options);
    if (type == "rain") return gen_rain(options);
    if (type == "cornell") return gen_cornell(options);
    fail("Unknown scene type: " + type);
}

// ---------------------------------------------------------------------------
// createCameraFromSceneData (src/scenes/scenes.ts:60-104)
// ---------------------------------------------------------------------------
namespace {

struct Box {
    V3 mn, mx;
};

// AABB.surroundingBox (src/geometry/aabb.ts:68-82)
Box surrounding(const Box& a, const Box& b) {
    return Box{mk<double>(js_min<double>(a.mn.x, b.mn.x), js_min<double>(a.mn.y, b.mn.y), js_min<double>(a.mn.z, b.mn.z)),
               mk<double>(js_max<double>(a.mx.x, b.mx.x), js_max<double>(a.mx.y, b.mx.y), js_max<double>(a.mx.z, b.mx.z))};
}

Box empty_box() { return Box{mk<double>(INFINITY, INFINITY, INFINITY), mk<double>(-INFINITY, -INFINITY, -INFINITY)}; }

float comp(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

struct Builder {
    const Value& scene;
    std::unordered_map<std::string, const Value*> matmap;
    SceneBuild out;
    std::vector<Box> boxes;  // per object

    explicit Builder(const Value& s) : scene(s) {}

    int add_mat(RtMat m) {
        out.mats.push_back(m);
        return (int)out.mats.size() - 1;
    }

    const Value* resolve(const Value* ref) {
        if (ref && ref->is_string()) {
            auto it = matmap.find(ref->str);
            return it == matmap.end() ? nullptr : it->second;
        }
        if (!ref || ref->is_null()) return nullptr;
        if (ref->is_bool() && !ref->b) return nullptr;
        if (ref->is_number() && (ref->num == 0 || std::isnan(ref->num))) return nullptr;
        return ref;
    }

    // createMaterial (src/scenes/scenes.ts:144-180). Returns a material index.
    int create_material(const Value* ref) {
        const Value* md = resolve(ref);
        if (!md) fail("Material not found: " + js_string(ref));
        const Value* tv = md->get("type");
        const std::string type = tv && tv->is_string() ? tv->str : js_string(tv);
        RtMat m{};
        m.c0 = m.c1 = -1;
        if (type == "lambert") {
            m.type = MAT_LAMBERT;
            V3 c = vec_from(md->get("color"), "materialData.color");
            m.color[0] = c.x; m.color[1] = c.y; m.color[2] = c.z;
        } else if (type == "metal") {
            m.type = MAT_METAL;
            V3 c = vec_from(md->get("color"), "materialData.color");
            m.color[0] = c.x; m.color[1] = c.y; m.color[2] = c.z;
            // Metal ctor: fuzz default 0.0; fuzz < 1 ? Math.max(0, fuzz) : 1 (src/materials/metal.ts:20)
            const Value* fv = md->get("fuzz");
            double fuzz = fv ? to_number(fv, 0.0) : 0.0;
            m.p0 = fuzz < 1 ? js_max<double>(0, fuzz) : 1;
        } else if (type == "glass") {
            m.type = MAT_GLASS;
            m.p0 = to_number(md->get("ior"), NAN);
        } else if (type == "light") {
            m.type = MAT_LIGHT;
            V3 c = vec_from(md->get("emit"), "materialData.emit");
            m.color[0] = c.x; m.color[1] = c.y; m.color[2] = c.z;
        } else if (type == "mixed") {
            m.type = MAT_MIXED;
            m.c0 = create_material(md->get("diff"));
            m.c1 = create_material(md->get("spec"));
            // weight = Math.max(0.0, Math.min(1.0, weight)) (src/materials/mixedMaterial.ts:29)
            m.p0 = js_max<double>(0.0, js_min<double>(1.0, to_number(md->get("weight"), NAN)));
        } else if (type == "layered") {
            m.type = MAT_LAYERED;
            // createDielectric (src/scenes/scenes.ts:182-199) runs before the inner material.
            const Value* oref = md->get("outer");
            const Value* od = resolve(oref);
            if (!od) fail("Material not found: " + js_string(oref));
            const Value* otv = od->get("type");
            if (!(otv && otv->is_string() && otv->str == "glass"))
                fail("Material is not a dielectric: " + js_string(oref));
            RtMat g{};
            g.type = MAT_GLASS;
            g.c0 = g.c1 = -1;
            g.p0 = to_number(od->get("ior"), NAN);
            m.c0 = add_mat(g);
            m.c1 = create_material(md->get("inner"));
        } else {
            fail("Unknown material type: " + type);
        }
        return add_mat(m);
    }

    // Material.emitted(rec) is a constant per material: DefaultMaterial -> BLACK,
    // DiffuseLight -> emit, Mixed -> E1*w + E2*(1-w), Layered -> inner's.
    V3 emitted_of(int mi) {
        const RtMat& m = out.mats[mi];
        switch (m.type) {
            case MAT_LIGHT: return v3(m.color[0], m.color[1], m.color[2]);
            case MAT_MIXED: {
                V3 e1 = scale<double>(emitted_of(m.c0), m.p0);
                V3 e2 = scale<double>(emitted_of(m.c1), 1.0 - m.p0);
                return add(e1, e2);
            }
            case MAT_LAYERED: return emitted_of(m.c1);
            default: return v3(0, 0, 0);
        }
    }
    bool can_scatter(int mi) {
        const RtMat& m = out.mats[mi];
        if (m.type == MAT_LIGHT) return false;
        if (m.type == MAT_MIXED) return can_scatter(m.c0) || can_scatter(m.c1);
        return true;
    }

    // Plane ctor (src/entities/plane.ts:180-200) + boxes (plane.ts:276-308,
    // quad.ts:400-422); Sphere ctor (sphere.ts:20-31).
    // Axis-aligned quad (u, v each along one axis): the kernel evaluates the
    // reference's Plane.intersect / alpha / beta with the zero terms dropped,
    // which rounds identically (pt_kernel.hpp aquad_t). Encoding:
    //   g4[3] = int code 1 + a + 3*vflag (a = normal axis; vflag: v along (a+2)%3),
    //   g3[3] = +-w[a] (sign folded from the cross product), g2[3] = v's nonzero
    //   component, g1[3] = u's nonzero component. code 0 = general quad.
    static void encode_axis_quad(RtPrim& p, V3 u, V3 v, V3 cp, V3 w) {
        const float uu[3] = {u.x, u.y, u.z}, vv[3] = {v.x, v.y, v.z}, cc[3] = {cp.x, cp.y, cp.z},
                    ww[3] = {w.x, w.y, w.z};
        auto only = [](const float* x) {
            int k = -1;
            for (int i = 0; i < 3; ++i) {
                if (!std::isfinite(x[i])) return -2;
                if (x[i] != 0.0f) k = (k == -1) ? i : -2;
            }
            return k;
        };
        const int iu = only(uu), iv = only(vv), a = only(cc), iw = only(ww);
        if (iu < 0 || iv < 0 || a < 0 || iw != a || iu == iv || iu == a || iv == a) return;
        const int b = (a + 1) % 3, c = (a + 2) % 3;
        const bool vflag = iv == c;  // then u is along b
        if (!(vflag ? iu == b : (iv == b && iu == c))) return;
        int32_t code = 1 + a + 3 * (vflag ? 1 : 0);
        std::memcpy(&p.g4[3], &code, sizeof code);
        p.g3[3] = vflag ? ww[a] : -ww[a];
        p.g2[3] = vv[iv];
        p.g1[3] = uu[iu];
    }

    RtPrim make_prim(const Value& od, int mat, Box& box, std::string& type_out) {
        RtPrim p{};
        p.mat = mat;
        const Value* tv = od.get("type");
        const std::string type = tv && tv->is_string() ? tv->str : js_string(tv);
        type_out = type;
        if (type == "sphere") {
            p.type = PRIM_SPHERE;
            V3 c = vec_from(od.get("pos"), "objectData.pos");
            double r = to_number(od.get("r"), NAN);
            p.s0 = r;
            p.g0[0] = c.x; p.g0[1] = c.y; p.g0[2] = c.z; p.g0[3] = (float)r;
            {  // reciprocal radius for the hit normal (kernel sphere_inv_radius)
                const double ir = 1.0 / r;
                std::memcpy(&p.g1[0], &ir, sizeof ir);
                const float irf = 1.0f / (float)r;
                p.g1[2] = irf;
            }
            V3 rv = mk<double>(r, r, r);
            box = Box{sub(c, rv), add(c, rv)};
            return p;
        }
        if (type == "plane" || type == "quad") {
            p.type = type == "plane" ? PRIM_PLANE : PRIM_QUAD;
            V3 q = vec_from(od.get("pos"), "objectData.pos");
            V3 u = vec_from(od.get("u"), "objectData.u");
            V3 v = vec_from(od.get("v"), "objectData.v");
            V3 cp = cross<double>(u, v);
            V3 n = unit<double>(cp);
            double d = dot<double>(n, q);
            double cl2 = len2<double>(cp);
            V3 w = divs<double>(cp, cl2);
            p.s0 = d;
            p.g0[0] = q.x; p.g0[1] = q.y; p.g0[2] = q.z; p.g0[3] = (float)d;
            p.g1[0] = u.x; p.g1[1] = u.y; p.g1[2] = u.z;
            p.g2[0] = v.x; p.g2[1] = v.y; p.g2[2] = v.z;
            p.g3[0] = n.x; p.g3[1] = n.y; p.g3[2] = n.z;
            p.g4[0] = w.x; p.g4[1] = w.y; p.g4[2] = w.z;
            // general quads: |w||u|, |w||v| (rounded up) scale the kernel's alpha/beta
            // error margins (pt_kernel.hpp planar_maybe); axis quads re-use the slots
            {
                const double wn = std::sqrt(len2<double>(w));
                p.g1[3] = (float)(wn * std::sqrt(len2<double>(u)) * (1.0 + 1e-5));
                p.g2[3] = (float)(wn * std::sqrt(len2<double>(v)) * (1.0 + 1e-5));
            }
            if (p.type == PRIM_QUAD) encode_axis_quad(p, u, v, cp, w);
            if (p.type == PRIM_PLANE) {
                const double eps = 1e-4;
                if (std::fabs((double)n.x) > 0.9999) {
                    double px = d / (double)n.x;
                    box = Box{mk<double>(px - eps, -INFINITY, -INFINITY), mk<double>(px + eps, INFINITY, INFINITY)};
                } else if (std::fabs((double)n.y) > 0.9999) {
                    double py = d / (double)n.y;
                    box = Box{mk<double>(-INFINITY, py - eps, -INFINITY), mk<double>(INFINITY, py + eps, INFINITY)};
                } else if (std::fabs((double)n.z) > 0.9999) {
                    double pz = d / (double)n.z;
                    box = Box{mk<double>(-INFINITY, -INFINITY, pz - eps), mk<double>(INFINITY, INFINITY, pz + eps)};
                } else {
                    box = Box{mk<double>(-INFINITY, -INFINITY, -INFINITY), mk<double>(INFINITY, INFINITY, INFINITY)};
                }
            } else {
                V3 v1 = q, v2 = add(q, u), v3_ = add(q, v), v4 = add(add(q, u), v);
                auto mn4 = [](double a, double b, double c, double e) {
                    return js_min<double>(js_min<double>(js_min<double>(a, b), c), e);
                };
                auto mx4 = [](double a, double b, double c, double e) {
                    return js_max<double>(js_max<double>(js_max<double>(a, b), c), e);
                };
                const double eps = 1e-4;
                double mnx = mn4(v1.x, v2.x, v3_.x, v4.x), mny = mn4(v1.y, v2.y, v3_.y, v4.y),
                       mnz = mn4(v1.z, v2.z, v3_.z, v4.z);
                double mxx = mx4(v1.x, v2.x, v3_.x, v4.x), mxy = mx4(v1.y, v2.y, v3_.y, v4.y),
                       mxz = mx4(v1.z, v2.z, v3_.z, v4.z);
                box = Box{mk<double>(mnx - eps, mny - eps, mnz - eps), mk<double>(mxx + eps, mxy + eps, mxz + eps)};
            }
            return p;
        }
        fail("Unknown object type: " + type);
    }

    // BVHNode ctor (src/geometry/bvh.ts:34-102). `list` is this node's
    // objectsList. Array.prototype.sort with the comparator
    // (a,b) => boxA.min[axis] < boxB.min[axis] ? -1 : 1 is V8's TimSort, which
    // only ever calls the comparator as (later element, earlier element); with
    // this comparator that makes ties keep input order, i.e. a stable sort.
    int build(std::vector<int> list, int depth, Box& node_box) {
        out.bvh_depth = std::max(out.bvh_depth, depth);
        Box nb = boxes[list[0]];
        for (size_t k = 1; k < list.size(); ++k) nb = surrounding(nb, boxes[list[k]]);
        const double xe = (double)nb.mx.x - (double)nb.mn.x;
        const double ye = (double)nb.mx.y - (double)nb.mn.y;
        const double ze = (double)nb.mx.z - (double)nb.mn.z;
        int axis = 0;
        if (ye > xe && ye > ze) axis = 1;
        else if (ze > xe && ze > ye) axis = 2;
        const size_t span = list.size();

        const int self = (int)out.nodes.size();
        out.nodes.push_back(RtNode{});
        auto less = [&](int a, int b) { return comp(boxes[a].mn, axis) < comp(boxes[b].mn, axis); };

        Box box;
        if (span <= 4) {
            std::vector<int> leaf;
            if (span == 1) {
                leaf = {list[0]};
                box = surrounding(boxes[list[0]], empty_box());
            } else if (span == 2) {
                if (less(list[0], list[1])) leaf = {list[0], list[1]};
                else leaf = {list[1], list[0]};
                box = surrounding(boxes[leaf[0]], boxes[leaf[1]]);
            } else {
                leaf = list;
                // HittableList.boundingBox (src/geometry/hittableList.ts:29-52)
                Box lb = boxes[leaf[0]];
                for (size_t k = 1; k < leaf.size(); ++k) lb = surrounding(lb, boxes[leaf[k]]);
                box = surrounding(lb, empty_box());
            }
            RtNode& n = out.nodes[self];
            n.a = (int32_t)out.prims.size();
            n.b = -(int32_t)leaf.size();
            for (int o : leaf) {
                out.prims.push_back(tmp_prims[o]);
                out.prim_object.push_back(o);
            }
        } else {
            std::stable_sort(list.begin(), list.end(), less);
            const size_t mid = span / 2;
            std::vector<int> l(list.begin(), list.begin() + mid), r(list.begin() + mid, list.end());
            Box lbx, rbx;
            int li = build(std::move(l), depth + 1, lbx);
            int ri = build(std::move(r), depth + 1, rbx);
            out.nodes[self].a = li;
            out.nodes[self].b = ri;
            box = surrounding(lbx, rbx);
        }
        RtNode& n = out.nodes[self];
        n.bmin[0] = box.mn.x; n.bmin[1] = box.mn.y; n.bmin[2] = box.mn.z;
        n.bmax[0] = box.mx.x; n.bmax[1] = box.mx.y; n.bmax[2] = box.mx.z;
        node_box = box;
        return self;
    }

    std::vector<RtPrim> tmp_prims;
};

// Spread-merge lookup: provided render options win over the scene's (scenes.ts:97-100).
const Value* render_opt(const Value* scene_render, const Value* provided, const char* key) {
    if (provided && provided->is_object()) {
        if (const Value* v = provided->get(key)) return v;
    }
    if (scene_render && scene_render->is_object()) {
        if (const Value* v = scene_render->get(key)) return v;
    }
    return nullptr;
}

int32_t loop_threshold(double x) {
    // Smallest integer n with (n >= x) for integer counters starting at 0.
    if (std::isnan(x)) return INT32_MAX;
    if (x <= 0) return 0;
    if (x > 1e9) return 1000000000;
    return (int32_t)std::ceil(x);
}

}  // namespace

// Boxes for the fast traversal (pt_kernel.hpp closest_hit_fast). The
// reference's AABB.hit never accepts a box that is inverted or flat on an
// axis (its per-axis interval is empty), and always accepts one with a NaN
// bound; a strict slab test would treat those differently, so they are
// encoded as "always reject" (NaN in bmin[0]) and "always accept" (infinite
// box). Every other box is padded outward by ~1e-6 relative, so the fp32
// slab test can never cull a box the exact primitive tests would hit.
std::vector<RtNode> make_fast_nodes(const std::vector<RtNode>& nodes) {
    std::vector<RtNode> out(nodes);
    for (RtNode& n : out) {
        bool nan = false, empty = false;
        for (int a = 0; a < 3; ++a) {
            if (std::isnan(n.bmin[a]) || std::isnan(n.bmax[a])) nan = true;
            else if (!(n.bmin[a] < n.bmax[a])) empty = true;
        }
        if (nan) {
            for (int a = 0; a < 3; ++a) { n.bmin[a] = -INFINITY; n.bmax[a] = INFINITY; }
        } else if (empty) {
            n.bmin[0] = NAN;
        } else {
            for (int a = 0; a < 3; ++a) {
                const double lo = n.bmin[a], hi = n.bmax[a];
                if (std::isfinite(lo)) n.bmin[a] = std::nextafter((float)(lo - 1e-6 * (1.0 + std::fabs(lo))), -INFINITY);
                if (std::isfinite(hi)) n.bmax[a] = std::nextafter((float)(hi + 1e-6 * (1.0 + std::fabs(hi))), INFINITY);
            }
        }
    }
    return out;
}

// fnodes (DFS order, node 0 = root) re-laid out as RtTNode: interior nodes get
// TNode slots in DFS order and carry both children's boxes.
std::vector<RtTNode> make_tnodes(const std::vector<RtNode>& f, int32_t& root_ref) {
    std::vector<int32_t> tidx(f.size(), -1);
    int32_t nt = 0;
    for (size_t i = 0; i < f.size(); ++i)
        if (f[i].b >= 0) tidx[i] = nt++;
    auto ref = [&](int32_t i) -> int32_t {
        if (f[i].b >= 0) return tidx[i];
        const int32_t count = -f[i].b;
        if (count < 1 || count > 7 || f[i].a >= (1 << 27)) throw std::runtime_error("BVH leaf does not fit the TNode code");
        return ~((f[i].a << 3) | count);
    };
    std::vector<RtTNode> out((size_t)nt);
    for (size_t i = 0; i < f.size(); ++i) {
        if (f[i].b < 0) continue;
        RtTNode& t = out[(size_t)tidx[i]];
        const int32_t ch[2] = {f[i].a, f[i].b};
        for (int k = 0; k < 2; ++k) {
            t.box[k] = f[(size_t)ch[k]];
            t.box[k].a = ref(ch[k]);
            t.box[k].b = 0;
        }
    }
    root_ref = f.empty() ? ~0 : ref(0);
    return out;
}

// The padded binary tree (DFS, node 0 = root) collapsed to 4-wide nodes: each
// 4-node takes a binary node's two children and keeps replacing its largest
// interior child by that child's two children until it holds four. Boxes are
// the binary tree's (padded) boxes, so every primitive stays inside each box on
// its path; boxes the reference can never enter (NaN-marked) become empty slots.
static int32_t t4_leaf_ref(const RtNode& n) {
    const int32_t count = -n.b;
    if (count < 1 || count > 7 || n.a >= (1 << 27)) throw std::runtime_error("BVH leaf does not fit the TNode code");
    return ~((n.a << 3) | count);
}
static double t4_area(const RtNode& n) {
    double e[3];
    for (int a = 0; a < 3; ++a) {
        e[a] = (double)n.bmax[a] - (double)n.bmin[a];
        if (!(e[a] >= 0) || !std::isfinite(e[a])) e[a] = 1e30;
    }
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
}
static int32_t t4_build(const std::vector<RtNode>& f, int32_t i, int depth, std::vector<RtT4Node>& out, int& max_depth) {
    max_depth = std::max(max_depth, depth);
    std::vector<int32_t> ch = {f[(size_t)i].a, f[(size_t)i].b};
    while (ch.size() < 4) {
        int best = -1;
        double best_a = -1.0;
        for (size_t k = 0; k < ch.size(); ++k) {
            const RtNode& c = f[(size_t)ch[k]];
            if (c.b >= 0 && !std::isnan(c.bmin[0]) && t4_area(c) > best_a) { best_a = t4_area(c); best = (int)k; }
        }
        if (best < 0) break;
        const RtNode c = f[(size_t)ch[(size_t)best]];
        ch[(size_t)best] = c.a;
        ch.insert(ch.begin() + best + 1, c.b);
    }
    const int32_t idx = (int32_t)out.size();
    out.push_back(RtT4Node{});
    for (int k = 0; k < 4; ++k) {
        RtT4Node& t = out[(size_t)idx];
        for (int a = 0; a < 3; ++a) { t.bmin[a][k] = NAN; t.bmax[a][k] = NAN; }
        t.ref[k] = kT4Empty;
        t.pad[k] = 0;
    }
    for (size_t k = 0; k < ch.size(); ++k) {
        const RtNode& c = f[(size_t)ch[k]];
        if (std::isnan(c.bmin[0])) continue;  // the reference never enters it: no hit below
        const int32_t r = c.b >= 0 ? t4_build(f, ch[k], depth + 1, out, max_depth) : t4_leaf_ref(c);
        RtT4Node& t = out[(size_t)idx];
        for (int a = 0; a < 3; ++a) { t.bmin[a][k] = c.bmin[a]; t.bmax[a][k] = c.bmax[a]; }
        t.ref[k] = r;
    }
    return idx;
}
// The 4-wide nodes re-numbered breadth-first (root 0, then its children, ...): any prefix of
// the array is the top of the tree - the nodes every ray's walk starts with - which a launch
// walking the tree from global memory copies into LDS (pt_kernel.hpp t4_node). The walk's
// result does not depend on node numbering (the (t, slot) minimum).
static std::vector<RtT4Node> t4_breadth_first(const std::vector<RtT4Node>& in) {
    std::vector<int32_t> order, idx(in.size(), -1);
    order.reserve(in.size());
    order.push_back(0);
    idx[0] = 0;
    for (size_t h = 0; h < order.size(); ++h)
        for (int k = 0; k < 4; ++k) {
            const int32_t r = in[(size_t)order[h]].ref[k];
            if (r >= 0) {  // interior child (leaf codes and empty slots are negative)
                idx[(size_t)r] = (int32_t)order.size();
                order.push_back(r);
            }
        }
    if (order.size() != in.size()) throw std::runtime_error("4-wide tree: unreachable nodes");
    std::vector<RtT4Node> out(in.size());
    for (size_t i = 0; i < order.size(); ++i) {
        RtT4Node n = in[(size_t)order[i]];
        for (int k = 0; k < 4; ++k)
            if (n.ref[k] >= 0) n.ref[k] = idx[(size_t)n.ref[k]];
        out[i] = n;
    }
    return out;
}

std::vector<RtT4Node> make_t4nodes(const std::vector<RtNode>& f, int32_t& root_ref, int& depth) {
    std::vector<RtT4Node> out;
    depth = 0;
    if (f.empty()) { root_ref = ~0; return out; }
    if (f[0].b < 0) { root_ref = t4_leaf_ref(f[0]); return out; }
    root_ref = t4_build(f, 0, 1, out, depth);  // the root is node 0 (pre-order)
    if (out.size() >= (1u << 24)) throw std::runtime_error("4-wide tree: more than 2^24 nodes");  // (t4_node: 24-bit multiply)
    return t4_breadth_first(out);
}

// ---------------------------------------------------------------------------
// Fast-traversal tree built for speed, not for the reference's visiting order:
// the fast traversal returns the (t, slot) minimum over all primitives, so any
// tree whose boxes enclose their primitives gives the reference's hit. Binned
// SAH (16 bins on the longest centroid axis, leaves of <= 4), falling back to
// median splits where the depth would outgrow the LDS traversal stack. Leaves
// index `order` (-> SceneBuild::tprims), i.e. reference leaf slots.
// ---------------------------------------------------------------------------
struct SahBuilder {
    const std::vector<Box>& pbox;  // per slot
    std::vector<int32_t> order;
    std::vector<RtNode> nodes;     // DFS, RtNode conventions (leaf: a = first, b = -count)
    int cap;                       // maximum depth (root = 1)
    int depth_seen = 0;
    // SAH constants: cost of a traversal step relative to one primitive test, the largest leaf
    // the cost rule may keep, and the size below which a node is always a leaf (defaults 1, 4, 2;
    // RT_AMD_SAH_CT / RT_AMD_SAH_MAXLEAF / RT_AMD_SAH_FORCELEAF override, for A/B)
    // One primitive per leaf where the walk tests a leaf's primitives exactly as it reaches them
    // (no deferred exact tests, pt_kernel.hpp leaf_test): trees too large for the LDS-resident copy
    // (> 1,024 primitives: every leaf costs an L2 round trip for its records and its pre-filter loop
    // runs at the lanes that hold it; spheres-100k 2048^2 spp16 with the fp64 leaf records: leaves
    // <= 4: 33.6 ms, <= 2: 32.1, 1: 30.1) and small ones (< 100 primitives; rain-50 1080p spp128:
    // 11.09 -> 10.91 ms). LDS-resident trees of 100 .. 1,024 primitives run the deferred exact tests
    // (rt_api.cpp v.defer), whose leaf loop is cheap per primitive: they keep <= 4 / 2 (spheres-500:
    // leaves of 1 5.72 -> 5.76 ms, of <= 2 7.27 ms) (profiles/r05/sah/).
    bool one_leaf = pbox.size() > 1024 || pbox.size() < 100;
    double trav_cost = env_double("RT_AMD_SAH_CT", 1.0);
    int max_leaf = std::min(7, std::max(1, (int)env_double("RT_AMD_SAH_MAXLEAF", one_leaf ? 1 : 4)));
    int force_leaf = std::min(max_leaf, std::max(1, (int)env_double("RT_AMD_SAH_FORCELEAF", one_leaf ? 1 : 2)));
    static double env_double(const char* name, double dflt) {
        const char* e = std::getenv(name);
        return (e && e[0]) ? std::atof(e) : dflt;
    }

    SahBuilder(const std::vector<Box>& b, int cap_) : pbox(b), cap(cap_) {
        order.resize(b.size());
        for (size_t i = 0; i < b.size(); ++i) order[i] = (int32_t)i;
    }
    static double area(const Box& b) {
        const double dx = (double)b.mx.x - b.mn.x, dy = (double)b.mx.y - b.mn.y, dz = (double)b.mx.z - b.mn.z;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
    static Box merge(const Box& a, const Box& b) {
        return Box{v3(std::min(a.mn.x, b.mn.x), std::min(a.mn.y, b.mn.y), std::min(a.mn.z, b.mn.z)),
                   v3(std::max(a.mx.x, b.mx.x), std::max(a.mx.y, b.mx.y), std::max(a.mx.z, b.mx.z))};
    }
    static float cen(const Box& b, int a) { return 0.5f * (comp(b.mn, a) + comp(b.mx, a)); }

    int build(int begin, int end, int depth) {
        depth_seen = std::max(depth_seen, depth);
        const int idx = (int)nodes.size();
        nodes.push_back(RtNode{});
        Box bb = pbox[(size_t)order[(size_t)begin]];
        Box cb{v3(INFINITY, INFINITY, INFINITY), v3(-INFINITY, -INFINITY, -INFINITY)};
        for (int i = begin; i < end; ++i) {
            const Box& b = pbox[(size_t)order[(size_t)i]];
            bb = merge(bb, b);
            const V3 c = v3(cen(b, 0), cen(b, 1), cen(b, 2));
            cb = merge(cb, Box{c, c});
        }
        auto set_box = [&](RtNode& n) {
            n.bmin[0] = bb.mn.x; n.bmin[1] = bb.mn.y; n.bmin[2] = bb.mn.z;
            n.bmax[0] = bb.mx.x; n.bmax[1] = bb.mx.y; n.bmax[2] = bb.mx.z;
        };
        const int count = end - begin;
        auto make_leaf = [&]() {
            RtNode& n = nodes[(size_t)idx];
            set_box(n);
            n.a = begin;
            n.b = -count;
            return idx;
        };
        if (count <= force_leaf) return make_leaf();
        int axis = 0;
        float ext[3] = {cb.mx.x - cb.mn.x, cb.mx.y - cb.mn.y, cb.mx.z - cb.mn.z};
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        int mid = -1;
        const int need = (int)std::ceil(std::log2(std::max(1.0, count / (double)max_leaf)));
        if (ext[axis] > 0.0f && depth + need + 2 < cap) {
            constexpr int kBins = 16;
            Box binb[kBins];
            int binn[kBins] = {0};
            const float lo = comp(cb.mn, axis), scale = kBins / ext[axis];
            auto bin_of = [&](const Box& b) {
                int k = (int)((cen(b, axis) - lo) * scale);
                return std::min(std::max(k, 0), kBins - 1);
            };
            for (int i = begin; i < end; ++i) {
                const Box& b = pbox[(size_t)order[(size_t)i]];
                const int k = bin_of(b);
                binb[k] = binn[k] ? merge(binb[k], b) : b;
                ++binn[k];
            }
            double best = INFINITY;
            int best_k = -1;
            for (int k = 1; k < kBins; ++k) {  // split between bin k-1 and k
                Box lb{}, rb{};
                int ln = 0, rn = 0;
                for (int q = 0; q < k; ++q) if (binn[q]) { lb = ln ? merge(lb, binb[q]) : binb[q]; ln += binn[q]; }
                for (int q = k; q < kBins; ++q) if (binn[q]) { rb = rn ? merge(rb, binb[q]) : binb[q]; rn += binn[q]; }
                if (!ln || !rn) continue;
                const double c = area(lb) * ln + area(rb) * rn;
                if (c < best) { best = c; best_k = k; }
            }
            const double leaf_cost = (double)count;
            const double split_cost = trav_cost + best / std::max(area(bb), 1e-30);
            if (count <= max_leaf && !(split_cost < leaf_cost)) return make_leaf();
            if (best_k > 0) {
                auto it = std::partition(order.begin() + begin, order.begin() + end,
                                         [&](int32_t s) { return bin_of(pbox[(size_t)s]) < best_k; });
                mid = (int)(it - order.begin());
                if (mid == begin || mid == end) mid = -1;
            }
        }
        if (mid < 0) {  // median split by centroid (balanced; also for coincident centroids)
            if (count <= max_leaf) return make_leaf();
            mid = begin + count / 2;
            std::nth_element(order.begin() + begin, order.begin() + mid, order.begin() + end, [&](int32_t x, int32_t y) {
                const float cx = cen(pbox[(size_t)x], axis), cy = cen(pbox[(size_t)y], axis);
                return cx < cy || (cx == cy && x < y);
            });
        }
        const int l = build(begin, mid, depth + 1);
        const int r = build(mid, end, depth + 1);
        RtNode& n = nodes[(size_t)idx];
        set_box(n);
        n.a = l;
        n.b = r;
        return idx;
    }
};

// The fast traversal is exact only if no primitive can be hit outside the box
// the reference gives it: a negative-radius sphere (inverted box, e.g. the
// default scene's hollow glass), a NaN bound, or a plane whose normal passes
// the 0.9999 axis test without being exactly axis-aligned (thin slab box around
// a tilted plane, src/entities/plane.ts:280-307). Such scenes use the
// reference-order traversal.
bool prims_inside_boxes(const std::vector<RtPrim>& prims) {
    for (const RtPrim& p : prims) {
        for (int k = 0; k < 4; ++k) {
            if (std::isnan(p.g0[k])) return false;
            // a sphere's g1 holds its reciprocal radius (double bits), its g2..g4 are unused
            if (p.type != PRIM_SPHERE &&
                (std::isnan(p.g1[k]) || std::isnan(p.g2[k]) || std::isnan(p.g3[k]) || std::isnan(p.g4[k])))
                return false;
        }
        if (std::isnan(p.s0)) return false;
        if (p.type == PRIM_SPHERE) {
            if (!(p.s0 > 0) || !std::isfinite(p.s0)) return false;
        } else if (p.type == PRIM_PLANE) {
            const double n[3] = {p.g3[0], p.g3[1], p.g3[2]};
            for (int a = 0; a < 3; ++a) {
                if (std::fabs(n[a]) > 0.9999) {
                    const bool exact = std::fabs(n[a]) == 1.0 && n[(a + 1) % 3] == 0.0 && n[(a + 2) % 3] == 0.0;
                    if (!exact) return false;
                    break;
                }
            }
        }
    }
    return true;
}

SceneBuild build_scene(const Value& scene_data, const Value* render_options) {
    if (!scene_data.is_object()) fail("sceneData must be an object");
    Builder b(scene_data);

    // materials lookup: sceneData.materials?.forEach(({id, material}) => ...)
    if (const Value* mats = scene_data.get("materials")) {
        if (mats->is_array()) {
            for (const Value& e : mats->arr) {
                const Value* id = e.get("id");
                const Value* m = e.get("material");
                b.matmap[js_string(id)] = m;
            }
        }
    }
    const Value* objs = scene_data.get("objects");
    if (!objs || !objs->is_array()) fail("Cannot read properties of undefined (reading 'map')");
    const size_t nobj = objs->arr.size();
    if (nobj == 0) fail("Cannot read properties of null (reading 'maximum')");  // BVHNode over an empty list

    b.boxes.resize(nobj);
    b.tmp_prims.resize(nobj);
    std::vector<std::string> types(nobj);
    for (size_t i = 0; i < nobj; ++i) {
        const Value& od = objs->arr[i];
        int mat = b.create_material(od.get("material"));
        b.tmp_prims[i] = b.make_prim(od, mat, b.boxes[i], types[i]);
    }
    // emitted constants + emissive-scatter flag
    int emissive_scatter = 0;
    for (size_t mi = 0; mi < b.out.mats.size(); ++mi) {
        V3 e = b.emitted_of((int)mi);
        RtMat& m = b.out.mats[mi];
        m.emitted[0] = e.x; m.emitted[1] = e.y; m.emitted[2] = e.z;
        bool nz = !(e.x == 0.0f && e.y == 0.0f && e.z == 0.0f);
        if (nz && b.can_scatter((int)mi)) emissive_scatter = 1;
    }

    // world = BVHNode.fromList(objects)
    std::vector<int> all(nobj);
    for (size_t i = 0; i < nobj; ++i) all[i] = (int)i;
    Box root_box;
    b.build(all, 1, root_box);

    // lights: objData.light && 'pdf' in object  (Sphere and Quad are PDFHittable)
    std::vector<int> slot_of(nobj);
    for (size_t s = 0; s < b.out.prim_object.size(); ++s) slot_of[b.out.prim_object[s]] = (int)s;
    for (size_t i = 0; i < nobj; ++i) {
        const Value& od = objs->arr[i];
        if (!truthy(od.get("light"))) continue;
        if (types[i] != "sphere" && types[i] != "quad") continue;
        RtLight l{};
        l.prim = slot_of[i];
        l.type = types[i] == "sphere" ? PRIM_SPHERE : PRIM_QUAD;
        if (l.type == PRIM_QUAD) {
            const RtPrim& p = b.tmp_prims[i];
            V3 u = v3(p.g1[0], p.g1[1], p.g1[2]), v = v3(p.g2[0], p.g2[1], p.g2[2]);
            l.area = vlength(cross<double>(u, v));  // Quad.area = u.cross(v).length()
        }
        b.out.lights.push_back(l);
    }

    // Camera (src/camera.ts:107-166) with createCameraFromSceneData's option mapping
    const Value* camd = scene_data.get("camera");
    if (!camd || !camd->is_object()) fail("Cannot read properties of undefined (reading 'vfov')");
    RtCamera& cam = b.out.cam;

    const Value* vfv = camd->get("vfov");
    const double vfov = vfv ? to_number(vfv, NAN) : NAN;  // undefined overrides the default
    if (!truthy(camd->get("from"))) fail("Cannot read properties of undefined (reading 'subtract')");
    if (!truthy(camd->get("at"))) fail("Cannot read properties of undefined (reading 'glVec')");
    if (!truthy(camd->get("up"))) fail("Cannot read properties of undefined (reading 'cross')");
    const V3 from = vec_from(camd->get("from"), "camera.from");
    const V3 at = vec_from(camd->get("at"), "camera.at");
    const V3 up = vec_from(camd->get("up"), "camera.up");
    const Value* apv = camd->get("aperture");
    const double aperture = apv ? to_number(apv, NAN) : NAN;
    const Value* fov = camd->get("focus");
    const double focus = fov ? to_number(fov, NAN) : NAN;
    const Value* bgv = camd->get("background");
    const bool has_bg = truthy(bgv);
    V3 bg_top{0, 0, 0}, bg_bottom{0, 0, 0};
    if (has_bg) {
        bg_top = vec_from(bgv->get("top"), "camera.background.top");
        bg_bottom = vec_from(bgv->get("bottom"), "camera.background.bottom");
    }

    // render options: {...defaultRenderData, ...sceneData.render, ...renderOptions}
    const Value* srender = scene_data.get("render");
    auto ropt = [&](const char* key) { return render_opt(srender, render_options, key); };
    const double width = ropt("width") ? to_number(ropt("width"), NAN) : 400;
    const double aspect = ropt("aspect") ? to_number(ropt("aspect"), NAN) : 16.0 / 9.0;
    const double samples = ropt("samples") ? to_number(ropt("samples"), NAN) : 100;
    const double depth = ropt("depth") ? to_number(ropt("depth"), NAN) : 100;
    const double aTol = ropt("aTolerance") ? to_number(ropt("aTolerance"), NAN) : 0.05;
    const double aBatch = ropt("aBatch") ? to_number(ropt("aBatch"), NAN) : 10;
    const bool roulette = ropt("roulette") ? truthy(ropt("roulette")) : true;
    const double rdepth = ropt("rouletteDepth") ? to_number(ropt("rouletteDepth"), NAN) : 3;
    std::string mode = "default";
    if (const Value* mv = ropt("mode")) mode = js_string(mv);
    const Value* sv = ropt("seed");
    const double seed = sv ? to_number(sv, 0) : (double)0x5EED;

    const double imageHeight = std::ceil(width / aspect);
    if (!(width >= 0) || width != std::floor(width) || width > 1e6 || !(imageHeight >= 0) || imageHeight > 1e6)
        fail("Invalid typed array length: image " + num_str(width) + "x" + num_str(imageHeight));
    if (std::isnan(depth)) fail("Maximum call stack size exceeded (depth is NaN)");

    const double focusDistance = (focus != 0 && !std::isnan(focus)) ? focus : vlength(sub(from, at));
    const double theta = vfov * (kPI / 180);
    const double h = std::tan(theta / 2);
    const double viewportHeight = 2 * h * focusDistance;
    const double aspectRatio = width / imageHeight;
    const double viewportWidth = viewportHeight * aspectRatio;
    const V3 w = unit<double>(sub(from, at));
    const V3 u = unit<double>(cross<double>(up, w));
    const V3 v = cross<double>(w, u);
    const V3 viewportU = scale<double>(u, viewportWidth);
    const V3 viewportV = scale<double>(v, -viewportHeight);
    const V3 pdu = divs<double>(viewportU, width);
    const V3 pdv = divs<double>(viewportV, imageHeight);
    const V3 halfU = divs<double>(viewportU, 2.0);
    const V3 halfV = divs<double>(viewportV, 2.0);
    const V3 upperLeft = sub(sub(sub(from, scale<double>(w, focusDistance)), halfU), halfV);
    const V3 p00 = add(upperLeft, scale<double>(add(pdu, pdv), 0.5));
    const V3 ddu = scale<double>(u, aperture / 2);
    const V3 ddv = scale<double>(v, aperture / 2);

    auto put = [](float* d, V3 s) { d[0] = s.x; d[1] = s.y; d[2] = s.z; d[3] = 0; };
    put(cam.pixel00, p00);
    put(cam.du, pdu);
    put(cam.dv, pdv);
    put(cam.center, from);
    put(cam.ddu, ddu);
    put(cam.ddv, ddv);
    put(cam.bg_top, bg_top);
    put(cam.bg_bottom, bg_bottom);
    cam.aperture = aperture;
    cam.samples = samples;
    cam.a_tolerance = aTol;
    cam.a_batch = aBatch;
    cam.depth_raw = depth;
    cam.width = (int32_t)width;
    cam.height = (int32_t)imageHeight;
    cam.n_samples = loop_threshold(samples);
    if (cam.n_samples == INT32_MAX) cam.n_samples = 0;  // NaN samples: the while loop never runs
    cam.depth = loop_threshold(depth);
    cam.roulette = roulette ? 1 : 0;
    cam.roulette_depth = loop_threshold(rdepth);
    cam.mode = mode == "bounces" ? MODE_BOUNCES : (mode == "samples" ? MODE_SAMPLES : MODE_DEFAULT);
    cam.adaptive = (aTol > 0 && samples > 1) ? 1 : 0;
    cam.n_lights = (int32_t)b.out.lights.size();
    cam.has_background = has_bg ? 1 : 0;
    cam.emissive_scatter = emissive_scatter;
    cam.n_nodes = (int32_t)b.out.nodes.size();
    cam.n_prims = (int32_t)b.out.prims.size();
    cam.n_mats = (int32_t)b.out.mats.size();
    cam.seed = (uint32_t)(int64_t)seed;
    cam.seed_mix = splitmix64(cam.seed);
    b.out.fnodes = make_fast_nodes(b.out.nodes);
    // fast-traversal tree: SAH over the reference's per-object boxes (finite boxes
    // only, i.e. no planes), else the reference tree itself
    {
        std::vector<Box> slot_box(b.out.prims.size());
        bool finite = true;
        for (size_t k = 0; k < slot_box.size(); ++k) {
            slot_box[k] = b.boxes[(size_t)b.out.prim_object[k]];
            const Box& x = slot_box[k];
            for (float v : {x.mn.x, x.mn.y, x.mn.z, x.mx.x, x.mx.y, x.mx.z})
                if (!std::isfinite(v)) finite = false;
            if (!(x.mn.x <= x.mx.x && x.mn.y <= x.mx.y && x.mn.z <= x.mx.z)) finite = false;
        }
        const char* env = std::getenv("RT_AMD_SAH");
        const bool sah = finite && slot_box.size() > 16 && !(env && env[0] == '0');
        if (sah) {
            SahBuilder sb(slot_box, std::max(b.out.bvh_depth + 2, 12));
            sb.build(0, (int)slot_box.size(), 1);
            b.out.tprims = sb.order;
            const std::vector<RtNode> padded = make_fast_nodes(sb.nodes);
            b.out.tnodes = make_tnodes(padded, b.out.troot);
            b.out.t4nodes = make_t4nodes(padded, b.out.t4root, b.out.t4depth);
            b.out.troot_box = padded[0];
            b.out.tdepth = sb.depth_seen;
        } else {
            b.out.tprims.resize(b.out.prims.size());
            for (size_t k = 0; k < b.out.tprims.size(); ++k) b.out.tprims[k] = (int32_t)k;
            b.out.tnodes = make_tnodes(b.out.fnodes, b.out.troot);
            b.out.t4nodes = make_t4nodes(b.out.fnodes, b.out.t4root, b.out.t4depth);
            b.out.troot_box = b.out.fnodes[0];
            b.out.tdepth = b.out.bvh_depth;
        }
        b.out.tprims.resize((b.out.tprims.size() + 3) / 4 * 4, 0);  // 16-byte blob sections
        // leaf-order sphere records for the fp32 pre-filter: contiguous per leaf and
        // a quarter of a primitive record, so large scenes stay cache-resident
        b.out.tsph.assign(b.out.tprims.size() * 4, std::numeric_limits<float>::quiet_NaN());
        b.out.tsph2.assign(b.out.tprims.size(), RtLeafSph{});
        for (size_t m = 0; m < b.out.tprims.size(); ++m) {
            const RtPrim& p = b.out.prims[(size_t)b.out.tprims[m]];
            RtLeafSph& q = b.out.tsph2[m];
            q.slot = b.out.tprims[m];
            for (int c = 0; c < 3; ++c) q.c[c] = std::numeric_limits<float>::quiet_NaN();
            q.r32 = std::numeric_limits<float>::quiet_NaN();
            if (p.type == PRIM_SPHERE) {
                for (int c = 0; c < 4; ++c) b.out.tsph[m * 4 + c] = p.g0[c];
                for (int c = 0; c < 3; ++c) q.c[c] = p.g0[c];
                q.r32 = p.g0[3];
                q.r64 = p.s0;  // the JS double radius (sphere_radius<double>)
            }
        }
    }
    // stack entries: reference DFS (depth + 1), binary fast tree (depth + 1),
    // 4-wide tree (up to 3 pushes per level + 1). The 4-wide node step (pt_kernel.hpp t4_step)
    // writes up to sp + 2 whatever it pushes: at a node of level L the stack holds at most
    // 3 (L - 1) entries, so its writes stay below 3 t4depth entries - inside this bound.
    cam.stack_depth = std::max(b.out.bvh_depth, 3 * b.out.t4depth + 1) + 1;
    b.out.fast_ok = prims_inside_boxes(b.out.prims);
    return std::move(b.out);
}

}  // namespace rt
