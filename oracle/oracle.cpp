// oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h for the rules and pinning status).
//
// A plain C++ restatement of isaac-chandler/cuda-raytracer, written from the reference source
// text (never compiled or linked against it).  Every function cites the reference lines it
// follows.  Arithmetic conventions (shared by contract with the HIP kernels, restated there
// independently):
//   * IEEE fp32/fp64, no contraction (-ffp-contract=off), no fast-math, no FTZ.
//   * min/max on floats are C fminf/fmaxf semantics (NaN-ignoring; ties return the first
//     argument, which only affects the sign of zero and never a comparison result).
//   * cosf/sinf/atanf are replaced by the deterministic float kernels rt_sincos/rt_atan01
//     below (the reference used nvcc --use_fast_math __sinf/__cosf: parity unpinned there).
//   * double sub-expressions are kept where the reference evaluates in double
//     (random.cuh:44, scene.cu:55-57, 190, 297, 357, 366, 380-381, 389-390).
//   * float->u16 in morton_code saturates (NaN/<=0 -> 0, >=65535 -> 65535), PTX cvt semantics.
#include "oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif
#ifdef ORC_FASTMATH
#include <pmmintrin.h>
#include <xmmintrin.h>
// FTZ/DAZ (nvcc -ftz=true) for the loading thread; the study renders with one thread
__attribute__((constructor)) static void orc_fastmath_ftz() {
    _MM_SET_FLUSH_ZERO_MODE(_MM_FLUSH_ZERO_ON);
    _MM_SET_DENORMALS_ZERO_MODE(_MM_DENORMALS_ZERO_ON);
}
#endif

namespace {

thread_local std::string g_err;

// ---------------------------------------------------------------- math.cuh:11-142
struct V3 { float x, y, z; };
static_assert(sizeof(V3) == 12, "Vec3 is 12 B");

inline float fmin_(float a, float b) { if (a != a) return b; if (b != b) return a; return (b < a) ? b : a; }
inline float fmax_(float a, float b) { if (a != a) return b; if (b != b) return a; return (b > a) ? b : a; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator*(float s, V3 v) { return {s * v.x, s * v.y, s * v.z}; }
inline V3 operator-(V3 v) { return {-v.x, -v.y, -v.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }           // :67
inline V3 cross(V3 a, V3 b) {                                                           // :72
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float magsq(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }                  // :82
// The fast-math study build (oracle/Makefile: build/liboracle_fastmath.so, -DORC_FASTMATH with
// -ffp-contract=fast -mfma) perturbs the restatement the way nvcc --use_fast_math (build.sh:2) moves
// the reference's GPU path away from IEEE arithmetic: FMA contraction (-fmad=true), division as a
// multiply by a float reciprocal (-prec-div=false), sqrt and 1/sqrt through a float reciprocal
// square root (-prec-sqrt=false, rsqrtf), __sinf/__cosf (argument scaled by 1/(2 pi) in float, the
// result to 2^-22 absolute: the MUFU's ~2^-21.4 error), and FTZ/DAZ.  It models the size of those
// deviations, not nvcc's exact bits (tools/fastmath_floor.py: the image error they alone cause).
// The IEEE build (liboracle.so, parity) expands every macro to the plain operation.
#ifdef ORC_FASTMATH
inline float FDIV(float a, float b) { return a * (float)(1.0 / (double)b); }
inline float FRSQRT(float x) { return (float)(1.0 / std::sqrt((double)x)); }
inline float FSQRT(float x) {
    if (!(x > 0) || std::isinf(x)) return sqrtf(x);
    return x * FRSQRT(x);
}
#else
#define FDIV(a, b) ((a) / (b))
#define FRSQRT(x) (1.0f / sqrtf(x))
#define FSQRT(x) sqrtf(x)
#endif
inline V3 normalise(V3 v) { return FRSQRT(magsq(v)) * v; }                              // :111
inline float clamp01(float x) { return fmax_(fmin_(x, 1.0f), 0.0f); }                   // :116-124
inline V3 vmin(V3 a, V3 b) { return {fmin_(a.x, b.x), fmin_(a.y, b.y), fmin_(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {fmax_(a.x, b.x), fmax_(a.y, b.y), fmax_(a.z, b.z)}; }
inline float comp(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
inline bool is_black(V3 v) { return v.x == 0 && v.y == 0 && v.z == 0; }

// Deterministic replacements for cosf/sinf (random.cuh:63-75) and atanf (scene.cu:297).
// Cody-Waite reduction by pi/2 + cephes minimax polynomials; valid for x >= 0 (the only use is
// random_radians in [0, 2*pi]).  Operation order is part of the contract with the HIP kernels.
inline void rt_sincos(float x, float *s, float *c) {
    const float fj = x * 0.636619772f;
    const int j = (int)(fj + 0.5f);
    const float jf = (float)j;
    const float r = ((x - jf * 1.5703125f) - jf * 4.837512969970703125e-4f) - jf * 7.54978995489188216e-8f;
    const float z = r * r;
    const float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    const float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
                     - 0.5f * z + 1.0f;
    switch (j & 3) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
    }
}
#ifdef ORC_FASTMATH
inline void fm_sincos(float x, float *s, float *c) {     // __sinf / __cosf (MUFU) stand-in
    const double t = (double)(x * 0.159154943f) * 6.283185307179586;
    *s = (float)(std::nearbyint(std::sin(t) * 4194304.0) / 4194304.0);
    *c = (float)(std::nearbyint(std::cos(t) * 4194304.0) / 4194304.0);
}
#endif
inline float rt_atan01(float x) {
    float y = 0.0f;
    if (x > 0.4142135623730950f) { y = 0.78539816339744830962f; x = (x - 1.0f) / (x + 1.0f); }
    const float z = x * x;
    return y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
                 - 3.33329491539e-1f) * z * x + x);
}

// ---------------------------------------------------------------- random.cuh:5-75
struct Rng { uint64_t state, inc; };
inline uint32_t xor_rand(Rng *r) {                                                     // :13-23
    const uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + (r->inc | 1);
    const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    const uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((0u - rot) & 31));
}
inline void xor_srand(Rng *r, uint32_t seed) {                                         // :25-30
    r->state = (uint64_t)seed * 6839056345687307ULL;
    r->inc = 820957824423429ULL;
    xor_rand(r);
}
inline float random01(Rng *r) { return (float)xor_rand(r) * (1.0f / 4294967296.0f); }  // :32-35
inline float random02(Rng *r) { return (float)xor_rand(r) * (2.0f / 4294967296.0f); }  // :37-40
inline float random_radians(Rng *r) {                                                  // :42-45 (double)
    return (float)((double)xor_rand(r) * (3.14159265358979323846 * 2 / 4294967295.0));
}
inline V3 random_on_sphere(Rng *r) {                                                   // :63-75
    const float r1 = random_radians(r);
    const float r2 = random02(r);
    const float x = FSQRT(r2 * (2 - r2));
    float s, c;
#ifdef ORC_FASTMATH
    fm_sincos(r1, &s, &c);
#else
    rt_sincos(r1, &s, &c);
#endif
    return {c * x, s * x, 1 - r2};
}

// ---------------------------------------------------------------- scene.cuh:9-166
struct Sphere { V3 center; float radius; };
struct Triangle { V3 p1, p2p1, p3p1, normal; };
struct Material { V3 diffuse; float metallicity; V3 specular; float roughness; V3 emitted; float ior; };
struct RayData { V3 origin, dir, transmitted, collected; };
struct Aabb {
    V3 mn{1e30f, 1e30f, 1e30f};
    V3 mx{-1e30f, -1e30f, -1e30f};
    void expand(V3 v) { mn = vmin(mn, v); mx = vmax(mx, v); }                          // scene.cu:833
    void expand(const Triangle &t) { expand(t.p1); expand(t.p2p1); expand(t.p3p1); }    // :839
    void expand(const Aabb &o) { mn = vmin(mn, o.mn); mx = vmax(mx, o.mx); }            // :846
    float half_area() const {                                                          // :852
        const V3 s = mx - mn;
        return s.x * s.y + s.x * s.z + s.y * s.z;
    }
};
struct BvhNode { Aabb aabb; int32_t child1 = 0, child2 = 0; };
static_assert(sizeof(Sphere) == 16 && sizeof(Triangle) == 48 && sizeof(Material) == 48, "layouts");
static_assert(sizeof(BvhNode) == 32 && sizeof(RayData) == 48, "layouts");
inline bool is_leaf(const BvhNode &n) { return n.child2 <= n.child1; }                 // :859

}  // namespace

struct orc_scene {
    std::vector<Sphere> spheres;
    std::vector<Triangle> triangles;
    std::vector<uint16_t> material_indices;
    std::vector<Material> materials;
    std::vector<BvhNode> bvh;
    std::vector<V3> env;
    int env_w = 0, env_h = 0;
    int width = 1920, height = 1080, ray_count = 1, bounces = 3;                        // :571-574
    float exposure = 0;
    V3 camera_position{0, 0, 0}, forward{0, 0, 0}, up{0, 0, 0};
    float vertical_fov = 0;
    V3 min_coord{0, 0, 0}, inv_dimensions{0, 0, 0};
    V3 scaled_right{0, 0, 0}, scaled_up{0, 0, 0}, near_plane_top_left{0, 0, 0};
    float inv_width = 0, inv_height = 0;
};

namespace {

// ---------------------------------------------------------------- scene.cu:62-76
void precompute_camera_data(orc_scene *s) {
    const V3 right = cross(s->up, s->forward);
    const float nph = 2.0f * std::tan(s->vertical_fov * 0.5f);
    const float npw = nph * s->width / s->height;
    s->scaled_right = npw * right;
    s->scaled_up = nph * s->up;
    s->near_plane_top_left = s->forward - 0.5f * s->scaled_right + 0.5f * s->scaled_up;
    s->inv_width = 1.0f / (s->width - 1);
    s->inv_height = 1.0f / (s->height - 1);
}

// ---------------------------------------------------------------- scene.cu:866-1000
void maybe_split(orc_scene *s, int node_index, int max_depth) {
    std::vector<BvhNode> &nodes = s->bvh;
    std::vector<Triangle> &tris = s->triangles;
    const int c2 = nodes[node_index].child2, c1 = nodes[node_index].child1;
    {
        Aabb box = nodes[node_index].aabb;
        for (int i = c2; i < c1; i++) box.expand(tris[i]);
        nodes[node_index].aabb = box;
    }
    const int our_count = c1 - c2;
    if (our_count <= 4 || max_depth == 0) return;
    const float our_cost = nodes[node_index].aabb.half_area() * our_count;
    constexpr int BINS = 8;
    int best_axis = 0;
    float best_position = 0;
    float best_cost = our_cost;
    for (int axis = 0; axis < 3; axis++) {
        float min_c = 1e30f, max_c = -1e30f;
        for (int i = c2; i < c1; i++) {
            min_c = fmin_(min_c, comp(tris[i].normal, axis));
            max_c = fmax_(max_c, comp(tris[i].normal, axis));
        }
        if (min_c == max_c) continue;
        float scale = BINS / (max_c - min_c);
        Aabb bin_box[BINS];
        int bin_count[BINS] = {0};
        for (int i = c2; i < c1; i++) {
            const int b = std::min(BINS - 1, (int)((comp(tris[i].normal, axis) - min_c) * scale));
            bin_count[b]++;
            bin_box[b].expand(tris[i]);
        }
        float left_area[BINS - 1], right_area[BINS - 1];
        int left_count[BINS - 1];
        int left_sum = 0;
        Aabb left_box, right_box;
        for (int i = 0; i + 1 < BINS; i++) {
            left_sum += bin_count[i];
            left_count[i] = left_sum;
            left_box.expand(bin_box[i]);
            left_area[i] = left_box.half_area();
            right_box.expand(bin_box[BINS - 1 - i]);
            right_area[BINS - 2 - i] = right_box.half_area();
        }
        scale = (max_c - min_c) / BINS;
        for (int i = 0; i + 1 < BINS; i++) {
            const float plane_cost = left_count[i] * left_area[i] + (our_count - left_count[i]) * right_area[i];
            if (plane_cost != 0 && plane_cost < best_cost) {
                best_axis = axis;
                best_position = min_c + scale * (i + 1);
                best_cost = plane_cost;
            }
        }
    }
    if (best_cost >= our_cost) return;
    int i = c2, j = c1 - 1;
    const int sc = (int)s->spheres.size();
    while (i <= j) {
        if (comp(tris[i].normal, best_axis) < best_position) {
            i++;
        } else {
            std::swap(tris[i], tris[j]);
            std::swap(s->material_indices[sc + i], s->material_indices[sc + j]);
            j--;
        }
    }
    if (i == c1 || i == c2) return;
    const int left = (int)nodes.size();
    nodes.emplace_back();
    const int right = (int)nodes.size();
    nodes.emplace_back();
    nodes[left].child2 = c2;
    nodes[left].child1 = i;
    nodes[right].child2 = i;
    nodes[right].child1 = c1;
    maybe_split(s, left, max_depth - 1);
    maybe_split(s, right, max_depth - 1);
    nodes[node_index].child1 = left;
    nodes[node_index].child2 = right;
}

// ---------------------------------------------------------------- scene.cu:1002-1036
void generate_bvh(orc_scene *s, int max_depth) {
    s->bvh.clear();
    s->bvh.reserve(std::max<size_t>(1, s->triangles.size() * 2));
    s->bvh.emplace_back();
    s->bvh[0].child2 = 0;
    s->bvh[0].child1 = (int)s->triangles.size();
    maybe_split(s, 0, max_depth);
    for (auto &t : s->triangles) {
        t.p2p1 = t.p2p1 - t.p1;
        t.p3p1 = t.p3p1 - t.p1;
        t.normal = normalise(cross(t.p3p1, t.p2p1));
    }
}

std::string join_root(const char *root, const std::string &p) {
    if (!root || !*root || (!p.empty() && p[0] == '/')) return p;
    std::string r(root);
    if (r.back() != '/') r += '/';
    return r + p;
}

// ---------------------------------------------------------------- scene.cu:491-546
bool load_ply(std::vector<Triangle> &out, const std::string &path) {
    std::ifstream f(path, std::ios_base::binary);
    if (!f) { g_err = "cannot open ply " + path; return false; }
    std::string line;
    std::getline(f, line); std::getline(f, line); std::getline(f, line);
    if (line.size() < 16) { g_err = "bad ply header " + path; return false; }
    const int vertex_count = std::stoi(line.substr(15));
    for (int k = 0; k < 9; k++) std::getline(f, line);
    if (line.size() < 14) { g_err = "bad ply header " + path; return false; }
    const int face_count = std::stoi(line.substr(13));
    std::getline(f, line); std::getline(f, line);
    struct Vertex { V3 position, normal; float u, v; };
    std::vector<Vertex> verts(vertex_count);
    f.read(reinterpret_cast<char *>(verts.data()), sizeof(Vertex) * verts.size());
    std::vector<int32_t> idx;
    for (int i = 0; i < face_count; i++) {
        const int n = f.get();
        if (n < 0) { g_err = "truncated ply " + path; return false; }
        idx.resize(n);
        f.read(reinterpret_cast<char *>(idx.data()), sizeof(int32_t) * n);
        for (int j = 2; j < n; j++) {
            Triangle t;
            t.p1 = verts[idx[0]].position;
            t.p2p1 = verts[idx[j - 1]].position;
            t.p3p1 = verts[idx[j]].position;
            t.normal = (1.0f / 3.0f) * (t.p1 + t.p2p1 + t.p3p1);
            out.push_back(t);
        }
    }
    return true;
}

// ---------------------------------------------------------------- scene.cu:548-567
bool load_pfm(orc_scene *s, const std::string &path) {
    std::ifstream f(path, std::ios_base::binary);
    if (!f) { g_err = "cannot open pfm " + path; return false; }
    std::string line;
    std::getline(f, line);
    std::getline(f, line);
    std::stringstream ss(line);
    ss >> s->env_w >> s->env_h;
    std::getline(f, line);
    s->env.assign((size_t)s->env_w * s->env_h, V3{0, 0, 0});
    f.read(reinterpret_cast<char *>(s->env.data()), sizeof(V3) * s->env.size());
    return true;
}

std::vector<std::string> split_ws(const std::string &s) {
    std::vector<std::string> out;
    std::istringstream is(s);
    for (std::string t; is >> t;) out.push_back(t);
    return out;
}
float num(const std::vector<std::string> &t, size_t i) { return i < t.size() ? std::strtof(t[i].c_str(), nullptr) : 0.0f; }
int inum(const std::vector<std::string> &t, size_t i) { return i < t.size() ? std::atoi(t[i].c_str()) : 0; }

// ---------------------------------------------------------------- scene.cu:569-831
orc_scene *load_scene(const char *path, int use_bvh, const char *root, const int32_t *image,
                      const float *exposure) {
    auto *s = new orc_scene();
    std::ifstream file(path);
    if (!file) { g_err = std::string("cannot open scene ") + path; delete s; return nullptr; }
    std::unordered_map<std::string, uint16_t> mat_map;
    std::vector<uint16_t> sphere_mats, tri_mats;
    bool have_env = false;
    for (std::string line; std::getline(file, line);) {
        while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
        if (line.empty()) continue;
        const size_t sp = line.find(' ');
        const std::string cmd = line.substr(0, sp);
        const std::vector<std::string> t = split_ws(line);
        auto mat_of = [&](const std::string &name, uint16_t *out) {
            auto it = mat_map.find(name);
            if (it == mat_map.end()) { g_err = "unknown material " + name; return false; }
            *out = it->second;
            return true;
        };
        if (cmd == "sky") {
            s->env.assign(1, V3{num(t, 1), num(t, 2), num(t, 3)});
            s->env_w = s->env_h = 1;
            have_env = true;
        } else if (cmd == "sky_map") {
            if (t.size() < 2 || !load_pfm(s, join_root(root, t[1]))) { delete s; return nullptr; }
            have_env = true;
            std::printf("Loaded environment map with size %d,%d\n", s->env_w, s->env_h);
        } else if (cmd == "camera") {
            s->camera_position = {num(t, 2), num(t, 3), num(t, 4)};
            s->forward = normalise(V3{num(t, 6), num(t, 7), num(t, 8)});
            s->up = normalise(V3{num(t, 10), num(t, 11), num(t, 12)});
            s->vertical_fov = (float)(num(t, 14) * (3.14159265358979323846 / 180));
        } else if (cmd == "material") {
            if (t.size() < 2) continue;
            mat_map[t[1]] = (uint16_t)s->materials.size();
            Material m;
            m.specular = {1, 1, 1};
            m.diffuse = {1, 1, 1};
            m.emitted = {0, 0, 0};
            m.metallicity = 0;
            m.roughness = 0;
            m.ior = 0;
            for (size_t k = 2; k < t.size(); k++) {
                if (t[k] == "diffuse") { m.diffuse = {num(t, k + 1), num(t, k + 2), num(t, k + 3)}; k += 3; }
                else if (t[k] == "specular") { m.specular = {num(t, k + 1), num(t, k + 2), num(t, k + 3)}; k += 3; }
                else if (t[k] == "emit") { m.emitted = {num(t, k + 1), num(t, k + 2), num(t, k + 3)}; k += 3; }
                else if (t[k] == "metallicity") { m.metallicity = num(t, ++k); }
                else if (t[k] == "roughness") { m.roughness = num(t, ++k); }
                else if (t[k] == "ior") { m.ior = num(t, ++k); }
            }
            s->materials.push_back(m);
        } else if (cmd == "sphere") {
            uint16_t m;
            if (t.size() < 2 || !mat_of(t[1], &m)) { delete s; return nullptr; }
            sphere_mats.push_back(m);
            s->spheres.push_back(Sphere{{num(t, 2), num(t, 3), num(t, 4)}, num(t, 5)});
        } else if (cmd == "triangle") {
            uint16_t m;
            if (t.size() < 2 || !mat_of(t[1], &m)) { delete s; return nullptr; }
            tri_mats.push_back(m);
            Triangle tr;
            tr.p1 = {num(t, 2), num(t, 3), num(t, 4)};
            tr.p2p1 = {num(t, 5), num(t, 6), num(t, 7)};
            tr.p3p1 = {num(t, 8), num(t, 9), num(t, 10)};
            tr.normal = (1.0f / 3.0f) * (tr.p1 + tr.p2p1 + tr.p3p1);
            s->triangles.push_back(tr);
        } else if (cmd == "quad") {
            uint16_t m;
            if (t.size() < 2 || !mat_of(t[1], &m)) { delete s; return nullptr; }
            tri_mats.push_back(m);
            tri_mats.push_back(m);
            const V3 p1{num(t, 2), num(t, 3), num(t, 4)}, p2{num(t, 5), num(t, 6), num(t, 7)};
            const V3 p3{num(t, 8), num(t, 9), num(t, 10)}, p4{num(t, 11), num(t, 12), num(t, 13)};
            Triangle a{p1, p2, p3, {0, 0, 0}};
            a.normal = (1.0f / 3.0f) * (a.p1 + a.p2p1 + a.p3p1);
            s->triangles.push_back(a);
            Triangle b{p1, p3, p4, {0, 0, 0}};
            b.normal = (1.0f / 3.0f) * (b.p1 + b.p2p1 + b.p3p1);
            s->triangles.push_back(b);
        } else if (cmd == "ply") {
            uint16_t m;
            if (t.size() < 3 || !mat_of(t[1], &m)) { delete s; return nullptr; }
            const size_t before = s->triangles.size();
            if (!load_ply(s->triangles, join_root(root, t[2]))) { delete s; return nullptr; }
            for (size_t k = before; k < s->triangles.size(); k++) tri_mats.push_back(m);
        } else if (cmd == "image") {
            s->width = inum(t, 1);
            s->height = inum(t, 2);
            s->ray_count = inum(t, 3);
            s->bounces = inum(t, 4);
            s->exposure = num(t, 5);
        }
    }
    if (image) { s->width = image[0]; s->height = image[1]; s->ray_count = image[2]; s->bounces = image[3]; }
    if (exposure) s->exposure = *exposure;
    if (!have_env) { s->env.assign(1, V3{0, 0, 0}); s->env_w = s->env_h = 1; }  // reference: UB
    s->material_indices = sphere_mats;
    s->material_indices.insert(s->material_indices.end(), tri_mats.begin(), tri_mats.end());
    precompute_camera_data(s);
    generate_bvh(s, use_bvh ? 30 : 0);
    s->min_coord = s->bvh[0].aabb.mn;
    V3 mx = s->bvh[0].aabb.mx;
    for (const auto &sp : s->spheres) {
        const V3 r{sp.radius, sp.radius, sp.radius};
        mx = vmax(mx, sp.center + r);
        s->min_coord = vmin(s->min_coord, sp.center - r);
    }
    s->inv_dimensions = {1 / mx.x, 1 / mx.y, 1 / mx.z};
    return s;
}

// ---------------------------------------------------------------- scene.cu:44-60 (key)
uint16_t sat_u16(double v) {
    if (!(v > 0.0)) return 0;           // NaN, <= 0
    if (v >= 65535.0) return 65535;
    return (uint16_t)v;
}
uint16_t interleave_5(uint16_t x) {     // scene.cu:44-51, including the 0x1000010100011 literal
    x = (uint16_t)((x | (x << 8)) & 0b1000000001111);
    x = (uint16_t)((x | (x << 4)) & 0x1000010100011LL);
    x = (uint16_t)((x | (x << 2)) & 0b1001001001001);
    return x;
}
uint16_t morton_code(V3 v) {            // scene.cu:53-60
    const uint16_t x = sat_u16((double)v.x * 31.99);
    const uint16_t y = sat_u16((double)v.y * 31.99);
    const uint16_t z = sat_u16((double)v.z * 31.99);
    return (uint16_t)(interleave_5(x) | (interleave_5(y) << 1) | (interleave_5(z) << 2));
}

// float(t) < 0.005 as double  <=>  t < 0x1.47ae16p-8f (smallest float whose double >= 0.005).
inline bool below_eps(float t) { return (double)t < 0.005; }

// ---------------------------------------------------------------- scene.cu:109-132
inline bool ray_aabb(const Aabb &b, V3 o, V3 n_inv, float &tmin, float tmax) {
    tmin = 0.0f;
    float t1 = (b.mn.x - o.x) * n_inv.x, t2 = (b.mx.x - o.x) * n_inv.x;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    t1 = (b.mn.y - o.y) * n_inv.y; t2 = (b.mx.y - o.y) * n_inv.y;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    t1 = (b.mn.z - o.z) * n_inv.z; t2 = (b.mx.z - o.z) * n_inv.z;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    return tmin <= tmax;
}

// Möller–Trumbore body, scene.cu:162-195. Returns true and t when accepted against `closest`.
inline bool ray_tri(const Triangle &tr, V3 o, V3 d, float closest, float *t_out) {
    const V3 h = cross(d, tr.p3p1);
    const float a = dot(h, tr.p2p1);
    if (a == 0) return false;
    const float f = FDIV(1.0f, a);
    const V3 s = o - tr.p1;
    const float u = dot(s, h) * f;
    if (u < 0 || u > 1) return false;
    const V3 q = cross(s, tr.p2p1);
    const float v = dot(d, q) * f;
    if (v < 0 || u + v > 1) return false;
    const float t = dot(tr.p3p1, q) * f;
    if (below_eps(t) || t >= closest) return false;
    *t_out = t;
    return true;
}

// Sphere body, scene.cu:340-371. Returns 1 if accepted (t_out set).
inline bool ray_sphere(const Sphere &sp, V3 o, V3 d, float closest, float *t_out) {
    const V3 off = sp.center - o;
    const float mhb = dot(off, d);
    const float qc = magsq(off) - sp.radius * sp.radius;
    const float qd = mhb * mhb - qc;
    if (qd < 0) return false;
    const float hs = FSQRT(qd);
    float t = mhb - hs;
    if (t < closest && !below_eps(t)) { *t_out = t; return true; }
    t = mhb + hs;
    if (t < closest && !below_eps(t)) { *t_out = t; return true; }
    return false;
}

struct Counters {
    uint64_t pn = 0, iv = 0, tt = 0, st = 0, ht = 0, hs = 0, miss = 0, live = 0, dead = 0;
    uint32_t max_stack = 0, max_ray_pn = 0;
    uint32_t max_ray_steps = 0;   // internal visits + triangle tests of one ray (the HIP trace's steps)
    // analysis only (tools/chain_models.py): the longest ray's dependent record fetches under trace-kernel
    // models -- [0] one fetch per internal step (root free) and per triangle (the round-5 kernel); [1] two-level
    // records (a descent fetches its node's record and its children's pair together, so a fetch serves two
    // levels; a stack pop fetches one level) with two triangles per fetch; [2] the same with the children's pair
    // index kept on the stack (pops fetch two levels too); [3] as [1] with one triangle per fetch
    uint32_t max_chain[4] = {0, 0, 0, 0};
    uint64_t sum_chain[4] = {0, 0, 0, 0};
    // analysis only: pushes the HIP trace kernel makes below its 8 LDS entries (global overflow stack)
    uint64_t ovf = 0;
    void add(const Counters &o) {
        ovf += o.ovf;
        for (int k = 0; k < 4; k++) {
            max_chain[k] = std::max(max_chain[k], o.max_chain[k]);
            sum_chain[k] += o.sum_chain[k];
        }
        pn += o.pn; iv += o.iv; tt += o.tt; st += o.st; ht += o.ht; hs += o.hs; miss += o.miss;
        live += o.live; dead += o.dead; max_stack = std::max(max_stack, o.max_stack);
        max_ray_pn = std::max(max_ray_pn, o.max_ray_pn);
        max_ray_steps = std::max(max_ray_steps, o.max_ray_steps);
    }
};

// Analysis instrumentation of the traversal (chain models, fetch records, overflow pushes): compiled into the
// strict liboracle.so only (-DORC_ANALYSIS), never into the timed cpu_baseline or the fast-math studies.
#ifdef ORC_ANALYSIS
#define ORC_A(...) __VA_ARGS__
#else
#define ORC_A(...)
#endif
// analysis only (orc_bounce_working_set): the records one traversal fetches, in order -- an internal node's id
// (its child-pair record), or kRecTri | triangle index; the root's record is free (scalar registers)
constexpr uint32_t kRecTri = 0x80000000u;
thread_local std::vector<uint32_t> *g_rec = nullptr;

// ---------------------------------------------------------------- scene.cu:134-241
void bvh_closest_hit(const orc_scene *s, V3 o, V3 d, float &closest, int &index, Counters &c) {
    const V3 n_inv{FDIV(1.0f, d.x), FDIV(1.0f, d.y), FDIV(1.0f, d.z)};
    uint32_t idx_stack[31];
    float dist_stack[31];
    int sc = 1;
    idx_stack[0] = 0;
    dist_stack[0] = 0;
    const int sphere_count = (int)s->spheres.size();
    ORC_A(uint32_t ch[4] = {0, 0, 0, 0};   // chain models (Counters::max_chain), analysis only
          bool desc = false, cover1 = false, cover2 = false, root = true;)
    while (sc) {
        sc--;
        const float dist = dist_stack[sc];
        ORC_A(const bool desc_now = desc; desc = false;)
        if (dist >= closest) continue;
        const BvhNode &node = s->bvh[idx_stack[sc]];
        c.pn++;
#ifdef ORC_ANALYSIS
        if (is_leaf(node)) {
            const uint32_t nt = (uint32_t)std::max(0, node.child1 - node.child2);
            ch[0] += nt; ch[1] += (nt + 1) / 2; ch[2] += (nt + 1) / 2; ch[3] += nt;
            cover1 = cover2 = false;
        } else if (root) {
            cover1 = cover2 = false;       // the root's record is in scalar registers: no fetch
        } else {
            if (g_rec) g_rec->push_back(idx_stack[sc]);
            ch[0]++;
            // [1]/[3]: covered when this is the descent of a node whose fetch brought its children's pair
            const bool c1 = desc_now && cover1;
            if (!c1) { ch[1]++; ch[3]++; }
            cover1 = !c1 && desc_now;      // a descent's fetch (mode B) brings the pair; a pop's does not
            const bool c2 = desc_now && cover2;
            if (!c2) ch[2]++;
            cover2 = !c2;                  // [2]: every fetch brings the pair
        }
        root = false;
#endif
        if (is_leaf(node)) {
            for (int i = node.child2; i < node.child1; i++) {
                c.tt++;
                ORC_A(if (g_rec) g_rec->push_back(kRecTri | (uint32_t)i);)
                float t;
                if (ray_tri(s->triangles[i], o, d, closest, &t)) {
                    closest = t;
                    index = sphere_count + i;
                }
            }
        } else {
            c.iv++;
            float d1, d2;
            const bool h1 = ray_aabb(s->bvh[node.child1].aabb, o, n_inv, d1, closest);
            const bool h2 = ray_aabb(s->bvh[node.child2].aabb, o, n_inv, d2, closest);
            if (h1 && h2) {
                ORC_A(if (sc >= 8) c.ovf++;)   // the kernel pushes one child here, at entry sc
                if (d1 < d2) {
                    idx_stack[sc] = node.child1; dist_stack[sc] = d1; sc++;
                    idx_stack[sc] = node.child2; dist_stack[sc] = d2; sc++;
                } else {
                    idx_stack[sc] = node.child2; dist_stack[sc] = d2; sc++;
                    idx_stack[sc] = node.child1; dist_stack[sc] = d1; sc++;
                }
            } else if (h1) {
                idx_stack[sc] = node.child1; dist_stack[sc] = d1; sc++;
            } else if (h2) {
                idx_stack[sc] = node.child2; dist_stack[sc] = d2; sc++;
            }
            ORC_A(desc = h1 || h2;)
            if ((uint32_t)sc > c.max_stack) c.max_stack = (uint32_t)sc;
        }
    }
#ifdef ORC_ANALYSIS
    for (int k = 0; k < 4; k++) {
        c.max_chain[k] = std::max(c.max_chain[k], ch[k]);
        c.sum_chain[k] += ch[k];
    }
#endif
}

// ---------------------------------------------------------------- scene.cu:284-318
V3 equal_area_project(V3 dir) {
    const float x = std::fabs(dir.x), y = std::fabs(dir.y), z = std::fabs(dir.z);
    const float r = FSQRT(1 - fmin_(z, 1.0f));
    const float a = fmax_(x, y);
    float b = fmin_(x, y);
    b = a == 0 ? 0 : FDIV(b, a);
    float phi = (float)((2 / 3.14159265358979323846) * (double)rt_atan01(b));
    if (x < y) phi = 1 - phi;
    float v = phi * r;
    float u = r - v;
    if (dir.z < 0) {
        const float old_v = v;
        v = 1 - u;
        u = 1 - old_v;
    }
    u = std::copysign(u, dir.x);
    v = std::copysign(v, dir.y);
    return {(u + 1) * 0.5f, (v + 1) * 0.5f, 0};
}

int env_texel(const orc_scene *s, V3 d) {                  // scene.cu:380-391
    const float dx = (float)((double)d.x * -0.386527 + (double)d.z * 0.922278);
    const float dy = (float)((double)d.x * -0.922278 + (double)d.z * -0.386527);
    const float dz = d.y;
    const V3 uv = equal_area_project({dx, dy, dz});
    const int tx = (int)((double)(clamp01(uv.x) * (s->env_w - 1)) + 0.5);
    const int ty = (int)((double)(clamp01(uv.y) * (s->env_h - 1)) + 0.5);
    return ty * s->env_h + tx;
}

// ---------------------------------------------------------------- scene.cu:320-487
// gpu: key-based early-out and key write (the __CUDA_ARCH__ branches); else CPU branches.
void process_ray(const orc_scene *s, RayData *rp, uint32_t *key, Rng rng, bool gpu, Counters &c) {
    if (gpu) {
        if (*key == 0xFFFFFFFFu) { c.dead++; return; }
    } else if (is_black(rp->transmitted)) {
        c.dead++;
        return;
    }
    c.live++;
    RayData rd = *rp;
    float closest = 1e30f;
    int index = -1;
    const V3 o = rd.origin, d = rd.dir;
    const int sphere_count = (int)s->spheres.size();
    for (int i = 0; i < sphere_count; i++) {
        c.st++;
        float t;
        if (ray_sphere(s->spheres[i], o, d, closest, &t)) { closest = t; index = i; }
    }
    const uint64_t pn0 = c.pn, steps0 = c.iv + c.tt;
    bvh_closest_hit(s, o, d, closest, index, c);
    c.max_ray_pn = std::max(c.max_ray_pn, (uint32_t)(c.pn - pn0));
    c.max_ray_steps = std::max(c.max_ray_steps, (uint32_t)(c.iv + c.tt - steps0));
    if (index == -1) {
        c.miss++;
        const V3 sky = s->env[env_texel(s, d)];
        rd.collected = rd.collected + sky * rd.transmitted;
        rd.transmitted = {0, 0, 0};
    } else {
        const V3 hit = o + closest * d;
        rd.origin = hit;
        V3 normal;
        if (index < sphere_count) {
            c.hs++;
            const Sphere &sp = s->spheres[index];
            normal = FDIV(1.0f, sp.radius) * (hit - sp.center);
        } else {
            c.ht++;
            normal = s->triangles[index - sphere_count].normal;
        }
        const Material &m = s->materials[s->material_indices[index]];
        rd.collected = rd.collected + m.emitted * rd.transmitted;
        const bool front = dot(normal, d) < 0;
        if (!front) normal = -normal;
        const V3 rough = normalise(normal + m.roughness * random_on_sphere(&rng));
        const float cos_theta = dot(rough, d);
        if (m.ior == 0) {
            if (random01(&rng) <= m.metallicity) {
                rd.transmitted = rd.transmitted * m.specular;
                rd.dir = d - (2 * cos_theta) * rough;
            } else {
                rd.transmitted = rd.transmitted * m.diffuse;
                rd.dir = normalise(normal + random_on_sphere(&rng));
            }
        } else {
            float ior = m.ior;
            float inv_ior = FDIV(1.0f, ior);
            if (front) std::swap(ior, inv_ior);
            const float sin2 = 1 - cos_theta * cos_theta;
            float r0 = FDIV(1 - ior, 1 + ior);
            r0 *= r0;
            const float cs = 1 + cos_theta;
            const float refl = r0 + (1 - r0) * cs * cs * cs * cs * cs;
            if (sin2 > inv_ior * inv_ior || random01(&rng) < refl) {
                rd.transmitted = rd.transmitted * m.specular;
                rd.dir = d - (2 * cos_theta) * rough;
            } else {
                rd.transmitted = rd.transmitted * m.diffuse;
                const V3 perp = ior * (d - cos_theta * rough);
                const V3 par = (-FSQRT(1 - magsq(perp))) * rough;
                rd.dir = normalise(par + perp);
            }
        }
    }
    if (gpu) {
        if (is_black(rd.transmitted)) {
            *key = 0xFFFFFFFFu;
        } else {
            *key = ((uint32_t)morton_code((rd.origin - s->min_coord) * s->inv_dimensions) << 16) |
                   (uint32_t)morton_code(0.5f * (rd.dir + V3{1, 1, 1}));
        }
    }
    *rp = rd;
}

// ---------------------------------------------------------------- scene.cu:78-105
RayData make_ray(const orc_scene *s, int rtc, int i, int seed) {
    Rng rng;
    xor_srand(&rng, (uint32_t)i * 0x85810BEAu + 709579u * (uint32_t)seed);
    const int fb = i / rtc;
    const int x = fb % s->width, y = fb / s->width;
    const float xc = (x + random01(&rng)) * s->inv_width;
    const float yc = (y + random01(&rng)) * s->inv_height;
    RayData r;
    r.origin = s->camera_position;
    r.dir = normalise(s->near_plane_top_left + xc * s->scaled_right - yc * s->scaled_up);
    r.transmitted = {1, 1, 1};
    r.collected = {0, 0, 0};
    return r;
}

void generate_ray(const orc_scene *s, RayData *rays, uint32_t *idx, uint32_t *keys, int rtc, int i, int seed) {
    if ((i / rtc) / s->width < s->height) {
        if (idx) { idx[i] = (uint32_t)i; keys[i] = 0; }
        rays[i] = make_ray(s, rtc, i, seed);
    }
}

int nthreads(int t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

// Pass p of the reference's `while (remaining_rays)` loop (raytracing.cu:222-227).
void pass_params(const orc_scene *s, int p, int *rtc, int *remaining_after) {
    const int before = s->ray_count - 20 * p;
    *rtc = std::min(before, 20);
    *remaining_after = before - *rtc;
}
int pass_total(const orc_scene *s) { return (s->ray_count + 19) / 20; }

// One GPU-semantics pass: generate, bounces (process + stable sort), per-pixel ordered sum.
// analysis only: called before bounce b with the pass's rays, slot -> ray and slot keys; true stops the pass
std::function<bool(int, const std::vector<RayData> &, const std::vector<uint32_t> &, const std::vector<uint32_t> &)>
    g_bounce_hook;

void gpu_pass(const orc_scene *s, int p, bool sort, float *pass_sum, Counters &total, uint64_t *hist,
              uint64_t *sorted, int threads, uint32_t *bounce_max_steps = nullptr, uint64_t *bounce_live = nullptr,
              uint64_t *bounce_chains = nullptr) {
    int rtc, rem;
    pass_params(s, p, &rtc, &rem);
    const int64_t n = (int64_t)rtc * s->width * s->height;
    std::vector<RayData> rays(n);
    std::vector<uint32_t> idx(n), keys(n), idx2, keys2;
    const int nt = nthreads(threads);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int64_t i = 0; i < n; i++) generate_ray(s, rays.data(), idx.data(), keys.data(), rtc, (int)i, rem);
    for (int b = 0; b < s->bounces; b++) {
        if (g_bounce_hook && g_bounce_hook(b, rays, idx, keys)) return;
        const uint32_t seed = (uint32_t)(rem * 20 + b);
        std::vector<Counters> per(nt);
#pragma omp parallel num_threads(nt)
        {
#ifdef _OPENMP
            Counters &c = per[omp_get_thread_num()];
#else
            Counters &c = per[0];
#endif
#pragma omp for schedule(dynamic, 4096)
            for (int64_t slot = 0; slot < n; slot++) {   // raytracing.cu:83-94
                Rng rng;
                xor_srand(&rng, (uint32_t)slot * 4137874753u + 279220567u * seed);
                process_ray(s, &rays[idx[slot]], &keys[slot], rng, true, c);
            }
        }
        {
            Counters bc;
            for (auto &c : per) bc.add(c);
            if (bounce_max_steps) bounce_max_steps[b] = bc.max_ray_steps;
            if (bounce_live) bounce_live[b] = bc.live;
            if (bounce_chains)
                for (int k = 0; k < 4; k++) {
                    bounce_chains[(size_t)b * 8 + k] = bc.max_chain[k];
                    bounce_chains[(size_t)b * 8 + 4 + k] = bc.sum_chain[k];
                }
        }
        for (auto &c : per) total.add(c);
        if (hist) {
            uint64_t *h = hist + (size_t)b * 65;
            for (int64_t k = 0; k < n; k++) h[orc_key_bucket(keys[k])]++;
        }
        if (sort && b + 1 != s->bounces) {              // raytracing.cu:238-247: stable sort pairs
            // cub::DeviceRadixSort::SortPairs is an LSD radix sort of the 32-bit keys: four stable 8-bit
            // counting passes (a pass whose digit is the same for every key moves nothing and is skipped)
            idx2.resize(n);
            keys2.resize(n);
            for (int shift = 0; shift < 32; shift += 8) {
                int64_t cnt[257] = {0};
                for (int64_t k = 0; k < n; k++) cnt[((keys[k] >> shift) & 0xFF) + 1]++;
                bool one = false;
                for (int d = 0; d < 256; d++) one = one || cnt[d + 1] == n;
                if (one) continue;
                for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
                for (int64_t k = 0; k < n; k++) {
                    const int64_t to = cnt[(keys[k] >> shift) & 0xFF]++;
                    keys2[to] = keys[k];
                    idx2[to] = idx[k];
                }
                idx.swap(idx2);
                keys.swap(keys2);
            }
            *sorted += (uint64_t)n;
        }
    }
    const int64_t pixels = (int64_t)s->width * s->height;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int64_t px = 0; px < pixels; px++) {
        V3 sum{0, 0, 0};
        for (int k = 0; k < rtc; k++) sum = sum + rays[px * rtc + k].collected;
        pass_sum[px * 3 + 0] = sum.x;
        pass_sum[px * 3 + 1] = sum.y;
        pass_sum[px * 3 + 2] = sum.z;
    }
    total.live += 0;
    (void)n;
}

// Pixel-tile sharding with the reorder on ("sort on" row) -- the distributed form of
// gpu_pass that the HIP renderer's tiled sort-on mode implements.  Owner `ti` of `tc` renders only
// the rays of its row stripes (stripes of `tr` rows dealt round-robin), each with its global ray
// index i = pixel * rtc + s (so generate seeds are the 1-GPU ones, scene.cu:78-105).  The process
// seed follows the ray's GLOBAL slot (raytracing.cu:89), which after a sort depends on every
// owner's keys (raytracing.cu:238-247).  Live rays always occupy global slots [0, Lg), so after
// each bounce but the last every owner writes bucket + 1 at the global slot of each of its rays
// into a zeroed byte array of length Lg, `exchange` sums the arrays over the owners (an
// all-reduce), and every owner ranks its rays exactly as the stable 65-bucket sort of all keys
// would: new slot = rays in smaller buckets + rays of the same bucket at smaller global slots.
// Nothing but those bytes crosses owners; rays never migrate.  With sort off the slot is the ray
// index and no exchange happens.  pass_sum: this owner's pixels only (the rest untouched).
void tile_pass(const orc_scene *s, int p, bool sort, int tc, int ti, int tr, orc_exchange_fn exchange, void *user,
               float *pass_sum, Counters &total, int threads) {
    int rtc, rem;
    pass_params(s, p, &rtc, &rem);
    const int W = s->width, H = s->height;
    std::vector<int64_t> pix;                          // own pixels, ascending (rows of own stripes)
    for (int k = ti; (int64_t)k * tr < H; k += tc)
        for (int y = k * tr; y < std::min(H, (k + 1) * tr); y++)
            for (int x = 0; x < W; x++) pix.push_back((int64_t)y * W + x);
    const int64_t m = (int64_t)pix.size() * rtc;
    std::vector<RayData> rays(m);
    std::vector<uint32_t> keys(m, 0), gslot(m), next(m);
    const int nt = nthreads(threads);
    for (int64_t j = 0; j < m; j++) {
        const int64_t gid = pix[j / rtc] * rtc + j % rtc;
        gslot[j] = (uint32_t)gid;                      // bounce 0: slot = ray index
        rays[j] = make_ray(s, rtc, (int)gid, rem);
    }
    std::vector<int64_t> live(m);                      // own live rays in global-slot order
    for (int64_t j = 0; j < m; j++) live[j] = j;
    int64_t Lg = (int64_t)rtc * W * H;                 // global live count: every generated ray
    for (int b = 0; b < s->bounces; b++) {
        const uint32_t seed = (uint32_t)(rem * 20 + b);
        std::vector<Counters> per(nt);
#pragma omp parallel num_threads(nt)
        {
#ifdef _OPENMP
            Counters &c = per[omp_get_thread_num()];
#else
            Counters &c = per[0];
#endif
#pragma omp for schedule(dynamic, 4096)
            for (int64_t q = 0; q < (int64_t)live.size(); q++) {
                const int64_t j = live[q];
                Rng rng;
                xor_srand(&rng, gslot[j] * 4137874753u + 279220567u * seed);   // raytracing.cu:89
                process_ray(s, &rays[j], &keys[j], rng, true, c);
            }
        }
        for (auto &c : per) total.add(c);
        if (b + 1 == s->bounces) break;
        if (!sort) {                                   // slot = ray index for the whole pass
            std::vector<int64_t> keep;
            for (int64_t j : live) if (keys[j] != 0xFFFFFFFFu) keep.push_back(j);
            live.swap(keep);
            continue;
        }
        std::vector<uint8_t> g((size_t)Lg, 0);
        for (int64_t j : live) g[gslot[j]] = (uint8_t)(orc_key_bucket(keys[j]) + 1);
        if (Lg > 0 && exchange(user, g.data(), Lg) != 0) throw std::runtime_error("tile exchange failed");
        uint64_t cnt[65] = {0};
        for (int64_t k = 0; k < Lg; k++) {
            if (g[k] < 1 || g[k] > 65) throw std::runtime_error("tile exchange: a slot has no owner");
            cnt[g[k] - 1]++;
        }
        uint64_t base[65], acc = 0;
        for (int k = 0; k < 65; k++) { base[k] = acc; acc += cnt[k]; }
        uint64_t seen[65] = {0};
        size_t q = 0;                                  // own live rays are in ascending global slot
        std::vector<int64_t> keep;
        for (int64_t k = 0; k < Lg; k++) {
            const int bk = g[k] - 1;
            if (q < live.size() && (int64_t)gslot[live[q]] == k) {
                const int64_t j = live[q++];
                if (bk != 64) { next[j] = (uint32_t)(base[bk] + seen[bk]); keep.push_back(j); }
            }
            seen[bk]++;
        }
        std::stable_sort(keep.begin(), keep.end(), [&](int64_t a, int64_t c) { return next[a] < next[c]; });
        for (int64_t j : keep) gslot[j] = next[j];
        live.swap(keep);
        Lg -= (int64_t)cnt[64];
    }
    for (size_t qp = 0; qp < pix.size(); qp++) {
        V3 sum{0, 0, 0};
        for (int k = 0; k < rtc; k++) sum = sum + rays[(int64_t)qp * rtc + k].collected;
        pass_sum[pix[qp] * 3 + 0] = sum.x;
        pass_sum[pix[qp] * 3 + 1] = sum.y;
        pass_sum[pix[qp] * 3 + 2] = sum.z;
    }
}

}  // namespace

// ==================================================================== C API
extern "C" {

const char *orc_last_error(void) { return g_err.c_str(); }

orc_scene *orc_load_scene(const char *path, int use_bvh, const char *asset_root, const int32_t *image,
                          const float *exposure) {
    try {
        return load_scene(path, use_bvh, asset_root, image, exposure);
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

void orc_free_scene(orc_scene *s) { delete s; }

void orc_get_info(const orc_scene *s, orc_info *o) {
    o->width = s->width; o->height = s->height; o->ray_count = s->ray_count; o->bounces = s->bounces;
    o->exposure = s->exposure;
    o->sphere_count = (int32_t)s->spheres.size();
    o->triangle_count = (int32_t)s->triangles.size();
    o->material_count = (int32_t)s->materials.size();
    o->bvh_node_count = (int32_t)s->bvh.size();
    o->env_width = s->env_w; o->env_height = s->env_h;
}

int orc_camera_floats(void) { return 29; }

void orc_get_arrays(const orc_scene *s, void *spheres, void *triangles, uint16_t *mi, void *materials,
                    void *bvh, float *env, float *cam) {
    if (spheres && !s->spheres.empty()) std::memcpy(spheres, s->spheres.data(), s->spheres.size() * 16);
    if (triangles && !s->triangles.empty()) std::memcpy(triangles, s->triangles.data(), s->triangles.size() * 48);
    if (mi && !s->material_indices.empty()) std::memcpy(mi, s->material_indices.data(), s->material_indices.size() * 2);
    if (materials && !s->materials.empty()) std::memcpy(materials, s->materials.data(), s->materials.size() * 48);
    if (bvh) std::memcpy(bvh, s->bvh.data(), s->bvh.size() * 32);
    if (env) std::memcpy(env, s->env.data(), s->env.size() * 12);
    if (cam) {
        const V3 v[] = {s->camera_position, s->forward, s->up};
        int k = 0;
        for (const V3 &x : v) { cam[k++] = x.x; cam[k++] = x.y; cam[k++] = x.z; }
        cam[k++] = s->vertical_fov;
        const V3 w[] = {s->min_coord, s->inv_dimensions, s->scaled_right, s->scaled_up, s->near_plane_top_left};
        for (const V3 &x : w) { cam[k++] = x.x; cam[k++] = x.y; cam[k++] = x.z; }
        cam[k++] = s->inv_width;
        cam[k++] = s->inv_height;
        cam[k++] = s->exposure;
    }
}

int orc_render_gpu_semantics(const orc_scene *s, int sort, int pass_begin, int pass_count, float *fb,
                             orc_stats *stats, uint64_t *bucket_hist, int threads) {
    const int P = pass_total(s);
    if (pass_count < 0) pass_count = P - pass_begin;
    if (pass_begin < 0 || pass_begin + pass_count > P) { g_err = "pass range"; return -1; }
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3);
    Counters total;
    uint64_t sorted = 0, generated = 0;
    for (int p = pass_begin; p < pass_begin + pass_count; p++) {
        uint64_t *h = bucket_hist ? bucket_hist + (size_t)(p - pass_begin) * s->bounces * 65 : nullptr;
        gpu_pass(s, p, sort != 0, sum.data(), total, h, &sorted, threads);
        int rtc, rem;
        pass_params(s, p, &rtc, &rem);
        generated += (uint64_t)rtc * pixels;
        for (int64_t k = 0; k < pixels * 3; k++) fb[k] = fb[k] + sum[k];
    }
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->generated_rays = generated;
        stats->live_segments = total.live;
        stats->dead_slots = total.dead;
        stats->nodes_popped = total.pn;
        stats->internal_visits = total.iv;
        stats->triangle_tests = total.tt;
        stats->sphere_tests = total.st;
        stats->hits_triangle = total.ht;
        stats->hits_sphere = total.hs;
        stats->misses = total.miss;
        stats->sorted_items = sorted;
        stats->max_stack = total.max_stack;
        stats->max_ray_nodes = total.max_ray_pn;
        stats->passes = (uint32_t)pass_count;
    }
    return 0;
}

int orc_render_tiled(const orc_scene *s, int sort, int tile_count, int tile_index, int tile_rows, int pass_begin,
                     int pass_count, orc_exchange_fn exchange, void *user, float *fb, orc_stats *stats, int threads) {
    const int P = pass_total(s);
    if (pass_count < 0) pass_count = P - pass_begin;
    if (pass_begin < 0 || pass_begin + pass_count > P) { g_err = "pass range"; return -1; }
    if (tile_count < 1 || tile_index < 0 || tile_index >= tile_count || tile_rows < 1 || (sort && !exchange)) {
        g_err = "bad tile arguments";
        return -1;
    }
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3, 0.0f);
    Counters total;
    uint64_t generated = 0;
    try {
        for (int p = pass_begin; p < pass_begin + pass_count; p++) {
            tile_pass(s, p, sort != 0, tile_count, tile_index, tile_rows, exchange, user, sum.data(), total, threads);
            for (int64_t k = 0; k < pixels * 3; k++) fb[k] = fb[k] + sum[k];   // other owners' pixels: + 0
        }
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->live_segments = total.live;
        stats->nodes_popped = total.pn;
        stats->internal_visits = total.iv;
        stats->triangle_tests = total.tt;
        stats->hits_triangle = total.ht;
        stats->hits_sphere = total.hs;
        stats->misses = total.miss;
        stats->passes = (uint32_t)pass_count;
        (void)generated;
    }
    return 0;
}

// Per bounce of pass p (GPU semantics): the longest ray's trace steps (internal visits + triangle
// tests, one HIP trace step each) and the live rays -- what bounds a tail bounce's latency.
int orc_pass_bounce_profile(const orc_scene *s, int sort, int pass, uint32_t *max_steps, uint64_t *live, int threads) {
    if (pass < 0 || pass >= pass_total(s)) { g_err = "pass range"; return -1; }
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3);
    Counters total;
    uint64_t sorted = 0;
    gpu_pass(s, pass, sort != 0, sum.data(), total, nullptr, &sorted, threads, max_steps, live);
    return 0;
}

// Analysis only (tools/chain_models.py): per bounce of pass p, the longest ray's dependent record fetches and
// their sum over the live rays under the trace-kernel models of Counters::max_chain: out[b*8 + k] = max,
// out[b*8 + 4 + k] = sum, k < 4.
int orc_pass_chain_profile(const orc_scene *s, int sort, int pass, uint64_t *out, int threads) {
#ifndef ORC_ANALYSIS
    g_err = "analysis build only (liboracle.so)";
    return -1;
#endif
    if (pass < 0 || pass >= pass_total(s)) { g_err = "pass range"; return -1; }
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3);
    Counters total;
    uint64_t sorted = 0;
    gpu_pass(s, pass, sort != 0, sum.data(), total, nullptr, &sorted, threads, nullptr, nullptr, out);
    return 0;
}

// Analysis only (tools/route_model.py, verdict r05 item 6): which scene bytes the trace kernel's rays in flight on
// one XCD touch at bounce `bounce` of pass p, under three ways of dealing the live slots to the 8 XCDs:
//   policy 0  contiguous eighths of the slots (the product: queue shard = blockIdx % 8, blocks dealt round-robin
//             over the XCDs, so an XCD's waves take the shard's slot range; after the reorder that range is a run of
//             buckets, i.e. of origin octants of the scene box)
//   policy 1  the x-th eighth of every bucket (round 5's XCD-affine order: a band of image rows)
//   policy 2  by the first depth-`depth` subtree the ray's traversal enters (the top-level treelet), 2^depth
//             treelets dealt to 8 XCDs round-robin
// For each XCD, its rays are taken in slot order in windows of `window` rays (the lanes one XCD holds resident);
// out (per policy, 6 doubles): mean and max over the sampled windows of the distinct bytes touched (64-B node
// records + 48-B triangles), the mean fetched bytes per window, the largest XCD's share of the rays, and, over
// the whole bounce, the scene bytes the 8 L2s miss (each 4 MB, 16-way LRU, 128-B lines, node records at 64 B
// per node id and then the triangles at 48 B; every XCD's rays in slot order, one after another) and the
// fetched bytes; then out[18..20] = the kernel's overflow-stack pushes over the bounce, the live rays, and the rays
// with at least one.
int orc_bounce_working_set(const orc_scene *s, int sort, int pass, int bounce, int window, int depth,
                           int windows_per_xcd, double *out, int threads) {
#ifndef ORC_ANALYSIS
    g_err = "analysis build only (liboracle.so)";
    return -1;
#endif
    if (pass < 0 || pass >= pass_total(s)) { g_err = "pass range"; return -1; }
    if (bounce < 0 || bounce >= s->bounces || window < 1 || depth < 1 || depth > 12 || windows_per_xcd < 1) {
        g_err = "bad arguments"; return -1;
    }
    const int nn = (int)s->bvh.size();
    std::vector<int> dep(nn, 0), par(nn, -1);           // node depths and parents (children follow their parent)
    for (int i = 0; i < nn; i++)
        if (!is_leaf(s->bvh[i])) {
            dep[s->bvh[i].child1] = dep[i] + 1;
            dep[s->bvh[i].child2] = dep[i] + 1;
            par[s->bvh[i].child1] = par[s->bvh[i].child2] = i;
        }
    const int nt = nthreads(threads);
    bool done = false;
    g_bounce_hook = [&](int b, const std::vector<RayData> &rays, const std::vector<uint32_t> &idx,
                        const std::vector<uint32_t> &keys) {
        if (b != bounce) return false;
        done = true;
        int64_t L = 0;                                  // live slots are a prefix after the reorder
        while (L < (int64_t)keys.size() && keys[L] != 0xFFFFFFFFu) L++;
        // per live slot: the records its traversal fetches (kept only for the slots a sampled window holds)
        std::vector<int> xcd[3];
        for (auto &v : xcd) v.assign(L, 0);
        std::vector<int64_t> bstart(66, L);             // bucket ranges (policy 1)
        for (int64_t k = L - 1; k >= 0; k--) bstart[orc_key_bucket(keys[k])] = k;
        for (int bk = 64; bk >= 0; bk--) bstart[bk] = std::min(bstart[bk], bstart[bk + 1]);
        std::vector<std::vector<uint32_t>> rec(L);
        std::vector<int> first_sub(L, 0);
        std::vector<uint64_t> ovf(L, 0);
#pragma omp parallel for schedule(dynamic, 1024) num_threads(nt)
        for (int64_t k = 0; k < L; k++) {
            std::vector<uint32_t> r;
            g_rec = &r;
            float closest = 1e30f;
            int index = -1;
            Counters c;
            const RayData &rd = rays[idx[k]];
            bvh_closest_hit(s, rd.origin, rd.dir, closest, index, c);
            g_rec = nullptr;
            ovf[k] = c.ovf;
            int sub = 0;
            for (uint32_t x : r)
                if (!(x & kRecTri) && dep[x] >= depth) {   // the first fetched node at the treelet depth or below
                    int a = (int)x;
                    while (dep[a] > depth) a = par[a];   // its depth-`depth` ancestor
                    sub = a;
                    break;
                }
            first_sub[k] = sub;
            rec[k].swap(r);
        }
        std::unordered_map<int, int> sub_id;           // depth-`depth` subtrees in node order -> 0, 1, ...
        {
            std::vector<int> subs;
            for (int i = 0; i < nn; i++) if (dep[i] == depth) subs.push_back(i);
            for (size_t i = 0; i < subs.size(); i++) sub_id[subs[i]] = (int)i;
        }
        for (int64_t k = 0; k < L; k++) {
            xcd[0][k] = (int)(k * 8 / L);
            const int bk = orc_key_bucket(keys[k]);
            const int64_t lo = bstart[bk], hi = bstart[bk + 1];
            xcd[1][k] = (int)((k - lo) * 8 / std::max<int64_t>(1, hi - lo));
            auto it = sub_id.find(first_sub[k]);
            xcd[2][k] = it == sub_id.end() ? 0 : it->second % 8;
        }
        for (int pol = 0; pol < 3; pol++) {
            std::vector<std::vector<int64_t>> seq(8);
            for (int64_t k = 0; k < L; k++) seq[xcd[pol][k]].push_back(k);
            size_t biggest = 0;
            for (auto &q : seq) biggest = std::max(biggest, q.size());
            std::vector<std::pair<int, int64_t>> wins;  // (xcd, first index in its sequence)
            for (int x = 0; x < 8; x++) {
                const int64_t m = (int64_t)seq[x].size();
                if (m == 0) continue;
                const int64_t nw = std::max<int64_t>(1, (m + window - 1) / window);
                for (int w = 0; w < windows_per_xcd && w < nw; w++)
                    wins.push_back({x, (nw * w / windows_per_xcd) * window});
            }
            std::vector<double> distinct(wins.size()), fetched(wins.size());
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
            for (int64_t wi = 0; wi < (int64_t)wins.size(); wi++) {
                std::vector<uint8_t> seen_n(nn, 0), seen_t(s->triangles.size(), 0);
                const auto &q = seq[wins[wi].first];
                const int64_t a = wins[wi].second, e = std::min<int64_t>((int64_t)q.size(), a + window);
                double db = 0, fb = 0;
                for (int64_t j = a; j < e; j++)
                    for (uint32_t x : rec[q[j]]) {
                        const bool tri = x & kRecTri;
                        const uint32_t i = x & ~kRecTri;
                        fb += tri ? 48 : 64;
                        uint8_t &sn = tri ? seen_t[i] : seen_n[i];
                        if (!sn) { sn = 1; db += tri ? 48 : 64; }
                    }
                distinct[wi] = db;
                fetched[wi] = fb;
            }
            double mean = 0, mx = 0, fm = 0;
            for (size_t i = 0; i < wins.size(); i++) { mean += distinct[i]; mx = std::max(mx, distinct[i]); fm += fetched[i]; }
            out[pol * 6 + 0] = wins.empty() ? 0 : mean / wins.size();
            out[pol * 6 + 1] = mx;
            out[pol * 6 + 2] = wins.empty() ? 0 : fm / wins.size();
            out[pol * 6 + 3] = L ? (double)biggest / (double)L : 0;
            // whole-bounce L2 model, one XCD per thread
            constexpr int kWays = 16, kSets = (4 << 20) / 128 / kWays;
            const uint64_t tri_base = (uint64_t)nn * 64;
            std::vector<double> miss(8, 0), all(8, 0);
#pragma omp parallel for schedule(dynamic, 1) num_threads(std::min(nt, 8))
            for (int x = 0; x < 8; x++) {
                std::vector<uint64_t> tag((size_t)kSets * kWays, ~0ull), age((size_t)kSets * kWays, 0);
                uint64_t clock = 0;
                double ms = 0, fs = 0;
                auto touch = [&](uint64_t line) {
                    const size_t set = (size_t)(line % kSets) * kWays;
                    clock++;
                    size_t victim = set;
                    for (size_t w = set; w < set + kWays; w++) {
                        if (tag[w] == line) { age[w] = clock; return; }
                        if (age[w] < age[victim]) victim = w;
                    }
                    tag[victim] = line;
                    age[victim] = clock;
                    ms += 128;
                };
                for (int64_t k : seq[x])
                    for (uint32_t r : rec[k]) {
                        const bool tri = r & kRecTri;
                        const uint64_t a = tri ? tri_base + (uint64_t)(r & ~kRecTri) * 48 : (uint64_t)r * 64;
                        const uint64_t b = a + (tri ? 47 : 63);
                        fs += tri ? 48 : 64;
                        touch(a / 128);
                        if (b / 128 != a / 128) touch(b / 128);
                    }
                miss[x] = ms;
                all[x] = fs;
            }
            double mt = 0, ft = 0;
            for (int x = 0; x < 8; x++) { mt += miss[x]; ft += all[x]; }
            out[pol * 6 + 4] = mt;
            out[pol * 6 + 5] = ft;
        }
        {                                               // out[18..20]: overflow pushes, live rays, rays that overflow
            uint64_t t = 0, r = 0;
            for (int64_t k = 0; k < L; k++) { t += ovf[k]; r += ovf[k] != 0; }
            out[18] = (double)t;
            out[19] = (double)L;
            out[20] = (double)r;
        }
        return true;
    };
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3);
    Counters total;
    uint64_t sorted = 0;
    try {
        gpu_pass(s, pass, sort != 0, sum.data(), total, nullptr, &sorted, threads);
    } catch (...) {
        g_bounce_hook = nullptr;
        throw;
    }
    g_bounce_hook = nullptr;
    if (!done) { g_err = "bounce not reached"; return -1; }
    return 0;
}

// Analysis only (tools/wave_model.py): would a finer trace ORDER (not slot order: slots, seeds and results stay) make
// the trace kernel's waves more coherent at bounce `bounce`?  Every live ray's fetch sequence (internal-node steps and
// triangle steps) is replayed through one model wave of 64 lanes that refills idle lanes in order once `refill` are
// idle (the kernel's rule), in two orders: (0) slot order; (1) within each run of `tile` slots, stably sorted by a
// finer key (origin on a 2^obits grid per axis, direction on a 2^dbits grid, Morton-interleaved).  Per order, out[6]:
// iterations, node-body iterations, triangle-body iterations, lane-steps (= the useful work, the same for both),
// distinct 128-B record lines requested summed over iterations, and the steps of the longest ray.
int orc_bounce_wave_model(const orc_scene *s, int sort, int pass, int bounce, int tile, int obits, int dbits,
                          int refill, double *out, int threads) {
#ifndef ORC_ANALYSIS
    g_err = "analysis build only (liboracle.so)";
    return -1;
#endif
    if (pass < 0 || pass >= pass_total(s)) { g_err = "pass range"; return -1; }
    if (bounce < 0 || bounce >= s->bounces || tile < 1 || obits < 0 || obits > 5 || dbits < 0 || dbits > 5 ||
        refill < 1 || refill > 64) {
        g_err = "bad arguments"; return -1;
    }
    const int nt = nthreads(threads);
    const int nn = (int)s->bvh.size();
    bool done = false;
    g_bounce_hook = [&](int b, const std::vector<RayData> &rays, const std::vector<uint32_t> &idx,
                        const std::vector<uint32_t> &keys) {
        if (b != bounce) return false;
        done = true;
        int64_t L = 0;
        while (L < (int64_t)keys.size() && keys[L] != 0xFFFFFFFFu) L++;
        std::vector<std::vector<uint32_t>> rec(L);
        std::vector<uint32_t> fine(L);
        auto q = [](float v, int bits) {
            const float x = std::min(std::max(v, 0.0f), 0.999999f);
            return (uint32_t)(x * (float)(1u << bits));
        };
        auto spread = [](uint32_t v) {           // 5 bits -> every third bit
            uint32_t r = 0;
            for (int i = 0; i < 5; i++) r |= ((v >> i) & 1u) << (3 * i);
            return r;
        };
#pragma omp parallel for schedule(dynamic, 1024) num_threads(nt)
        for (int64_t k = 0; k < L; k++) {
            std::vector<uint32_t> r;
            g_rec = &r;
            float closest = 1e30f;
            int index = -1;
            Counters c;
            const RayData &rd = rays[idx[k]];
            bvh_closest_hit(s, rd.origin, rd.dir, closest, index, c);
            g_rec = nullptr;
            rec[k].swap(r);
            const V3 o = (rd.origin - s->min_coord) * s->inv_dimensions, d = 0.5f * (rd.dir + V3{1, 1, 1});
            const uint32_t ko = spread(q(o.x, obits)) | spread(q(o.y, obits)) << 1 | spread(q(o.z, obits)) << 2;
            const uint32_t kd = spread(q(d.x, dbits)) | spread(q(d.y, dbits)) << 1 | spread(q(d.z, dbits)) << 2;
            fine[k] = ko << 15 | kd;
        }
        const uint64_t tri_base = (uint64_t)nn * 64;
        for (int ord = 0; ord < 2; ord++) {
            std::vector<int64_t> order(L);
            for (int64_t k = 0; k < L; k++) order[k] = k;
            if (ord == 1)
                for (int64_t a = 0; a < L; a += tile) {
                    const int64_t e = std::min<int64_t>(L, a + tile);
                    std::stable_sort(order.begin() + a, order.begin() + e,
                                     [&](int64_t x, int64_t y) { return fine[x] < fine[y]; });
                }
            // one model wave per eighth of the order (the queue shards), summed
            double it = 0, itn = 0, itt = 0, lanes = 0, lines = 0, longest = 0;
#pragma omp parallel for schedule(static, 1) num_threads(std::min(nt, 8)) reduction(+ : it, itn, itt, lanes, lines) \
    reduction(max : longest)
            for (int sh = 0; sh < 8; sh++) {
                const int64_t lo = L * sh / 8, hi = L * (sh + 1) / 8;
                int64_t next = lo;
                int64_t ray[64];
                size_t pos[64];
                for (int l = 0; l < 64; l++) ray[l] = -1;
                std::vector<uint64_t> ln;
                while (true) {
                    int idle = 0;
                    for (int l = 0; l < 64; l++) idle += ray[l] < 0;
                    if (idle >= refill || idle == 64)
                        for (int l = 0; l < 64 && next < hi; l++)
                            if (ray[l] < 0) {
                                ray[l] = order[next++];
                                pos[l] = 0;
                                longest = std::max(longest, (double)rec[ray[l]].size());
                            }
                    bool any = false, anyn = false, anyt = false;
                    ln.clear();
                    for (int l = 0; l < 64; l++) {
                        if (ray[l] < 0) continue;
                        const auto &r = rec[ray[l]];
                        if (pos[l] >= r.size()) { ray[l] = -1; continue; }
                        const uint32_t x = r[pos[l]++];
                        const bool tri = x & kRecTri;
                        (tri ? anyt : anyn) = true;
                        any = true;
                        lanes += 1;
                        const uint64_t a = tri ? tri_base + (uint64_t)(x & ~kRecTri) * 48 : (uint64_t)x * 64;
                        ln.push_back(a / 128);
                        if ((a + (tri ? 47 : 63)) / 128 != a / 128) ln.push_back((a + (tri ? 47 : 63)) / 128);
                    }
                    if (!any) {
                        if (next >= hi) break;
                        continue;
                    }
                    it += 1;
                    itn += anyn;
                    itt += anyt;
                    std::sort(ln.begin(), ln.end());
                    lines += (double)(std::unique(ln.begin(), ln.end()) - ln.begin());
                }
            }
            out[ord * 6 + 0] = it;
            out[ord * 6 + 1] = itn;
            out[ord * 6 + 2] = itt;
            out[ord * 6 + 3] = lanes;
            out[ord * 6 + 4] = lines;
            out[ord * 6 + 5] = longest;
        }
        return true;
    };
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<float> sum(pixels * 3);
    Counters total;
    uint64_t sorted = 0;
    try {
        gpu_pass(s, pass, sort != 0, sum.data(), total, nullptr, &sorted, threads);
    } catch (...) {
        g_bounce_hook = nullptr;
        throw;
    }
    g_bounce_hook = nullptr;
    if (!done) { g_err = "bounce not reached"; return -1; }
    return 0;
}

int orc_render_pass_sums(const orc_scene *s, int sort, int pass_begin, int pass_count, float *out, int threads) {
    const int P = pass_total(s);
    if (pass_count < 0) pass_count = P - pass_begin;
    if (pass_begin < 0 || pass_begin + pass_count > P) { g_err = "pass range"; return -1; }
    const int64_t pixels = (int64_t)s->width * s->height;
    Counters total;
    uint64_t sorted = 0;
    for (int p = pass_begin; p < pass_begin + pass_count; p++)
        gpu_pass(s, p, sort != 0, out + (size_t)(p - pass_begin) * pixels * 3, total, nullptr, &sorted, threads);
    return 0;
}

// raytracing.cu:122-163 (timed span = "CPU Took").  The inner loop's `i` shadows the bounce index,
// so the seed does not depend on the bounce (raytracing.cu:142-149).
int orc_render_cpu_path(const orc_scene *s, float *fb, int pass_limit, int threads, double *seconds) {
    return orc_render_cpu_path_counted(s, fb, pass_limit, threads, seconds, nullptr);
}

int orc_render_cpu_path_counted(const orc_scene *s, float *fb, int pass_limit, int threads, double *seconds,
                                uint64_t *live_out) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    const int nt = nthreads(threads);
    const int64_t pixels = (int64_t)s->width * s->height;
    std::vector<RayData> rays((size_t)pixels * 20);
    std::memset(fb, 0, sizeof(float) * pixels * 3);
    int remaining = s->ray_count;
    int passes = 0;
    Counters dummy;
    while (remaining && (pass_limit < 0 || passes < pass_limit)) {
        const int rtc = std::min(remaining, 20);
        remaining -= rtc;
        const int total = rtc * s->width * s->height;
#pragma omp parallel for schedule(dynamic, 1000) num_threads(nt)
        for (int i = 0; i < total; i++) generate_ray(s, rays.data(), nullptr, nullptr, rtc, i, remaining);
        for (int b = 0; b < s->bounces; b++) {
            uint64_t live = 0;
#pragma omp parallel for schedule(dynamic, 1000) num_threads(nt) reduction(+ : live)
            for (int i = 0; i < total; i++) {
                Rng rng;
                xor_srand(&rng, 1905678123u * (uint32_t)i + 345903u * (uint32_t)(remaining * 20 + i));
                Counters c;
                process_ray(s, &rays[i], nullptr, rng, false, c);
                live += c.live;
            }
            if (live_out) *live_out += live;
        }
        for (int i = 0; i < total; i++) {                    // raytracing.cu:114-120
            float *p = fb + (size_t)(i / rtc) * 3;
            p[0] = p[0] + rays[i].collected.x;
            p[1] = p[1] + rays[i].collected.y;
            p[2] = p[2] + rays[i].collected.z;
        }
        passes++;
    }
    (void)dummy;
    const auto t1 = std::chrono::high_resolution_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    return passes;
}

// raytracing.cu:21-74 with the launch parameters of :376-382.
void orc_closest_hit(const orc_scene *s, const float *rays, int n, float *t_out, int32_t *index_out, orc_stats *st) {
    Counters c;
    const int sphere_count = (int)s->spheres.size();
    for (int i = 0; i < n; i++) {
        const float *r = rays + (size_t)i * 6;
        const V3 o{r[0], r[1], r[2]}, d{r[3], r[4], r[5]};
        float closest = 1e30f;                 // scene.cu:328-374, as process_ray
        int index = -1;
        for (int k = 0; k < sphere_count; k++) {
            c.st++;
            float t;
            if (ray_sphere(s->spheres[k], o, d, closest, &t)) { closest = t; index = k; }
        }
        bvh_closest_hit(s, o, d, closest, index, c);
        if (t_out) t_out[i] = closest;
        if (index_out) index_out[i] = index;
    }
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->live_segments = (uint64_t)n;
        st->nodes_popped = c.pn;
        st->internal_visits = c.iv;
        st->triangle_tests = c.tt;
        st->sphere_tests = c.st;
        st->max_stack = c.max_stack;
    }
}

void orc_bloom(float *fb, int w, int h, float threshold, int radius) {
    const int64_t n = (int64_t)w * h;
    std::vector<V3> img(n), bright(n), blur(n);
    std::memcpy(img.data(), fb, sizeof(V3) * n);
    for (int64_t i = 0; i < n; i++) {
        const float lum = dot(img[i], V3{0.2126f, 0.7152f, 0.0722f});
        bright[i] = lum > threshold ? img[i] : V3{0, 0, 0};
    }
    for (int64_t i = 0; i < n; i++) {
        const int x = (int)(i % w), y = (int)(i / w);
        V3 sum{0, 0, 0};
        int count = 0;
        for (int dx = -radius; dx <= radius; dx++) {
            const int nx = x + dx;
            if (nx >= 0 && nx < w) { sum = sum + bright[(int64_t)y * w + nx]; count++; }
        }
        blur[i] = (1.0f / count) * sum;
    }
    for (int64_t i = 0; i < n; i++) {
        const int x = (int)(i % w), y = (int)(i / w);
        V3 sum{0, 0, 0};
        int count = 0;
        for (int dy = -radius; dy <= radius; dy++) {
            const int ny = y + dy;
            if (ny >= 0 && ny < h) { sum = sum + blur[(int64_t)ny * w + x]; count++; }
        }
        bright[i] = (1.0f / count) * sum;
    }
    for (int64_t i = 0; i < n; i++) img[i] = img[i] + bright[i];
    std::memcpy(fb, img.data(), sizeof(V3) * n);
}

// raytracing.cu:286-303
void orc_tonemap(const float *fb, int w, int h, float exposure, int ray_count, uint8_t *out) {
    const float scale = exposure / ray_count;
    for (int64_t i = 0; i < (int64_t)w * h * 3; i++) {
        const float p = scale * fb[i];
        const float v = sqrtf(p / (p + 1)) * 255.999f;
        out[i] = (v == v && v > 0) ? (uint8_t)(int)v : 0;
    }
}

void orc_pcg_stream(uint32_t seed, int n, uint32_t *out) {
    Rng r;
    xor_srand(&r, seed);
    for (int i = 0; i < n; i++) out[i] = xor_rand(&r);
}
void orc_random_draws(uint32_t seed, int n, float *r01, float *r02, float *rad) {
    Rng a, b, c;
    xor_srand(&a, seed); xor_srand(&b, seed); xor_srand(&c, seed);
    for (int i = 0; i < n; i++) { r01[i] = random01(&a); r02[i] = random02(&b); rad[i] = random_radians(&c); }
}
void orc_random_on_sphere(uint32_t seed, int n, float *out) {
    Rng r;
    xor_srand(&r, seed);
    for (int i = 0; i < n; i++) {
        const V3 v = random_on_sphere(&r);
        out[3 * i] = v.x; out[3 * i + 1] = v.y; out[3 * i + 2] = v.z;
    }
}
void orc_sincos(const float *x, int n, float *s, float *c) {
    for (int i = 0; i < n; i++) rt_sincos(x[i], &s[i], &c[i]);
}
float orc_atan01(float x) { return rt_atan01(x); }
uint32_t orc_generate_seed(int32_t i, int32_t seed) { return (uint32_t)i * 0x85810BEAu + 709579u * (uint32_t)seed; }
uint32_t orc_process_seed(int32_t slot, int32_t seed) { return (uint32_t)slot * 4137874753u + 279220567u * (uint32_t)seed; }
uint32_t orc_cpu_seed(int32_t i, int32_t rem) { return 1905678123u * (uint32_t)i + 345903u * (uint32_t)(rem * 20 + i); }
uint16_t orc_interleave_5(uint16_t x) { return interleave_5(x); }
uint32_t orc_morton(float x, float y, float z) { return morton_code(V3{x, y, z}); }
int orc_key_bucket(uint32_t key) {
    if (key == 0xFFFFFFFFu) return 64;
    const uint32_t mo = key >> 16, md = key & 0xFFFF;
    const uint32_t qo = (mo & 1) | (((mo >> 1) & 1) << 1) | (((mo >> 2) & 1) << 2);
    const uint32_t qd = (md & 1) | (((md >> 1) & 1) << 1) | (((md >> 2) & 1) << 2);
    return (int)((qo << 3) | qd);
}
int orc_ray_aabb(const float *bmin, const float *bmax, const float *o, const float *d, float tmax, float *tmin) {
    Aabb b;
    b.mn = {bmin[0], bmin[1], bmin[2]};
    b.mx = {bmax[0], bmax[1], bmax[2]};
    const V3 n_inv{1 / d[0], 1 / d[1], 1 / d[2]};
    return ray_aabb(b, V3{o[0], o[1], o[2]}, n_inv, *tmin, tmax) ? 1 : 0;
}
int orc_ray_triangle(const float *t12, const float *o, const float *d, float closest, float *t) {
    Triangle tr;
    std::memcpy(&tr, t12, 48);
    return ray_tri(tr, V3{o[0], o[1], o[2]}, V3{d[0], d[1], d[2]}, closest, t) ? 1 : 0;
}
int orc_ray_sphere(const float *s4, const float *o, const float *d, float closest, float *t) {
    Sphere sp{{s4[0], s4[1], s4[2]}, s4[3]};
    return ray_sphere(sp, V3{o[0], o[1], o[2]}, V3{d[0], d[1], d[2]}, closest, t) ? 1 : 0;
}
void orc_env_project(const float *dir, float *uv) {
    const V3 r = equal_area_project(V3{dir[0], dir[1], dir[2]});
    uv[0] = r.x; uv[1] = r.y;
}
int orc_env_texel(const float *dir, int w, int h) {
    orc_scene s;
    s.env_w = w; s.env_h = h;
    return env_texel(&s, V3{dir[0], dir[1], dir[2]});
}

}  // extern "C"
