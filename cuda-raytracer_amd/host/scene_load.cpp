// scene_load.cpp — host scene loading and BVH construction for the MI355X path tracer.
//
// Implements rt_scene_load (include/rt_abi.h), the drop-in for load_scene
// (reference scene.cu:569-831) and Scene::generate_bvh (scene.cu:1002-1036).  The
// arrays it produces are the inputs of both the HIP path and the CPU path, so they must be
// byte-identical to the reference's: the binned-SAH split search below keeps the
// reference's float expression order, its fminf/fmaxf tie semantics and its in-place
// partition (tests/test_scene_parity.py checks this against the oracle).
#include "rt_abi.h"
#include "rt_host.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

namespace rtamd {

thread_local std::string g_error;

int fail(int code, const std::string &msg) {
    g_error = msg;
    return code;
}

namespace {

// fminf/fmaxf as glibc implements them (the reference's host min/max, math.cuh:126-142).
inline float fmin_(float a, float b) { if (a != a) return b; if (b != b) return a; return (b < a) ? b : a; }
inline float fmax_(float a, float b) { if (a != a) return b; if (b != b) return a; return (b > a) ? b : a; }
inline rt_vec3 add(rt_vec3 a, rt_vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline rt_vec3 sub(rt_vec3 a, rt_vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline rt_vec3 scale(float s, rt_vec3 v) { return {s * v.x, s * v.y, s * v.z}; }
inline rt_vec3 cross(rt_vec3 a, rt_vec3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline rt_vec3 normalise(rt_vec3 v) { return scale(1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z), v); }
inline rt_vec3 vmin(rt_vec3 a, rt_vec3 b) { return {fmin_(a.x, b.x), fmin_(a.y, b.y), fmin_(a.z, b.z)}; }
inline rt_vec3 vmax(rt_vec3 a, rt_vec3 b) { return {fmax_(a.x, b.x), fmax_(a.y, b.y), fmax_(a.z, b.z)}; }
inline rt_vec3 centroid(rt_vec3 a, rt_vec3 b, rt_vec3 c) { return scale(1.0f / 3.0f, add(add(a, b), c)); }

struct Box {
    rt_vec3 lo{1e30f, 1e30f, 1e30f}, hi{-1e30f, -1e30f, -1e30f};
    void grow(rt_vec3 p) { lo = vmin(lo, p); hi = vmax(hi, p); }
    void grow(const rt_triangle &t) { grow(t.p1); grow(t.p2p1); grow(t.p3p1); }
    void grow(const Box &b) { lo = vmin(lo, b.lo); hi = vmax(hi, b.hi); }
    float half_area() const {
        const rt_vec3 s = sub(hi, lo);
        return s.x * s.y + s.x * s.z + s.y * s.z;
    }
};

// Binned SAH builder (scene.cu:866-1000).  Triangles are in build representation
// (p1, p2, p3, centroid); `cent` caches the per-axis centroid so the split search reads
// 12 B instead of 48 B per triangle.
class BvhBuilder {
public:
    BvhBuilder(std::vector<rt_triangle> &tris, uint16_t *tri_mats, std::vector<rt_bvh_node> &nodes)
        : tris_(tris), mats_(tri_mats), nodes_(nodes) {}

    void build(int max_depth) {
        nodes_.clear();
        nodes_.reserve(std::max<size_t>(1, tris_.size() * 2));
        rt_bvh_node root{};
        root.min_bound = {1e30f, 1e30f, 1e30f};
        root.max_bound = {-1e30f, -1e30f, -1e30f};
        root.child2 = 0;
        root.child1 = (int32_t)tris_.size();
        nodes_.push_back(root);
        split(0, max_depth);
    }

private:
    static constexpr int kBins = 8;
    std::vector<rt_triangle> &tris_;
    uint16_t *mats_;
    std::vector<rt_bvh_node> &nodes_;

    static float axis_of(const rt_vec3 &v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

    void split(int ni, int max_depth) {
        const int lo = nodes_[ni].child2, hi = nodes_[ni].child1;
        Box box;
        box.lo = nodes_[ni].min_bound;
        box.hi = nodes_[ni].max_bound;
        for (int i = lo; i < hi; i++) box.grow(tris_[i]);
        nodes_[ni].min_bound = box.lo;
        nodes_[ni].max_bound = box.hi;
        const int count = hi - lo;
        if (count <= 4 || max_depth == 0) return;
        const float own_cost = box.half_area() * count;
        int best_axis = 0;
        float best_pos = 0, best_cost = own_cost;
        for (int axis = 0; axis < 3; axis++) {
            float cmin = 1e30f, cmax = -1e30f;
            for (int i = lo; i < hi; i++) {
                const float c = axis_of(tris_[i].normal, axis);
                cmin = fmin_(cmin, c);
                cmax = fmax_(cmax, c);
            }
            if (cmin == cmax) continue;
            const float k = kBins / (cmax - cmin);
            Box bins[kBins];
            int counts[kBins] = {0};
            for (int i = lo; i < hi; i++) {
                const int b = std::min(kBins - 1, (int)((axis_of(tris_[i].normal, axis) - cmin) * k));
                counts[b]++;
                bins[b].grow(tris_[i]);
            }
            float larea[kBins - 1], rarea[kBins - 1];
            int lcount[kBins - 1];
            Box lbox, rbox;
            int lsum = 0;
            for (int i = 0; i + 1 < kBins; i++) {
                lsum += counts[i];
                lcount[i] = lsum;
                lbox.grow(bins[i]);
                larea[i] = lbox.half_area();
                rbox.grow(bins[kBins - 1 - i]);
                rarea[kBins - 2 - i] = rbox.half_area();
            }
            const float step = (cmax - cmin) / kBins;
            for (int i = 0; i + 1 < kBins; i++) {
                const float cost = lcount[i] * larea[i] + (count - lcount[i]) * rarea[i];
                if (cost != 0 && cost < best_cost) {
                    best_axis = axis;
                    best_pos = cmin + step * (i + 1);
                    best_cost = cost;
                }
            }
        }
        if (best_cost >= own_cost) return;
        // In-place two-pointer partition, swapping material indices along (scene.cu:960-975).
        int i = lo, j = hi - 1;
        while (i <= j) {
            if (axis_of(tris_[i].normal, best_axis) < best_pos) {
                i++;
            } else {
                std::swap(tris_[i], tris_[j]);
                std::swap(mats_[i], mats_[j]);
                j--;
            }
        }
        if (i == hi || i == lo) return;
        const int left = (int)nodes_.size();
        rt_bvh_node child{};
        child.min_bound = {1e30f, 1e30f, 1e30f};
        child.max_bound = {-1e30f, -1e30f, -1e30f};
        child.child2 = lo;
        child.child1 = i;
        nodes_.push_back(child);
        child.child2 = i;
        child.child1 = hi;
        nodes_.push_back(child);
        split(left, max_depth - 1);
        split(left + 1, max_depth - 1);
        nodes_[ni].child1 = left;
        nodes_[ni].child2 = left + 1;
    }
};

std::string resolve(const char *root, const std::string &p) {
    if (!root || !*root || (!p.empty() && p[0] == '/')) return p;
    std::string r(root);
    if (r.back() != '/') r += '/';
    return r + p;
}

std::vector<std::string> tokens_of(const std::string &line) {
    std::vector<std::string> t;
    size_t i = 0;
    while (i < line.size()) {
        while (i < line.size() && std::isspace((unsigned char)line[i])) i++;
        const size_t b = i;
        while (i < line.size() && !std::isspace((unsigned char)line[i])) i++;
        if (i > b) t.emplace_back(line, b, i - b);
    }
    return t;
}
float fnum(const std::vector<std::string> &t, size_t i) { return i < t.size() ? std::strtof(t[i].c_str(), nullptr) : 0.0f; }
int inum(const std::vector<std::string> &t, size_t i) { return i < t.size() ? (int)std::strtol(t[i].c_str(), nullptr, 10) : 0; }

// Binary little-endian PLY as exported by pbrt-v4 scenes (scene.cu:491-546): vertex
// records of 8 floats (x y z nx ny nz u v), faces as uint8 count + int32 indices,
// triangulated as a fan.  The header is parsed by keyword instead of by fixed line
// offsets, which yields the same result on the reference's files.
int load_ply(const std::string &path, std::vector<rt_triangle> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(RT_E_IO, "cannot open ply file '" + path + "'");
    std::string line;
    long vcount = -1, fcount = -1;
    int vprops = 0;
    bool in_vertex = false;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const auto t = tokens_of(line);
        if (t.empty()) continue;
        if (t[0] == "element" && t.size() >= 3) {
            in_vertex = t[1] == "vertex";
            if (in_vertex) vcount = std::strtol(t[2].c_str(), nullptr, 10);
            else if (t[1] == "face") fcount = std::strtol(t[2].c_str(), nullptr, 10);
        } else if (t[0] == "property" && in_vertex) {
            vprops++;
        } else if (t[0] == "end_header") {
            break;
        }
    }
    if (vcount < 0 || fcount < 0 || vprops != 8)
        return fail(RT_E_IO, "unsupported ply header in '" + path + "'");
    std::vector<float> verts((size_t)vcount * 8);
    f.read(reinterpret_cast<char *>(verts.data()), (std::streamsize)(verts.size() * sizeof(float)));
    std::vector<char> rest((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    size_t pos = 0;
    std::vector<int32_t> idx;
    out.reserve(out.size() + (size_t)fcount);
    for (long k = 0; k < fcount; k++) {
        if (pos >= rest.size()) return fail(RT_E_IO, "truncated ply file '" + path + "'");
        const int n = (unsigned char)rest[pos++];
        if (pos + 4 * (size_t)n > rest.size()) return fail(RT_E_IO, "truncated ply file '" + path + "'");
        idx.resize(n);
        std::memcpy(idx.data(), rest.data() + pos, 4 * (size_t)n);
        pos += 4 * (size_t)n;
        for (int j = 2; j < n; j++) {
            for (int q : {idx[0], idx[j - 1], idx[j]})
                if (q < 0 || q >= vcount) return fail(RT_E_IO, "ply index out of range in '" + path + "'");
            auto vtx = [&](int q) { return rt_vec3{verts[8 * (size_t)q], verts[8 * (size_t)q + 1], verts[8 * (size_t)q + 2]}; };
            rt_triangle t;
            t.p1 = vtx(idx[0]);
            t.p2p1 = vtx(idx[j - 1]);
            t.p3p1 = vtx(idx[j]);
            t.normal = centroid(t.p1, t.p2p1, t.p3p1);
            out.push_back(t);
        }
    }
    return RT_OK;
}

// Raw PFM (scene.cu:548-567): "PF", "W H", scale line, then W*H RGB floats, no flip.
int load_pfm(const std::string &path, std::vector<rt_vec3> &env, int &w, int &h) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(RT_E_IO, "cannot open environment map '" + path + "'");
    std::string line;
    std::getline(f, line);
    std::getline(f, line);
    std::stringstream ss(line);
    w = h = 0;
    ss >> w >> h;
    std::getline(f, line);
    if (w <= 0 || h <= 0) return fail(RT_E_IO, "bad pfm header in '" + path + "'");
    env.assign((size_t)w * h, rt_vec3{0, 0, 0});
    f.read(reinterpret_cast<char *>(env.data()), (std::streamsize)(env.size() * sizeof(rt_vec3)));
    return RT_OK;
}

}  // namespace
}  // namespace rtamd

struct rt_scene_host {
    rt_scene view{};
    std::vector<rt_sphere> spheres;
    std::vector<rt_triangle> triangles;
    std::vector<uint16_t> material_indices;
    std::vector<rt_material> materials;
    std::vector<rt_bvh_node> bvh;
    std::vector<rt_vec3> env;
    double bvh_ms = 0;
};

using namespace rtamd;

extern "C" {

void rt_default_load_opts(rt_load_opts *o) {
    std::memset(o, 0, sizeof(*o));
    o->use_bvh = 1;
}

int rt_scene_load(const char *path, const rt_load_opts *opts_in, rt_scene_host **out) {
    if (!path || !out) return fail(RT_E_INVALID, "rt_scene_load: null argument");
    *out = nullptr;
    rt_load_opts opts;
    if (opts_in) opts = *opts_in; else rt_default_load_opts(&opts);
    std::ifstream file(path);
    if (!file) return fail(RT_E_IO, std::string("cannot open scene file '") + path + "'");
    auto s = new rt_scene_host();
    rt_scene &v = s->view;
    v.width = 1920;                                   // scene.cu:571-574
    v.height = 1080;
    v.ray_count = 1;
    v.bounces = 3;
    std::unordered_map<std::string, uint16_t> mat_ids;
    std::vector<uint16_t> sphere_mats, tri_mats;
    bool have_env = false;
    auto bad = [&](int code) { delete s; return code; };
    for (std::string line; std::getline(file, line);) {
        while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
        if (line.empty()) continue;
        const std::string cmd = line.substr(0, line.find(' '));
        const auto t = tokens_of(line);
        auto material = [&](size_t i, uint16_t *id) {
            if (i >= t.size()) return false;
            auto it = mat_ids.find(t[i]);
            if (it == mat_ids.end()) { g_error = "unknown material '" + t[i] + "'"; return false; }
            *id = it->second;
            return true;
        };
        if (cmd == "sky") {
            s->env.assign(1, rt_vec3{fnum(t, 1), fnum(t, 2), fnum(t, 3)});
            v.environment_map_width = v.environment_map_height = 1;
            have_env = true;
        } else if (cmd == "sky_map") {
            if (t.size() < 2) return bad(fail(RT_E_INVALID, "sky_map without a path"));
            const int rc = load_pfm(resolve(opts.asset_root, t[1]), s->env, v.environment_map_width,
                                    v.environment_map_height);
            if (rc) return bad(rc);
            have_env = true;
            if (!opts.quiet)
                std::printf("Loaded environment map with size %d,%d\n", v.environment_map_width, v.environment_map_height);
        } else if (cmd == "camera") {
            v.camera_position = {fnum(t, 2), fnum(t, 3), fnum(t, 4)};
            v.forward = normalise(rt_vec3{fnum(t, 6), fnum(t, 7), fnum(t, 8)});
            v.up = normalise(rt_vec3{fnum(t, 10), fnum(t, 11), fnum(t, 12)});
            v.vertical_fov = (float)(fnum(t, 14) * (3.14159265358979323846 / 180));
        } else if (cmd == "material") {
            if (t.size() < 2) continue;
            mat_ids[t[1]] = (uint16_t)s->materials.size();
            rt_material m;
            m.specular_albedo = {1, 1, 1};
            m.diffuse_albedo = {1, 1, 1};
            m.emitted = {0, 0, 0};
            m.metallicity = 0;
            m.roughness = 0;
            m.index_of_refraction = 0;
            for (size_t k = 2; k < t.size(); k++) {
                const std::string &p = t[k];
                if (p == "diffuse") { m.diffuse_albedo = {fnum(t, k + 1), fnum(t, k + 2), fnum(t, k + 3)}; k += 3; }
                else if (p == "specular") { m.specular_albedo = {fnum(t, k + 1), fnum(t, k + 2), fnum(t, k + 3)}; k += 3; }
                else if (p == "emit") { m.emitted = {fnum(t, k + 1), fnum(t, k + 2), fnum(t, k + 3)}; k += 3; }
                else if (p == "metallicity") m.metallicity = fnum(t, ++k);
                else if (p == "roughness") m.roughness = fnum(t, ++k);
                else if (p == "ior") m.index_of_refraction = fnum(t, ++k);
            }
            s->materials.push_back(m);
        } else if (cmd == "sphere") {
            uint16_t id;
            if (!material(1, &id)) return bad(RT_E_INVALID);
            sphere_mats.push_back(id);
            s->spheres.push_back(rt_sphere{{fnum(t, 2), fnum(t, 3), fnum(t, 4)}, fnum(t, 5)});
        } else if (cmd == "triangle" || cmd == "quad") {
            uint16_t id;
            if (!material(1, &id)) return bad(RT_E_INVALID);
            const rt_vec3 p1{fnum(t, 2), fnum(t, 3), fnum(t, 4)}, p2{fnum(t, 5), fnum(t, 6), fnum(t, 7)};
            const rt_vec3 p3{fnum(t, 8), fnum(t, 9), fnum(t, 10)};
            s->triangles.push_back(rt_triangle{p1, p2, p3, centroid(p1, p2, p3)});
            tri_mats.push_back(id);
            if (cmd == "quad") {                      // corners (0,1,2) and (0,2,3), scene.cu:761-775
                const rt_vec3 p4{fnum(t, 11), fnum(t, 12), fnum(t, 13)};
                s->triangles.push_back(rt_triangle{p1, p3, p4, centroid(p1, p3, p4)});
                tri_mats.push_back(id);
            }
        } else if (cmd == "ply") {
            uint16_t id;
            if (!material(1, &id)) return bad(RT_E_INVALID);
            if (t.size() < 3) return bad(fail(RT_E_INVALID, "ply without a path"));
            const size_t before = s->triangles.size();
            const int rc = load_ply(resolve(opts.asset_root, t[2]), s->triangles);
            if (rc) return bad(rc);
            tri_mats.insert(tri_mats.end(), s->triangles.size() - before, id);
        } else if (cmd == "image") {
            v.width = inum(t, 1);
            v.height = inum(t, 2);
            v.ray_count = inum(t, 3);
            v.bounces = inum(t, 4);
            v.exposure = fnum(t, 5);
        }
    }
    if (opts.image_override) {
        v.width = opts.width;
        v.height = opts.height;
        v.ray_count = opts.ray_count;
        v.bounces = opts.bounces;
    }
    if (opts.exposure_override) v.exposure = opts.exposure;
    if (v.width < 2 || v.height < 2 || v.ray_count < 0 || v.bounces < 0)
        return bad(fail(RT_E_INVALID, "scene image must be at least 2x2 with non-negative spp/bounces"));
    if (!have_env) {                                  // reference reads an unset map: UB
        s->env.assign(1, rt_vec3{0, 0, 0});
        v.environment_map_width = v.environment_map_height = 1;
    }
    if (s->spheres.size() + s->triangles.size() > 0x7fffffff || s->materials.size() > 65535)
        return bad(fail(RT_E_INVALID, "scene too large"));
    s->material_indices = sphere_mats;
    s->material_indices.insert(s->material_indices.end(), tri_mats.begin(), tri_mats.end());

    // Camera precompute (scene.cu:62-76).
    const rt_vec3 right = cross(v.up, v.forward);
    const float nph = 2.0f * std::tan(v.vertical_fov * 0.5f);
    const float npw = nph * v.width / v.height;
    v.scaled_right = scale(npw, right);
    v.scaled_up = scale(nph, v.up);
    v.near_plane_top_left = add(sub(v.forward, scale(0.5f, v.scaled_right)), scale(0.5f, v.scaled_up));
    v.inv_width = 1.0f / (v.width - 1);
    v.inv_height = 1.0f / (v.height - 1);

    // BVH (scene.cu:1002-1036), then the ray-tracing triangle representation.
    const auto t0 = std::chrono::high_resolution_clock::now();
    BvhBuilder(s->triangles, s->material_indices.data() + s->spheres.size(), s->bvh).build(opts.use_bvh ? 30 : 0);
    const auto t1 = std::chrono::high_resolution_clock::now();
    s->bvh_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (!opts.quiet) {
        std::printf("Triangle count: %zu\n", s->triangles.size());
        std::printf("BVH Took %gms\n", s->bvh_ms);
        std::printf("Node count: %zu\n", s->bvh.size());
    }
    for (auto &tr : s->triangles) {
        tr.p2p1 = sub(tr.p2p1, tr.p1);
        tr.p3p1 = sub(tr.p3p1, tr.p1);
        tr.normal = normalise(cross(tr.p3p1, tr.p2p1));
    }
    // Reorder-key bounds (scene.cu:822-830): note inv_dimensions = 1 / max, not 1 / (max - min).
    v.min_coord = s->bvh[0].min_bound;
    rt_vec3 mx = s->bvh[0].max_bound;
    for (const auto &sp : s->spheres) {
        const rt_vec3 r{sp.radius, sp.radius, sp.radius};
        mx = vmax(mx, add(sp.center, r));
        v.min_coord = vmin(v.min_coord, sub(sp.center, r));
    }
    v.inv_dimensions = {1 / mx.x, 1 / mx.y, 1 / mx.z};

    v.spheres = s->spheres.data();
    v.sphere_count = (int32_t)s->spheres.size();
    v.triangles = s->triangles.data();
    v.triangle_count = (int32_t)s->triangles.size();
    v.material_indices = s->material_indices.data();
    v.materials = s->materials.data();
    v.material_count = (int32_t)s->materials.size();
    v.bvh = s->bvh.data();
    v.bvh_node_count = (int32_t)s->bvh.size();
    v.environment_map = s->env.data();
    *out = s;
    return RT_OK;
}

const rt_scene *rt_scene_view(const rt_scene_host *s) { return s ? &s->view : nullptr; }
double rt_scene_bvh_ms(const rt_scene_host *s) { return s ? s->bvh_ms : 0.0; }
void rt_scene_free(rt_scene_host *s) { delete s; }
const char *rt_last_error(void) { return g_error.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

}  // extern "C"
