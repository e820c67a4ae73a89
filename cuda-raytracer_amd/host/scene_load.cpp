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
#include <atomic>
#include <thread>
#include <vector>

namespace rtamd {

thread_local std::string g_error;

int fail(int code, const std::string &msg) {
    g_error = msg;
    return code;
}

// GPU binned-SAH build (csrc/bvh_build.hip): same output as BvhBuilder below.
int gpu_build_bvh(std::vector<rt_triangle> &tris, uint16_t *tri_mats, std::vector<rt_bvh_node> &nodes,
                  int max_depth, int device);

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
// (p1, p2, p3, centroid).
//
// Same decisions and the same output as the reference's single-threaded recursion, faster:
// * per-triangle boxes and the three centroid coordinates live in side arrays (permuted with
//   the triangles), so the bound and binning passes read 24 + 4 B per triangle instead of
//   48 B and grow by 6 min/max instead of 18 (the reference's min keeps the earliest of equal
//   values, which makes growing by a triangle's box equal to growing by its three vertices);
// * subtrees of at least kParallelMin triangles are built on their own thread.  Splitting X
//   appends X's two children, then the first child's subtree, then the second's; a subtree's
//   shape and triangle order depend only on its own range, so it can be built into a
//   separate array with the same local numbering and spliced in with child indices shifted.
// The node array and triangle order are byte-identical to the serial build
// (tests/test_scene_parity.py compares them with the oracle's serial restatement).
class BvhBuilder {
public:
    BvhBuilder(std::vector<rt_triangle> &tris, uint16_t *tri_mats, std::vector<rt_bvh_node> &nodes)
        : tris_(tris), mats_(tri_mats), nodes_(nodes) {}

    void build(int max_depth, int threads) {
        const int n = (int)tris_.size();
        box_.resize(n);
        for (int a = 0; a < 3; a++) cent_[a].resize(n);
        for (int i = 0; i < n; i++) {
            box_[i] = Box();
            box_[i].grow(tris_[i]);
            cent_[0][i] = tris_[i].normal.x;
            cent_[1][i] = tris_[i].normal.y;
            cent_[2][i] = tris_[i].normal.z;
        }
        spare_threads_ = threads - 1;
        nodes_.clear();
        rt_bvh_node root = fresh(0, n);
        std::vector<rt_bvh_node> desc;
        build_desc(root, max_depth, desc);
        nodes_.reserve(1 + desc.size());
        nodes_.push_back(shifted(root, 1));
        for (const rt_bvh_node &d : desc) nodes_.push_back(shifted(d, 1));
    }

private:
    static constexpr int kBins = 8;
    static constexpr int kParallelMin = 4096;   // smaller subtrees are not worth a thread
    std::vector<rt_triangle> &tris_;
    uint16_t *mats_;
    std::vector<rt_bvh_node> &nodes_;
    std::vector<Box> box_;
    std::vector<float> cent_[3];
    std::atomic<int> spare_threads_{0};

    static rt_bvh_node fresh(int lo, int hi) {  // a child as the reference creates it
        rt_bvh_node n{};
        n.min_bound = {1e30f, 1e30f, 1e30f};
        n.max_bound = {-1e30f, -1e30f, -1e30f};
        n.child2 = lo;
        n.child1 = hi;
        return n;
    }
    // internal nodes have child1 < child2 (adjacent children); leaves child2 <= child1
    static rt_bvh_node shifted(rt_bvh_node n, int by) {
        if (n.child1 < n.child2) { n.child1 += by; n.child2 += by; }
        return n;
    }

    // Bounds of node n's range, then the split decision and the in-place partition of
    // scene.cu:866-1000.  Returns the split index, or -1 when n stays a leaf.
    int decide(rt_bvh_node &n, int max_depth) {
        const int lo = n.child2, hi = n.child1;
        Box box;
        box.lo = n.min_bound;
        box.hi = n.max_bound;
        for (int i = lo; i < hi; i++) box.grow(box_[i]);
        n.min_bound = box.lo;
        n.max_bound = box.hi;
        const int count = hi - lo;
        if (count <= 4 || max_depth == 0) return -1;
        const float own_cost = box.half_area() * count;
        int best_axis = 0;
        float best_pos = 0, best_cost = own_cost;
        for (int axis = 0; axis < 3; axis++) {
            const float *c = cent_[axis].data();
            float cmin = 1e30f, cmax = -1e30f;
            for (int i = lo; i < hi; i++) {
                cmin = fmin_(cmin, c[i]);
                cmax = fmax_(cmax, c[i]);
            }
            if (cmin == cmax) continue;
            const float k = kBins / (cmax - cmin);
            Box bins[kBins];
            int counts[kBins] = {0};
            for (int i = lo; i < hi; i++) {
                const int b = std::min(kBins - 1, (int)((c[i] - cmin) * k));
                counts[b]++;
                bins[b].grow(box_[i]);
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
        if (best_cost >= own_cost) return -1;
        // In-place two-pointer partition, swapping material indices along (scene.cu:960-975);
        // the side arrays follow the triangles.
        const float *c = cent_[best_axis].data();
        int i = lo, j = hi - 1;
        while (i <= j) {
            if (c[i] < best_pos) {
                i++;
            } else {
                std::swap(tris_[i], tris_[j]);
                std::swap(mats_[i], mats_[j]);
                std::swap(box_[i], box_[j]);
                for (int a = 0; a < 3; a++) std::swap(cent_[a][i], cent_[a][j]);
                j--;
            }
        }
        if (i == hi || i == lo) return -1;
        return i;
    }

    // The reference's recursion on one array: node ni's children are appended at the end.
    void split(std::vector<rt_bvh_node> &nodes, int ni, int max_depth) {
        rt_bvh_node n = nodes[ni];
        const int mid = decide(n, max_depth);
        nodes[ni] = n;
        if (mid < 0) return;
        const int left = (int)nodes.size();
        nodes.push_back(fresh(n.child2, mid));
        nodes.push_back(fresh(mid, n.child1));
        split(nodes, left, max_depth - 1);
        split(nodes, left + 1, max_depth - 1);
        nodes[ni].child1 = left;
        nodes[ni].child2 = left + 1;
    }

    bool take_thread() {
        int s = spare_threads_.load();
        while (s > 0)
            if (spare_threads_.compare_exchange_weak(s, s - 1)) return true;
        return false;
    }

    // Node `self` (already created by its parent) and, in `desc`, everything the reference
    // appends while splitting it, numbered from 0 (its children are desc[0] and desc[1]).
    void build_desc(rt_bvh_node &self, int max_depth, std::vector<rt_bvh_node> &desc) {
        const int lo = self.child2, hi = self.child1;
        const int mid = decide(self, max_depth);
        if (mid < 0) return;
        rt_bvh_node c1 = fresh(lo, mid), c2 = fresh(mid, hi);
        self.child1 = 0;
        self.child2 = 1;
        if (std::min(mid - lo, hi - mid) < kParallelMin || !take_thread()) {
            desc.push_back(c1);
            desc.push_back(c2);
            split(desc, 0, max_depth - 1);
            split(desc, 1, max_depth - 1);
            return;
        }
        std::vector<rt_bvh_node> d1, d2;
        std::thread other([&] { build_desc(c2, max_depth - 1, d2); });
        build_desc(c1, max_depth - 1, d1);
        other.join();
        spare_threads_++;
        const int b1 = 2, b2 = 2 + (int)d1.size();
        desc.reserve(2 + d1.size() + d2.size());
        desc.push_back(shifted(c1, b1));
        desc.push_back(shifted(c2, b2));
        for (const rt_bvh_node &d : d1) desc.push_back(shifted(d, b1));
        for (const rt_bvh_node &d : d2) desc.push_back(shifted(d, b2));
    }
};

// Threads for the BVH build: RT_BVH_THREADS (1 = single-threaded, as the reference), default
// 16, at most the hardware's.
int bvh_threads() {
    int threads = 16;
    if (const char *e = std::getenv("RT_BVH_THREADS")) threads = std::max(1, std::atoi(e));
    return std::max(1, std::min<int>(threads, (int)std::max(1u, std::thread::hardware_concurrency())));
}

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
    o->bvh_device = -1;
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
    if (opts.bvh_device >= 0) {
        if (int rc = rtamd::gpu_build_bvh(s->triangles, s->material_indices.data() + s->spheres.size(), s->bvh,
                                          opts.use_bvh ? 30 : 0, opts.bvh_device))
            return bad(rc);
    } else {
        BvhBuilder(s->triangles, s->material_indices.data() + s->spheres.size(), s->bvh)
            .build(opts.use_bvh ? 30 : 0, bvh_threads());
    }
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
