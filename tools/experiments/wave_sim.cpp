// Measurement only (not product, not test): a wave-level cost model of trace_kernel's stepping
// policies, driven by the exact per-lane step sequences of the kernel's traversal (the reference's
// far-child-first order, scene.cu:134-241, in the kernel's step structure: root step at refill,
// one node or one triangle per step, pop loop) on bounce-0 and bounce-1-like rays of a scene.
// Used to choose which traversal schedule to build ("Trace lane utilisation"); the
// cost constants are issue slots (VALU + SALU + branch wave-instructions) read from the gfx950 ISA
// of trace_kernel<true,false,0> (see the table in main()).
//
//   g++ -O2 -std=c++17 -Ioracle tools/experiments/wave_sim.cpp -Loracle/build -loracle \
//       -Wl,-rpath,$PWD/oracle/build -o /tmp/wave_sim
//   /tmp/wave_sim assets/teapot.scene assets [stride]
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V mul(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V norm(V a) { float l = std::sqrt(dot(a, a)); return mul(a, 1 / l); }

struct Tri { V p1, e1, e2, n; };
struct Node { V mn, mx; int32_t c1, c2; };
static bool is_leaf(const Node &n) { return n.c2 <= n.c1; }

static bool slab(const Node &b, V o, V inv, float &tmin, float tmax) {
    tmin = 0.0f;
    float t1 = (b.mn.x - o.x) * inv.x, t2 = (b.mx.x - o.x) * inv.x;
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin));
    tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    t1 = (b.mn.y - o.y) * inv.y; t2 = (b.mx.y - o.y) * inv.y;
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin));
    tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    t1 = (b.mn.z - o.z) * inv.z; t2 = (b.mx.z - o.z) * inv.z;
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin));
    tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    return tmin <= tmax;
}

static bool tri(const Tri &tr, V o, V d, float closest, float &t) {
    const V h = cross(d, tr.e2);
    const float a = dot(h, tr.e1);
    if (a == 0) return false;
    const float f = 1 / a;
    const V s = sub(o, tr.p1);
    const float u = dot(s, h) * f;
    if (u < 0 || u > 1) return false;
    const V q = cross(s, tr.e1);
    const float v = dot(d, q) * f;
    if (v < 0 || u + v > 1) return false;
    t = dot(tr.e2, q) * f;
    if ((double)t < 0.005 || t >= closest) return false;
    return true;
}

// One lane's action sequence.  Action: kind 0 = node step, 1 = leaf of c triangles (c triangle
// steps in the kernel); pops = pop-loop iterations after it (0: the lane continues without one).
// The root step (done at refill) is action 0 of every ray.
struct Act { uint8_t kind, c; uint16_t pops; };
struct RayTrace { std::vector<Act> acts; };

struct Scene {
    std::vector<Tri> tris;
    std::vector<Node> bvh;
};

static RayTrace record(const Scene &S, V o, V d, float closest, float *closest_out, int *index_out) {
    RayTrace rt;
    const V inv{1 / d.x, 1 / d.y, 1 / d.z};
    uint32_t st[64];
    float sd[64];
    int sp = 0;
    int index = -1;
    uint32_t ref = 0;
    bool done = false;
    // pop loop: returns the number of iterations; sets ref/leaf or done
    auto pop_loop = [&](int &ti, int &te) -> int {
        int n = 0;
        while (true) {
            n++;
            if (sp == 0) { done = true; return n; }
            sp--;
            if (sd[sp] >= closest) continue;
            ref = st[sp];
            const Node &nd = S.bvh[ref];
            if (is_leaf(nd)) { ti = nd.c2; te = nd.c1; if (ti == te) continue; }
            else { ti = te = 0; }
            return n;
        }
    };
    auto node_step = [&](int &ti, int &te) -> bool {   // returns need
        const Node &nd = S.bvh[ref];
        float t0, t1;
        const bool h0 = slab(S.bvh[nd.c1], o, inv, t0, closest), h1 = slab(S.bvh[nd.c2], o, inv, t1, closest);
        const bool both = h0 && h1, any = h0 || h1;
        const bool sel1 = h1 && (!h0 || t0 < t1);
        const uint32_t next = sel1 ? nd.c2 : nd.c1, nearr = sel1 ? nd.c1 : nd.c2;
        const float next_t = sel1 ? t1 : t0, near_t = sel1 ? t0 : t1;
        if (both) { st[sp] = nearr; sd[sp] = near_t; sp++; }
        if (any && !(next_t >= closest)) {
            ref = next;
            const Node &nn = S.bvh[ref];
            if (is_leaf(nn)) { ti = nn.c2; te = nn.c1; return ti == te; }
            ti = te = 0;
            return false;
        }
        return true;
    };
    int ti = 0, te = 0;
    // root step
    {
        Act a{0, 0, 0};
        if (node_step(ti, te)) a.pops = (uint16_t)pop_loop(ti, te);
        rt.acts.push_back(a);
    }
    while (!done) {
        if (ti < te) {
            Act a{1, (uint8_t)std::min(255, te - ti), 0};
            for (; ti < te; ti++) {
                float t;
                if (tri(S.tris[ti], o, d, closest, t)) { closest = t; index = ti; }
            }
            a.pops = (uint16_t)pop_loop(ti, te);
            rt.acts.push_back(a);
        } else {
            Act a{0, 0, 0};
            if (node_step(ti, te)) a.pops = (uint16_t)pop_loop(ti, te);
            rt.acts.push_back(a);
        }
    }
    *closest_out = closest;
    *index_out = index;
    return rt;
}

// ---------------------------------------------------------------- wave model
struct Cost {
    // issue slots per wave-instruction stream segment (trace_kernel<true,false,0>, gfx950 ISA)
    double head = 10;      // loop head: idle ballot, refill test, active ballot
    double common = 14;    // step: record address select, the record loads, kind branch
    double node = 72;      // child-pair slab test, push, descend (VALU 46 + SALU/branch 26)
    double tri = 76;       // Möller–Trumbore + accept (VALU 61 + SALU/branch 15)
    double pop = 28;       // one pop-loop iteration
    double refill = 90;    // store finished hits, queue atomics, ray loads + setup
    double dist = 34;      // parallel leaf: scan of counts, owner table, o/d exchange through LDS
    double merge = 9;      // parallel leaf: one sequential merge step per owner triangle
    double kindsel = 6;    // while-while: choose the iteration kind
};

struct Result {
    double issue = 0, iters = 0, lane_work = 0, rays = 0;
    double node_lanes = 0, node_iters = 0, tri_lanes = 0, tri_iters = 0;
    double chain = 0;      // sum over rays of the iterations from refill to completion
};

enum Policy { BASE, PLEAF, WW, HY };

// One wave of 64 lanes fed from a ray queue; refill when >= refill_at lanes are idle.
static Result simulate(const std::vector<RayTrace> &rays, Policy pol, int refill_at, int theta, const Cost &C) {
    Result R;
    struct Lane { int ray = -1; size_t a = 0; int left = 0; bool pending = false; long start = 0; };
    Lane L[64];
    size_t next_ray = 0;
    long iter = 0;
    auto finish = [&](Lane &l) { R.chain += (double)(iter - l.start); l.ray = -1; };
    // apply the pops of action a of lane l: the lane moves on to action a+1 (or finishes)
    auto advance = [&](Lane &l) {
        l.a++;
        if (l.a >= rays[l.ray].acts.size()) { finish(l); return; }
        const Act &n = rays[l.ray].acts[l.a];
        l.left = n.kind == 1 ? n.c : 0;
        l.pending = false;
    };
    while (true) {
        int idle = 0;
        for (auto &l : L) idle += l.ray < 0;
        R.issue += C.head;
        if (next_ray < rays.size() && idle >= refill_at) {
            R.issue += C.refill;
            int maxp = 0;
            bool any = false;
            for (auto &l : L)
                if (l.ray < 0 && next_ray < rays.size()) {
                    l.ray = (int)next_ray++;
                    l.a = 0;
                    l.start = iter;
                    R.rays++;
                    const Act &r0 = rays[l.ray].acts[0];
                    any = true;
                    maxp = std::max<int>(maxp, r0.pops);
                    R.lane_work += 1;
                    advance(l);   // the root step is done at refill
                }
            if (any) R.issue += C.node + C.pop * maxp;
        }
        int active = 0;
        for (auto &l : L) active += l.ray >= 0;
        if (!active) {
            if (next_ray >= rays.size()) break;
            continue;
        }
        iter++;
        R.iters++;
        if (pol == BASE) {
            // each active lane does its next step: one triangle of its leaf, or one node
            bool anyn = false, anyt = false;
            int maxp = 0, nn = 0, nt = 0;
            for (auto &l : L) {
                if (l.ray < 0) continue;
                const Act &c = rays[l.ray].acts[l.a];
                if (c.kind == 1) {
                    anyt = true; nt++;
                    if (--l.left == 0) { maxp = std::max<int>(maxp, c.pops); advance(l); }
                } else {
                    anyn = true; nn++;
                    maxp = std::max<int>(maxp, c.pops);
                    advance(l);
                }
            }
            R.issue += C.common + (anyn ? C.node : 0) + (anyt ? C.tri : 0) + C.pop * maxp;
            R.lane_work += nn + nt;
            R.node_lanes += nn; R.node_iters += anyn; R.tri_lanes += nt; R.tri_iters += anyt;
        } else {
            // leaf lanes: their remaining triangles, distributed over the wave's 64 lanes in lane order
            int T = 0, nn = 0;
            for (auto &l : L) {
                if (l.ray < 0) continue;
                const Act &c = rays[l.ray].acts[l.a];
                if (c.kind == 1) T += l.left; else nn++;
            }
            const bool do_leaf = pol == PLEAF ? T > 0 : (T >= theta || (nn == 0 && T > 0));
            const bool do_node = (pol == PLEAF || pol == HY) ? nn > 0 : !do_leaf;
            int maxp = 0, maxm = 0, done_t = 0;
            if (do_leaf) {
                int cap = 64;
                for (auto &l : L) {
                    if (l.ray < 0 || cap == 0) continue;
                    const Act &c = rays[l.ray].acts[l.a];
                    if (c.kind != 1) continue;
                    const int k = std::min(cap, l.left);
                    cap -= k; l.left -= k; done_t += k;
                    maxm = std::max(maxm, k);
                    if (l.left == 0) l.pending = true;   // pops after this iteration's merge
                }
                R.issue += C.dist + C.tri + C.merge * maxm;
                R.tri_lanes += done_t; R.tri_iters += 1;
            }
            if (do_node) {
                for (auto &l : L) {
                    if (l.ray < 0) continue;
                    const Act &c = rays[l.ray].acts[l.a];
                    if (c.kind != 0) continue;
                    maxp = std::max<int>(maxp, c.pops);
                    l.pending = true;
                }
                R.issue += C.common + C.node;
                R.node_lanes += nn; R.node_iters += 1;
            }
            for (auto &l : L) {
                if (l.ray < 0 || !l.pending) continue;
                const Act &c = rays[l.ray].acts[l.a];
                maxp = std::max<int>(maxp, c.pops);
                advance(l);
            }
            R.issue += C.pop * maxp + (pol == WW ? C.kindsel : 0);
            R.lane_work += (do_node ? nn : 0) + done_t;
        }
    }
    return R;
}

int main(int argc, char **argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s scene asset_root [stride]\n", argv[0]); return 2; }
    const int stride = argc > 3 ? std::atoi(argv[3]) : 8;
    orc_scene *s = orc_load_scene(argv[1], 1, argv[2], nullptr, nullptr);
    if (!s) { std::fprintf(stderr, "%s\n", orc_last_error()); return 1; }
    orc_info info;
    orc_get_info(s, &info);
    Scene S;
    std::vector<float> sph(4 * (size_t)info.sphere_count + 4);
    S.tris.resize(info.triangle_count);
    S.bvh.resize(info.bvh_node_count);
    std::vector<float> cam(orc_camera_floats());
    orc_get_arrays(s, sph.data(), S.tris.data(), nullptr, nullptr, S.bvh.data(), nullptr, cam.data());
    if (info.sphere_count) std::printf("note: sphere loop not modelled (%d spheres)\n", info.sphere_count);
    const V pos{cam[0], cam[1], cam[2]};
    const V sr{cam[16], cam[17], cam[18]}, su{cam[19], cam[20], cam[21]}, tl{cam[22], cam[23], cam[24]};
    const float inv_w = cam[25], inv_h = cam[26];
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::vector<RayTrace> rays[2];
    // rays in pixel order (bounce 0) and, for the bounce-1 set, shuffled (the reorder's 6-bit key
    // scatters neighbouring pixels' secondary rays over 64 buckets)
    for (int y = 0; y < info.height; y += 1)
        for (int x = (y * 3) % stride; x < info.width; x += stride) {
            V o = pos;
            V d = norm(sub(add(tl, mul(sr, (x + U(rng)) * inv_w)), mul(su, (y + U(rng)) * inv_h)));
            float t;
            int idx;
            rays[0].push_back(record(S, o, d, 1e30f, &t, &idx));
            if (idx < 0) continue;
            const Tri &T = S.tris[idx];
            V n = norm(T.n);
            if (dot(n, d) > 0) n = mul(n, -1);
            const V hit = add(o, mul(d, t));
            const V a = std::fabs(n.x) > 0.5f ? V{0, 1, 0} : V{1, 0, 0};
            const V t1 = norm(cross(a, n)), t2 = cross(n, t1);
            const float r1 = 2 * 3.14159265f * U(rng), r2 = U(rng), sq = std::sqrt(r2);
            d = norm(add(add(mul(t1, std::cos(r1) * sq), mul(t2, std::sin(r1) * sq)), mul(n, std::sqrt(1 - r2))));
            rays[1].push_back(record(S, hit, d, 1e30f, &t, &idx));
        }
    std::shuffle(rays[1].begin(), rays[1].end(), rng);
    Cost C;
    if (argc > 4) C.dist = std::atof(argv[4]);
    if (argc > 5) C.merge = std::atof(argv[5]);
    for (int b = 1; b < 2; b++) {
        double acts = 0, tris = 0, leaves = 0;
        for (auto &r : rays[b])
            for (auto &a : r.acts) { acts++; if (a.kind) { tris += a.c; leaves++; } }
        std::printf("bounce %d: %zu rays, %.2f node steps, %.2f leaves, %.2f triangles per ray (%.2f per leaf)\n", b,
                    rays[b].size(), (acts - leaves) / rays[b].size(), leaves / rays[b].size(), tris / rays[b].size(),
                    tris / std::max(1.0, leaves));
        struct Cfg { const char *name; Policy p; int refill, theta; };
        const Cfg cfgs[] = {{"base r24", BASE, 24, 0},  {"base r64", BASE, 64, 0},  {"pleaf r24", PLEAF, 24, 0},
                            {"ww t16 r24", WW, 24, 16}, {"ww t32 r24", WW, 24, 32}, {"ww t48 r24", WW, 24, 48},
                            {"ww t64 r24", WW, 24, 64}, {"ww t32 r16", WW, 16, 32}, {"ww t48 r16", WW, 16, 48},
                            {"ww t48 r8", WW, 8, 48},   {"hy t32 r24", HY, 24, 32}, {"hy t48 r24", HY, 24, 48},
                            {"hy t48 r16", HY, 16, 48}};
        double base_issue = 0;
        for (const Cfg &c : cfgs) {
            const Result R = simulate(rays[b], c.p, b == 0 && c.p == BASE && c.refill == 24 ? 64 : c.refill, c.theta, C);
            if (base_issue == 0) base_issue = R.issue;
            std::printf("  %-12s issue/ray %7.1f (x%.3f)  iters/ray %6.2f  chain/ray %6.2f  lanes/iter %5.1f  "
                        "node lanes/iter %5.1f  tri lanes/iter %5.1f  node iters %.2f tri iters %.2f per iter\n",
                        c.name, R.issue / R.rays, R.issue / base_issue, R.iters * 64 / R.rays, R.chain / R.rays,
                        R.lane_work / R.iters, R.node_lanes / std::max(1.0, R.node_iters),
                        R.tri_lanes / std::max(1.0, R.tri_iters), R.node_iters / R.iters, R.tri_iters / R.iters);
        }
    }
    orc_free_scene(s);
    return 0;
}
