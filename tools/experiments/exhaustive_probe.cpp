// Measurement only (not product, not test): how much traversal work an order-free closest-hit
// search would do next to the reference's far-first traversal (scene.cu:134-241), and how often its
// answer could differ from the reference's.
//
// An order-free search tests every triangle of every leaf whose whole root path the ray's slab tests
// accept (no culling by the running closest, only by the sphere/initial closest), so its work does
// not depend on visit order.  Its minimum t* equals the reference's answer whenever the winning
// triangle's path entry distances are all below t* (the reference cannot have culled it: its
// running closest never drops below t*) and no other triangle ties t*; otherwise a ray would have
// to be re-traced in the reference order.  This probe counts both, per bounce-0 / bounce-1 ray.
//
//   g++ -O2 -std=c++17 -Ioracle tools/experiments/exhaustive_probe.cpp -Loracle/build -loracle \
//       -Wl,-rpath,$PWD/oracle/build -o /tmp/exhaustive_probe
//   /tmp/exhaustive_probe assets/teapot/teapot.scene assets/teapot [stride]
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
static bool leaf(const Node &n) { return n.c2 <= n.c1; }

static float fmin_(float a, float b) { return std::fmin(a, b); }
static float fmax_(float a, float b) { return std::fmax(a, b); }

static bool slab(const Node &b, V o, V inv, float &tmin, float tmax) {
    tmin = 0.0f;
    float t1 = (b.mn.x - o.x) * inv.x, t2 = (b.mx.x - o.x) * inv.x;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    t1 = (b.mn.y - o.y) * inv.y; t2 = (b.mx.y - o.y) * inv.y;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    t1 = (b.mn.z - o.z) * inv.z; t2 = (b.mx.z - o.z) * inv.z;
    tmin = fmin_(fmax_(t1, tmin), fmax_(t2, tmin));
    tmax = fmax_(fmin_(t1, tmax), fmin_(t2, tmax));
    return tmin <= tmax;
}

// Möller–Trumbore with the reference's rejects; `closest` as given.
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

struct Work { uint64_t iv = 0, tt = 0; };

static void reference(const std::vector<Node> &bvh, const std::vector<Tri> &tris, int sph, V o, V d, float &closest,
                      int &index, Work &w) {
    const V inv{1 / d.x, 1 / d.y, 1 / d.z};
    uint32_t is[64]; float ds[64]; int sc = 1; is[0] = 0; ds[0] = 0;
    while (sc) {
        sc--;
        if (ds[sc] >= closest) continue;
        const Node &n = bvh[is[sc]];
        if (leaf(n)) {
            for (int i = n.c2; i < n.c1; i++) {
                w.tt++;
                float t;
                if (tri(tris[i], o, d, closest, t)) { closest = t; index = sph + i; }
            }
        } else {
            w.iv++;
            float d1, d2;
            const bool h1 = slab(bvh[n.c1], o, inv, d1, closest), h2 = slab(bvh[n.c2], o, inv, d2, closest);
            if (h1 && h2) {
                if (d1 < d2) { is[sc] = n.c1; ds[sc++] = d1; is[sc] = n.c2; ds[sc++] = d2; }
                else { is[sc] = n.c2; ds[sc++] = d2; is[sc] = n.c1; ds[sc++] = d1; }
            } else if (h1) { is[sc] = n.c1; ds[sc++] = d1; }
            else if (h2) { is[sc] = n.c2; ds[sc++] = d2; }
        }
    }
}

// Order-free: every statically hit subtree (culled only by the initial closest c0).  Returns the
// minimum t*, its index, and whether the reference is guaranteed to return the same (path entry
// distances of the winner all < t*, no tie at t*).
static bool exhaustive(const std::vector<Node> &bvh, const std::vector<Tri> &tris, int sph, V o, V d, float c0,
                       float &best, int &index, Work &w, bool &tie) {
    const V inv{1 / d.x, 1 / d.y, 1 / d.z};
    uint32_t is[64]; float pm[64]; int sc = 1; is[0] = 0; pm[0] = 0;
    float win_pm = 0, second = c0;
    tie = false;
    best = c0;
    while (sc) {
        sc--;
        const Node &n = bvh[is[sc]];
        const float pmax = pm[sc];
        if (pmax >= c0) continue;       // the reference culls it whatever it finds (closest <= c0)
        if (leaf(n)) {
            for (int i = n.c2; i < n.c1; i++) {
                w.tt++;
                float t;
                if (tri(tris[i], o, d, c0, t)) {
                    if (t < best) { second = best; best = t; index = sph + i; win_pm = pmax; tie = false; }
                    else if (t == best) tie = true;
                    else second = std::min(second, t);
                }
            }
        } else {
            w.iv++;
            float d1, d2;
            const bool h1 = slab(bvh[n.c1], o, inv, d1, c0), h2 = slab(bvh[n.c2], o, inv, d2, c0);
            if (h1) { is[sc] = n.c1; pm[sc++] = std::max(pmax, d1); }
            if (h2) { is[sc] = n.c2; pm[sc++] = std::max(pmax, d2); }
        }
    }
    // the reference's running closest stays >= min(second, c0) until the winner is found, and every
    // path node of the winner has entry < that: it is neither culled at a slab test nor at a pop
    return best == c0 || (!tie && (win_pm < best || win_pm < second));
}

int main(int argc, char **argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s scene asset_root [stride]\n", argv[0]); return 2; }
    const int stride = argc > 3 ? std::atoi(argv[3]) : 16;
    orc_scene *s = orc_load_scene(argv[1], 1, argv[2], nullptr, nullptr);
    if (!s) { std::fprintf(stderr, "%s\n", orc_last_error()); return 1; }
    orc_info info;
    orc_get_info(s, &info);
    std::vector<float> sph(4 * (size_t)info.sphere_count + 4);
    std::vector<Tri> tris(info.triangle_count);
    std::vector<Node> bvh(info.bvh_node_count);
    std::vector<float> cam(orc_camera_floats());
    orc_get_arrays(s, sph.data(), tris.data(), nullptr, nullptr, bvh.data(), nullptr, cam.data());
    // camera block: pos(3) fwd(3) up(3) fov(1) min(3) inv_dim(3) sr(3) su(3) tl(3) inv_w inv_h
    const V pos{cam[0], cam[1], cam[2]};
    const V sr{cam[16], cam[17], cam[18]}, su{cam[19], cam[20], cam[21]}, tl{cam[22], cam[23], cam[24]};
    const float inv_w = cam[25], inv_h = cam[26];
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    Work wr[2], we[2];
    uint64_t rays[2] = {0, 0}, unsafe[2] = {0, 0}, ties[2] = {0, 0}, differ[2] = {0, 0};
    uint64_t max_ref[2] = {0, 0}, max_free[2] = {0, 0}, max_ratio_steps[2][2] = {{0, 0}, {0, 0}};
    double max_ratio[2] = {0, 0};
    for (int y = 0; y < info.height; y++)
        for (int x = (y * 7) % stride; x < info.width; x += stride) {
            V o = pos;
            V d = norm(sub(add(tl, mul(sr, (x + U(rng)) * inv_w)), mul(su, (y + U(rng)) * inv_h)));
            for (int b = 0; b < 2; b++) {
                float c0 = 1e30f;
                int i0 = -1;
                for (int k = 0; k < info.sphere_count; k++) {
                    const V c{sph[4 * k], sph[4 * k + 1], sph[4 * k + 2]};
                    const float r = sph[4 * k + 3];
                    const V off = sub(c, o);
                    const float mhb = dot(off, d), qd = mhb * mhb - (dot(off, off) - r * r);
                    if (qd < 0) continue;
                    const float hs = std::sqrt(qd);
                    float t = mhb - hs;
                    if (!(t < c0 && t >= 0.005f)) t = mhb + hs;
                    if (t < c0 && t >= 0.005f) { c0 = t; i0 = k; }
                }
                float cr = c0, ce;
                int ir = i0, ie = i0;
                bool tie;
                const Work r0 = wr[b], e0 = we[b];
                reference(bvh, tris, info.sphere_count, o, d, cr, ir, wr[b]);
                const bool safe = exhaustive(bvh, tris, info.sphere_count, o, d, c0, ce, ie, we[b], tie);
                const uint64_t sr = wr[b].iv + wr[b].tt - r0.iv - r0.tt, se = we[b].iv + we[b].tt - e0.iv - e0.tt;
                max_ref[b] = std::max(max_ref[b], sr);
                max_free[b] = std::max(max_free[b], se);
                if ((double)se / std::max<uint64_t>(sr, 1) > max_ratio[b]) {
                    max_ratio[b] = (double)se / std::max<uint64_t>(sr, 1);
                    max_ratio_steps[b][0] = sr; max_ratio_steps[b][1] = se;
                }
                rays[b]++;
                if (!safe) unsafe[b]++;
                if (tie) ties[b]++;
                if (safe && (ce != cr || ie != ir)) differ[b]++;
                if (ir < info.sphere_count) break;   // miss or sphere: no secondary ray from here
                // secondary: cosine-weighted about the triangle normal (approximates a diffuse bounce)
                const Tri &T = tris[ir - info.sphere_count];
                V n = norm(T.n);
                if (dot(n, d) > 0) n = mul(n, -1);
                const V hit = add(o, mul(d, cr));
                const V a = std::fabs(n.x) > 0.5f ? V{0, 1, 0} : V{1, 0, 0};
                const V t1 = norm(cross(a, n)), t2 = cross(n, t1);
                const float r1 = 2 * 3.14159265f * U(rng), r2 = U(rng), sq = std::sqrt(r2);
                d = norm(add(add(mul(t1, std::cos(r1) * sq), mul(t2, std::sin(r1) * sq)), mul(n, std::sqrt(1 - r2))));
                o = hit;
            }
        }
    for (int b = 0; b < 2; b++) {
        const double n = (double)std::max<uint64_t>(1, rays[b]);
        std::printf("bounce %d: rays %llu  reference iv %.1f tt %.1f steps %.1f | order-free iv %.1f tt %.1f steps %.1f "
                    "(x%.3f) | re-trace needed %.5f (ties %.5f) | safe but different %llu\n",
                    b, (unsigned long long)rays[b], wr[b].iv / n, wr[b].tt / n, (wr[b].iv + wr[b].tt) / n, we[b].iv / n,
                    we[b].tt / n, (we[b].iv + we[b].tt) / n, (double)(we[b].iv + we[b].tt) / std::max<uint64_t>(1, wr[b].iv + wr[b].tt),
                    unsafe[b] / n, ties[b] / n, (unsigned long long)differ[b]);
        std::printf("   longest ray: reference %llu steps, order-free %llu; worst ratio %.1f (%llu -> %llu)\n",
                    (unsigned long long)max_ref[b], (unsigned long long)max_free[b], max_ratio[b],
                    (unsigned long long)max_ratio_steps[b][0], (unsigned long long)max_ratio_steps[b][1]);
    }
    orc_free_scene(s);
    return 0;
}
