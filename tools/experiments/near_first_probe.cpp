// Measurement only (not product, not test): traversal steps of the reference's far-child-first
// order (scene.cu:196-225: both hit children pushed near then far, the far one popped first)
// against near-child-first, on camera rays and two diffuse bounces, and how often their closest-hit
// answers differ.  Round 4: teapot x0.52 / 0.71 / 0.75 steps at bounces 0 / 1 / 2,
// no differing answer among the probed rays -- but no per-ray test can prove equality, so the
// render keeps the reference order.
//
//   g++ -O2 -std=c++17 -Ioracle tools/experiments/near_first_probe.cpp -Loracle/build -loracle \
//       -Wl,-rpath,$PWD/oracle/build -o /tmp/nf && /tmp/nf assets/teapot/teapot.scene assets/teapot 8
#include "oracle.h"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin)); tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    t1 = (b.mn.y - o.y) * inv.y; t2 = (b.mx.y - o.y) * inv.y;
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin)); tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    t1 = (b.mn.z - o.z) * inv.z; t2 = (b.mx.z - o.z) * inv.z;
    tmin = std::fmin(std::fmax(t1, tmin), std::fmax(t2, tmin)); tmax = std::fmax(std::fmin(t1, tmax), std::fmin(t2, tmax));
    return tmin <= tmax;
}
static bool tri(const Tri &tr, V o, V d, float closest, float &t) {
    const V h = cross(d, tr.e2); const float a = dot(h, tr.e1); if (a == 0) return false;
    const float f = 1 / a; const V s = sub(o, tr.p1); const float u = dot(s, h) * f; if (u < 0 || u > 1) return false;
    const V q = cross(s, tr.e1); const float v = dot(d, q) * f; if (v < 0 || u + v > 1) return false;
    t = dot(tr.e2, q) * f; if ((double)t < 0.005 || t >= closest) return false; return true;
}
static int trav(const std::vector<Node> &bvh, const std::vector<Tri> &tris, V o, V d, float &closest, int &index, bool near_first) {
    const V inv{1 / d.x, 1 / d.y, 1 / d.z};
    uint32_t is[64]; float ds[64]; int sc = 1; is[0] = 0; ds[0] = 0; int steps = 0;
    while (sc) {
        sc--;
        if (ds[sc] >= closest) continue;
        const Node &n = bvh[is[sc]];
        if (is_leaf(n)) {
            for (int i = n.c2; i < n.c1; i++) { steps++; float t; if (tri(tris[i], o, d, closest, t)) { closest = t; index = i; } }
        } else {
            steps++;
            float d1, d2;
            const bool h1 = slab(bvh[n.c1], o, inv, d1, closest), h2 = slab(bvh[n.c2], o, inv, d2, closest);
            if (h1 && h2) {
                bool c1_near = d1 < d2;      // reference: push near then far (far popped first)
                uint32_t nr = c1_near ? n.c1 : n.c2, fr = c1_near ? n.c2 : n.c1; float dn = c1_near ? d1 : d2, df = c1_near ? d2 : d1;
                if (!near_first) { is[sc] = nr; ds[sc++] = dn; is[sc] = fr; ds[sc++] = df; }
                else { is[sc] = fr; ds[sc++] = df; is[sc] = nr; ds[sc++] = dn; }
            } else if (h1) { is[sc] = n.c1; ds[sc++] = d1; }
            else if (h2) { is[sc] = n.c2; ds[sc++] = d2; }
        }
    }
    return steps;
}
int main(int argc, char **argv) {
    const int stride = argc > 3 ? std::atoi(argv[3]) : 8;
    orc_scene *s = orc_load_scene(argv[1], 1, argv[2], nullptr, nullptr);
    orc_info info; orc_get_info(s, &info);
    std::vector<float> sph(4 * (size_t)info.sphere_count + 4);
    std::vector<Tri> tris(info.triangle_count); std::vector<Node> bvh(info.bvh_node_count);
    std::vector<float> cam(orc_camera_floats());
    orc_get_arrays(s, sph.data(), tris.data(), nullptr, nullptr, bvh.data(), nullptr, cam.data());
    const V pos{cam[0], cam[1], cam[2]};
    const V sr{cam[16], cam[17], cam[18]}, su{cam[19], cam[20], cam[21]}, tl{cam[22], cam[23], cam[24]};
    const float inv_w = cam[25], inv_h = cam[26];
    std::mt19937 rng(1234); std::uniform_real_distribution<float> U(0.f, 1.f);
    long long rays[3] = {0}, sr_[3] = {0}, sn[3] = {0}, diff[3] = {0}, difft[3] = {0};
    for (int y = 0; y < info.height; y++)
        for (int x = (y * 3) % stride; x < info.width; x += stride) {
            V o = pos; V d = norm(sub(add(tl, mul(sr, (x + U(rng)) * inv_w)), mul(su, (y + U(rng)) * inv_h)));
            for (int b = 0; b < 3; b++) {
                float c1 = 1e30f, c2 = 1e30f; int i1 = -1, i2 = -1;
                sr_[b] += trav(bvh, tris, o, d, c1, i1, false);
                sn[b] += trav(bvh, tris, o, d, c2, i2, true);
                rays[b]++;
                if (i1 != i2) diff[b]++;
                if (c1 != c2) difft[b]++;
                if (i1 < 0) break;
                const Tri &T = tris[i1]; V n = norm(T.n); if (dot(n, d) > 0) n = mul(n, -1);
                const V hit = add(o, mul(d, c1));
                const V a = std::fabs(n.x) > 0.5f ? V{0, 1, 0} : V{1, 0, 0};
                const V t1 = norm(cross(a, n)), t2 = cross(n, t1);
                const float r1 = 2 * 3.14159265f * U(rng), r2 = U(rng), sq = std::sqrt(r2);
                d = norm(add(add(mul(t1, std::cos(r1) * sq), mul(t2, std::sin(r1) * sq)), mul(n, std::sqrt(1 - r2))));
                o = hit;
            }
        }
    for (int b = 0; b < 3; b++)
        std::printf("bounce %d: %lld rays, far-first %.2f steps, near-first %.2f steps (x%.3f), index differs %lld, t differs %lld\n",
                    b, rays[b], (double)sr_[b] / rays[b], (double)sn[b] / rays[b], (double)sn[b] / sr_[b], diff[b], difft[b]);
}
