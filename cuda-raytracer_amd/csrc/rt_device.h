// rt_device.h — device-side arithmetic for the gfx950 path tracer.
//
// Bit-exact contract with the reference semantics (restated independently in oracle/):
//   * compiled with -ffp-contract=off (and the pragma below): no FMA contraction;
//   * IEEE fp32 division/sqrt (HIP's default correctly-rounded forms), no FTZ;
//   * fminf/fmaxf = v_min_f32/v_max_f32 (NaN-ignoring; only the sign of a zero tie can
//     differ from glibc and it never reaches a comparison result);
//   * cosf/sinf/atanf -> rt_sincos/rt_atan01 (deterministic float kernels);
//   * double where the reference evaluates in double.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

// Functions below are shared by the gfx950 kernels and the host `cpu` path (cpu_render.hip).
#define RT_HD __host__ __device__ __forceinline__

namespace rtd {

struct V3 { float x, y, z; };

RT_HD V3 v3(float x, float y, float z) { return {x, y, z}; }
RT_HD V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD V3 operator*(float s, V3 v) { return {s * v.x, s * v.y, s * v.z}; }
RT_HD V3 operator-(V3 v) { return {-v.x, -v.y, -v.z}; }
// math.cuh:67-114 — left-to-right sums, reciprocal-then-multiply normalise.
RT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
RT_HD float magsq(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
RT_HD V3 normalise(V3 v) { return (1.0f / sqrtf(magsq(v))) * v; }
RT_HD float clamp01(float x) { return fmaxf(fminf(x, 1.0f), 0.0f); }
RT_HD bool is_black(V3 v) { return v.x == 0 && v.y == 0 && v.z == 0; }

// (double)t < 0.005  <=>  t < 0x1.47ae16p-8f  (scene.cu:190, 357, 366).
constexpr float kEps = 0x1.47ae16p-8f;

// Deterministic sin/cos for x >= 0 (random_on_sphere, random.cuh:63-75): Cody-Waite
// reduction by pi/2 and cephes minimax polynomials, fixed evaluation order.
RT_HD void rt_sincos(float x, float &s, float &c) {
    const float fj = x * 0.636619772f;
    const int j = (int)(fj + 0.5f);
    const float jf = (float)j;
    const float r = ((x - jf * 1.5703125f) - jf * 4.837512969970703125e-4f) - jf * 7.54978995489188216e-8f;
    const float z = r * r;
    const float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    const float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
                     - 0.5f * z + 1.0f;
    const int q = j & 3;
    const float a = (q & 1) ? cp : sp;
    const float b = (q & 1) ? sp : cp;
    s = (q & 2) ? -a : a;
    c = ((q + 1) & 2) ? -b : b;
}

// atanf on [0, 1] (equal_area_project_sphere_to_square, scene.cu:297).
RT_HD float rt_atan01(float x) {
    float y = 0.0f;
    if (x > 0.4142135623730950f) { y = 0.78539816339744830962f; x = (x - 1.0f) / (x + 1.0f); }
    const float z = x * x;
    return y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
                 - 3.33329491539e-1f) * z * x + x);
}

// PCG-XSH-RR (random.cuh:13-45).
struct Rng { uint64_t state, inc; };
RT_HD uint32_t pcg(Rng &r) {
    const uint64_t old = r.state;
    r.state = old * 6364136223846793005ULL + (r.inc | 1);
    const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    const uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((0u - rot) & 31));
}
RT_HD Rng pcg_seed(uint32_t seed) {
    Rng r;
    r.state = (uint64_t)seed * 6839056345687307ULL;
    r.inc = 820957824423429ULL;
    pcg(r);
    return r;
}
RT_HD float random01(Rng &r) { return (float)pcg(r) * 0x1p-32f; }
RT_HD float random02(Rng &r) { return (float)pcg(r) * 0x1p-31f; }
RT_HD float random_radians(Rng &r) {
    return (float)((double)pcg(r) * (3.14159265358979323846 * 2 / 4294967295.0));
}
RT_HD V3 random_on_sphere(Rng &r) {
    const float r1 = random_radians(r);
    const float r2 = random02(r);
    const float x = sqrtf(r2 * (2 - r2));
    float s, c;
    rt_sincos(r1, s, c);
    return {c * x, s * x, 1 - r2};
}

// Reorder bucket of a live ray: the 6 bits the reference's 32-bit key actually carries
// (interleave_5(x) == (x & 1) * 0x41, scene.cu:44-60), in key order: oz oy ox dz dy dx.
// 64 = terminated (key 0xFFFFFFFF) sorts last.
RT_HD uint32_t quant_bit(float v) {
    const double q = (double)v * 31.99;
    if (!(q > 0.0)) return 0;                 // NaN / <= 0 saturate to 0 (PTX cvt)
    if (q >= 65535.0) return 1;               // 65535 is odd
    return (uint32_t)q & 1u;
}
RT_HD uint32_t bucket_of(V3 o, V3 d, V3 min_coord, V3 inv_dim) {
    const V3 a = (o - min_coord) * inv_dim;
    const V3 b = 0.5f * (d + v3(1, 1, 1));
    return (quant_bit(a.z) << 5) | (quant_bit(a.y) << 4) | (quant_bit(a.x) << 3) |
           (quant_bit(b.z) << 2) | (quant_bit(b.y) << 1) | quant_bit(b.x);
}

// ray_aabb_intersection, scene.cu:109-132 (branchless slab, fminf/fmaxf).
RT_HD bool slab(float lx, float ly, float lz, float hx, float hy, float hz, V3 o, float ix, float iy, float iz,
                float tmax, float &tmin) {
    tmin = 0.0f;
    float t1 = (lx - o.x) * ix, t2 = (hx - o.x) * ix;
    tmin = fminf(fmaxf(t1, tmin), fmaxf(t2, tmin));
    tmax = fmaxf(fminf(t1, tmax), fminf(t2, tmax));
    t1 = (ly - o.y) * iy; t2 = (hy - o.y) * iy;
    tmin = fminf(fmaxf(t1, tmin), fmaxf(t2, tmin));
    tmax = fmaxf(fminf(t1, tmax), fminf(t2, tmax));
    t1 = (lz - o.z) * iz; t2 = (hz - o.z) * iz;
    tmin = fminf(fmaxf(t1, tmin), fmaxf(t2, tmin));
    tmax = fmaxf(fminf(t1, tmax), fminf(t2, tmax));
    return tmin <= tmax;
}

// Möller–Trumbore body, scene.cu:166-191: accepted hit distance in t, else false.
RT_HD bool ray_triangle(V3 o, V3 d, V3 p1, V3 e1, V3 e2, float closest, float &t) {
    const V3 h = cross(d, e2);
    const float a = dot(h, e1);
    if (a == 0) return false;
    const float f = 1 / a;
    const V3 s = o - p1;
    const float u = dot(s, h) * f;
    if (u < 0 || u > 1) return false;
    const V3 q = cross(s, e1);
    const float v = dot(d, q) * f;
    if (v < 0 || u + v > 1) return false;
    t = dot(e2, q) * f;
    return !(t < kEps || t >= closest);
}

// Sphere body, scene.cu:340-371 (assumes |d| = 1 like the reference).
RT_HD bool ray_sphere(V3 o, V3 d, V3 c, float radius, float closest, float &t) {
    const V3 off = c - o;
    const float mhb = dot(off, d);
    const float qc = magsq(off) - radius * radius;
    const float qd = mhb * mhb - qc;
    if (qd < 0) return false;
    const float hs = sqrtf(qd);
    t = mhb - hs;
    if (t < closest && !(t < kEps)) return true;
    t = mhb + hs;
    return t < closest && !(t < kEps);
}

// Environment lookup for a ray that hit nothing: rotation (scene.cu:380-382, in double),
// equal-area square projection (scene.cu:284-318), nearest texel with the reference's
// row stride of env_h (scene.cu:389-391).
RT_HD V3 sky_color(const float *env, int env_w, int env_h, V3 dir) {
    const float dx = (float)((double)dir.x * -0.386527 + (double)dir.z * 0.922278);
    const float dy = (float)((double)dir.x * -0.922278 + (double)dir.z * -0.386527);
    const float dz = dir.y;
    const float x = fabsf(dx), y = fabsf(dy), z = fabsf(dz);
    const float r = sqrtf(1 - fminf(z, 1.0f));
    const float a = fmaxf(x, y);
    float b = fminf(x, y);
    b = a == 0 ? 0 : b / a;
    float phi = (float)((2 / 3.14159265358979323846) * (double)rt_atan01(b));
    if (x < y) phi = 1 - phi;
    float v = phi * r;
    float u = r - v;
    if (dz < 0) {
        const float old_v = v;
        v = 1 - u;
        u = 1 - old_v;
    }
    u = copysignf(u, dx);
    v = copysignf(v, dy);
    const float cu = (u + 1) * 0.5f, cv = (v + 1) * 0.5f;
    const int tx = (int)((double)(clamp01(cu) * (env_w - 1)) + 0.5);
    const int ty = (int)((double)(clamp01(cv) * (env_h - 1)) + 0.5);
    const float *e = env + (size_t)(ty * env_h + tx) * 3;
    return v3(e[0], e[1], e[2]);
}

struct Mat { V3 diffuse; float metal; V3 spec; float rough; V3 emit; float ior; };

RT_HD Mat load_mat(const float4 *m) {
    const float4 a = m[0], b = m[1], c = m[2];
    return {v3(a.x, a.y, a.z), a.w, v3(b.x, b.y, b.z), b.w, v3(c.x, c.y, c.z), c.w};
}

// Surface interaction after the closest hit (scene.cu:398-477): emission, rough normal,
// specular / diffuse / dielectric scatter.  RNG draw order is part of the contract.
RT_HD void scatter(V3 d, V3 normal, const Mat &m, Rng &rng, V3 &T, V3 &C, V3 &nd) {
    C = C + m.emit * T;
    const bool front = dot(normal, d) < 0;
    if (!front) normal = -normal;
    const V3 rough = normalise(normal + m.rough * random_on_sphere(rng));
    const float cos_theta = dot(rough, d);
    if (m.ior == 0) {
        if (random01(rng) <= m.metal) {
            T = T * m.spec;
            nd = d - (2 * cos_theta) * rough;
        } else {
            T = T * m.diffuse;
            nd = normalise(normal + random_on_sphere(rng));
        }
    } else {
        float ior = m.ior;
        float inv_ior = 1 / ior;
        if (front) { const float tmp = inv_ior; inv_ior = ior; ior = tmp; }
        const float sin2 = 1 - cos_theta * cos_theta;
        float r0 = (1 - ior) / (1 + ior);
        r0 *= r0;
        const float cs = 1 + cos_theta;
        const float refl = r0 + (1 - r0) * cs * cs * cs * cs * cs;
        if (sin2 > inv_ior * inv_ior || random01(rng) < refl) {
            T = T * m.spec;
            nd = d - (2 * cos_theta) * rough;
        } else {
            T = T * m.diffuse;
            const V3 perp = ior * (d - cos_theta * rough);
            const V3 par = (-sqrtf(1 - magsq(perp))) * rough;
            nd = normalise(par + perp);
        }
    }
}

}  // namespace rtd
