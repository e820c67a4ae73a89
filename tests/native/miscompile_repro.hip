// miscompile_repro.hip — TEST INFRASTRUCTURE: standalone check of the gfx950 code-generation
// problem worked around in shade_one (csrc/rt_render.hip, bounce-0 branch): with the ray's
// throughput T a compile-time constant (1, 1, 1), ROCm 7.2 clang dropped T.xy on the
// dielectric-reflect path of scatter() (scene.cu:443-476) inside the shade kernel; T.z was right.
// The product launders T through an empty asm so it is opaque, which gives bounce 0 the same
// code shape as later bounces.
//
// Two kernels run scatter() on the same rays (unit directions, random normals, a dielectric and a
// metal material, fixed seeds), one with T = (1, 1, 1) folded in (CONSTANT) and one laundered
// (LAUNDERED, the product's form); the host computes the same function from the same source.
// Prints one JSON line: how many rays each kernel got wrong, and how many took the dielectric
// reflect path.  The laundered kernel must match bit for bit; the constant one documents whether
// this standalone shape reproduces the problem (it may not: it was register-allocation dependent).
//   miscompile_repro [n]
#include "rt_device.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace rtd;

struct Out { float tx, ty, tz, cx, cy, cz, nx, ny, nz, path; };

// path: 0 opaque, 1 dielectric reflect (TIR or Schlick), 2 dielectric refract
__host__ __device__ inline int reflect_path(V3 d, V3 normal, const Mat &m, Rng rng) {
    if (m.ior == 0) return 0;
    const bool front = dot(normal, d) < 0;
    if (!front) normal = -normal;
    const V3 rough = normalise(normal + m.rough * random_on_sphere(rng));
    const float c = dot(rough, d);
    float ior = m.ior, inv = 1 / ior;
    if (front) { const float t = inv; inv = ior; ior = t; }
    float r0 = (1 - ior) / (1 + ior);
    r0 *= r0;
    const float cs = 1 + c;
    return (1 - c * c > inv * inv || random01(rng) < r0 + (1 - r0) * cs * cs * cs * cs * cs) ? 1 : 2;
}

template <bool LAUNDER>
__global__ void scatter_kernel(const float *dirs, const float *normals, const Mat *mats, int n, Out *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const V3 d = v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
    const V3 nrm = v3(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
    const Mat m = mats[i & 1];
    Rng rng = pcg_seed((uint32_t)i * 4137874753u + 279220567u);
    float tx = 1.f, ty = 1.f, tz = 1.f;
    if (LAUNDER) asm volatile("" : "+v"(tx), "+v"(ty), "+v"(tz));
    V3 T = v3(tx, ty, tz), C = v3(0, 0, 0), nd = d;
    const int path = reflect_path(d, nrm, m, rng);
    scatter(d, nrm, m, rng, T, C, nd);
    out[i] = Out{T.x, T.y, T.z, C.x, C.y, C.z, nd.x, nd.y, nd.z, (float)path};
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 1 << 16;
    std::vector<float> dirs(3 * n), normals(3 * n);
    Rng g = pcg_seed(12345u);
    for (int i = 0; i < n; i++) {
        const V3 d = random_on_sphere(g), nr = random_on_sphere(g);
        dirs[3 * i] = d.x; dirs[3 * i + 1] = d.y; dirs[3 * i + 2] = d.z;
        normals[3 * i] = nr.x; normals[3 * i + 1] = nr.y; normals[3 * i + 2] = nr.z;
    }
    // glass (ior 1.5, roughness 0, specular (0.9, 0.8, 0.7) so that a dropped T.xy is visible) and a metal
    const Mat mats[2] = {{v3(1, 1, 1), 0, v3(0.9f, 0.8f, 0.7f), 0, v3(0, 0, 0), 1.5f},
                         {v3(0.5f, 0.6f, 0.7f), 0.5f, v3(0.3f, 0.2f, 0.1f), 0.2f, v3(0, 0, 0), 0}};
    float *dd, *dn;
    Mat *dm;
    Out *o1, *o2;
    if (hipMalloc(&dd, 12 * n) || hipMalloc(&dn, 12 * n) || hipMalloc(&dm, sizeof(mats)) ||
        hipMalloc(&o1, sizeof(Out) * n) || hipMalloc(&o2, sizeof(Out) * n)) {
        std::printf("{\"error\": \"hipMalloc\"}\n");
        return 1;
    }
    (void)hipMemcpy(dd, dirs.data(), 12 * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(dn, normals.data(), 12 * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(dm, mats, sizeof(mats), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(scatter_kernel<false>, dim3((n + 255) / 256), dim3(256), 0, 0, dd, dn, dm, n, o1);
    hipLaunchKernelGGL(scatter_kernel<true>, dim3((n + 255) / 256), dim3(256), 0, 0, dd, dn, dm, n, o2);
    std::vector<Out> c(n), l(n);
    if (hipMemcpy(c.data(), o1, sizeof(Out) * n, hipMemcpyDeviceToHost) ||
        hipMemcpy(l.data(), o2, sizeof(Out) * n, hipMemcpyDeviceToHost)) {
        std::printf("{\"error\": \"kernel\"}\n");
        return 1;
    }
    int bad_const = 0, bad_laund = 0, reflect = 0, bad_const_reflect = 0;
    for (int i = 0; i < n; i++) {
        const V3 d = v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        const V3 nrm = v3(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
        Rng rng = pcg_seed((uint32_t)i * 4137874753u + 279220567u);
        V3 T = v3(1, 1, 1), C = v3(0, 0, 0), nd = d;
        const int path = reflect_path(d, nrm, mats[i & 1], rng);
        scatter(d, nrm, mats[i & 1], rng, T, C, nd);
        const Out h{T.x, T.y, T.z, C.x, C.y, C.z, nd.x, nd.y, nd.z, (float)path};
        reflect += path == 1;
        const bool bc = std::memcmp(&h, &c[i], sizeof(Out)) != 0, bl = std::memcmp(&h, &l[i], sizeof(Out)) != 0;
        bad_const += bc;
        bad_laund += bl;
        bad_const_reflect += bc && path == 1;
    }
    std::printf("{\"n\": %d, \"dielectric_reflect\": %d, \"laundered_mismatch\": %d, \"constant_mismatch\": %d, "
                "\"constant_mismatch_on_reflect\": %d}\n", n, reflect, bad_laund, bad_const, bad_const_reflect);
    return 0;
}
