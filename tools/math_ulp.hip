// math_ulp.hip — TEST INFRASTRUCTURE: distance of the path tracer's float sin/cos/atan kernels
// (rt_sincos, rt_atan01 in csrc/rt_device.h, used by random_on_sphere and the env-map projection)
// from glibc's sinf/cosf/atanf (what the reference `cpu` path called, random.cuh:63-75 and
// scene.cu:297) and from the correctly rounded value (double sin/cos/atan rounded to float), over
// every float in the ranges the renderer feeds them: [0, 2*pi] for rt_sincos (random_radians can
// return float(2*pi)) and [0, 1] for rt_atan01.  The reference GPU path used nvcc --use_fast_math
// __sinf/__cosf, whose bits are not reproducible here: this bounds the part of the
// "parity unpinned" exposure that these kernels contribute.
//
//   math_ulp [stride]      (stride 1 = exhaustive; prints one JSON line)
// Host code only (hipcc compiles rt_device.h's __host__ __device__ functions for the CPU).
#include "rt_device.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {

uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
float from_bits(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
// ulp distance between two finite floats (monotonic integer mapping of the float line)
int64_t ulps(float a, float b) {
    auto key = [](float f) -> int64_t {
        const int32_t i = (int32_t)bits(f);
        return i < 0 ? (int64_t)INT32_MIN - i : (int64_t)i;
    };
    const int64_t d = key(a) - key(b);
    return d < 0 ? -d : d;
}

struct Stat {
    int64_t max_ulp_glibc = 0, max_ulp_exact = 0;
    double max_abs_exact = 0;
    float worst_x = 0;
    uint64_t n = 0, differ_glibc = 0;
    void add(float x, float mine, float glibc, float exact) {
        n++;
        const int64_t ug = ulps(mine, glibc), ue = ulps(mine, exact);
        if (ug) differ_glibc++;
        if (ug > max_ulp_glibc) { max_ulp_glibc = ug; worst_x = x; }
        if (ue > max_ulp_exact) max_ulp_exact = ue;
        const double a = std::fabs((double)mine - (double)exact);
        if (a > max_abs_exact) max_abs_exact = a;
    }
    void print(const char *name, bool comma) const {
        std::printf("\"%s\": {\"n\": %llu, \"max_ulp_vs_glibc\": %lld, \"differ_from_glibc\": %llu, "
                    "\"max_ulp_vs_correctly_rounded\": %lld, \"max_abs_err\": %.3e, \"worst_x_vs_glibc\": %.9g}%s",
                    name, (unsigned long long)n, (long long)max_ulp_glibc, (unsigned long long)differ_glibc,
                    (long long)max_ulp_exact, max_abs_exact, worst_x, comma ? ", " : "");
    }
};

}  // namespace

int main(int argc, char **argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1u;
    const float two_pi = (float)(3.14159265358979323846 * 2);
    Stat s, c, a;
    for (uint32_t u = 0; u <= bits(two_pi); u += stride) {
        const float x = from_bits(u);
        float ms, mc;
        rtd::rt_sincos(x, ms, mc);
        s.add(x, ms, sinf(x), (float)std::sin((double)x));
        c.add(x, mc, cosf(x), (float)std::cos((double)x));
    }
    for (uint32_t u = 0; u <= bits(1.0f); u += stride) {
        const float x = from_bits(u);
        a.add(x, rtd::rt_atan01(x), atanf(x), (float)std::atan((double)x));
    }
    std::printf("{\"stride\": %u, ", stride);
    s.print("sin_0_2pi", true);
    c.print("cos_0_2pi", true);
    a.print("atan_0_1", false);
    std::printf("}\n");
    return 0;
}
