// Exhaustive check (all 2^32 fp32 inputs) of the hardware sqrt against the correctly rounded
// sqrtf the render uses (-fhip-fp32-correctly-rounded-divide-sqrt), and of a one-step
// FMA-corrected variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t base, unsigned long long *bad, uint32_t *ex) {
    const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float a = __uint_as_float(bits);
    if (!(a >= 0x1p-120f && a <= 0x1p120f)) return;     // positive normal range only
    const float ref = sqrtf(a);
    const float s = __builtin_amdgcn_sqrtf(a);
    if (__float_as_uint(s) != __float_as_uint(ref)) { atomicAdd(bad, 1ull); *ex = bits; }
    // one correction: s +- 1 ulp chosen by the sign of the residual a - s*s
    const float sp = __uint_as_float(__float_as_uint(s) + 1), sm = __uint_as_float(__float_as_uint(s) - 1);
    const float rm = __builtin_fmaf(-sm, s, a), rp = __builtin_fmaf(-sp, s, a);
    float c = s;
    if (rm <= 0.0f) c = sm;
    if (rp > 0.0f) c = sp;
    if (__float_as_uint(c) != __float_as_uint(ref)) { atomicAdd(bad + 1, 1ull); ex[1] = bits; }
}

int main() {
    unsigned long long *d;
    uint32_t *ex;
    hipMalloc(&d, 16); hipMalloc(&ex, 8);
    hipMemset(d, 0, 16); hipMemset(ex, 0, 8);
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)base, d, ex);
    unsigned long long h[2]; uint32_t e[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    hipMemcpy(e, ex, 8, hipMemcpyDeviceToHost);
    std::printf("v_sqrt_f32: %llu mismatches (e.g. 0x%08x); corrected: %llu (e.g. 0x%08x)\n", h[0], e[0], h[1], e[1]);
    return 0;
}
