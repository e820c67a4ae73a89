// Microbenchmark: chip-wide rate of dependent random 64-B record fetches (the trace step's
// memory pattern), plain per-lane loads (4 x dwordx4) vs 2 lanes per record (DPP exchange).
// Build: hipcc --offload-arch=gfx950 -O3 -o gather_bench gather_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <chrono>
#include <cstring>

__global__ __launch_bounds__(256) void chase_plain(const float4 *__restrict__ tab, uint32_t mask, int steps,
                                                   uint32_t *out) {
    uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 2654435761u & mask;
    float acc = 0;
    for (int s = 0; s < steps; s++) {
        const float4 *r = tab + (size_t)i * 4;
        const float4 a = r[0], b = r[1], c = r[2], d = r[3];
        acc += a.x + b.y + c.z;
        i = (__float_as_uint(d.w) ^ (uint32_t)s) & mask;
    }
    out[blockIdx.x * 256 + threadIdx.x] = i + (uint32_t)acc;
}

// 2 lanes per record: lane pair loads the even lane's record (parts 0..3 over 2 loads) and the
// odd lane's record (2 loads); each load instruction touches 32 lines instead of 64.
__global__ __launch_bounds__(256) void chase_pair(const float4 *__restrict__ tab, uint32_t mask, int steps,
                                                  uint32_t *out) {
    uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 2654435761u & mask;
    const uint32_t lane = threadIdx.x & 63, odd = lane & 1;
    float acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint32_t ie = __shfl(i, lane & ~1u), io = __shfl(i, lane | 1u);
        const float4 *re = tab + (size_t)ie * 4 + odd, *ro = tab + (size_t)io * 4 + odd;
        const float4 e0 = re[0], e1 = re[2], o0 = ro[0], o1 = ro[2];   // parts odd, odd+2
        // even lane needs e0 (part0), e1 (part2) own + parts 1,3 from partner's e0/e1
        // odd lane needs parts 0,2 from partner's o0/o1 and o0/o1 own (parts 1,3)
        const float4 x0 = odd ? o0 : e0, x1 = odd ? o1 : e1;          // mine: parts odd, odd+2 of my record
        const float4 y0 = odd ? e0 : o0, y1 = odd ? e1 : o1;          // partner's record: send
        float4 z0, z1;                                                 // partner sends me my other parts
        z0.x = __shfl_xor(y0.x, 1); z0.y = __shfl_xor(y0.y, 1); z0.z = __shfl_xor(y0.z, 1); z0.w = __shfl_xor(y0.w, 1);
        z1.x = __shfl_xor(y1.x, 1); z1.y = __shfl_xor(y1.y, 1); z1.z = __shfl_xor(y1.z, 1); z1.w = __shfl_xor(y1.w, 1);
        const float4 p0 = odd ? z0 : x0, p1 = odd ? x0 : z0, p2 = odd ? z1 : x1, p3 = odd ? x1 : z1;
        (void)p1;
        acc += p0.x + p1.y + p2.z;
        i = (__float_as_uint(p3.w) ^ (uint32_t)s) & mask;
    }
    out[blockIdx.x * 256 + threadIdx.x] = i + (uint32_t)acc;
}

int main() {
    const int steps = 400;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4 * 4);
    for (uint32_t mb : {2u, 4u, 8u, 16u, 64u}) {
        const uint32_t n = mb * (1u << 20) / 64;   // records (power of two)
        std::vector<float4> h((size_t)n * 4);
        uint64_t x = 88172645463325252ull;
        for (size_t k = 0; k < h.size(); k++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            uint32_t u = (uint32_t)x; float f; std::memcpy(&f, &u, 4); h[k] = make_float4(1, 1, 1, f);
        }
        float4 *tab;
        hipMalloc(&tab, h.size() * 16);
        hipMemcpy(tab, h.data(), h.size() * 16, hipMemcpyHostToDevice);
        for (int occ : {2, 4, 8}) {
            const int blocks = cus * occ;   // occ workgroups of 4 waves per CU
            for (int kind = 0; kind < 2; kind++) {
                auto run = [&]() {
                    if (kind == 0) hipLaunchKernelGGL(chase_plain, dim3(blocks), dim3(256), 0, 0, tab, n - 1, steps, out);
                    else hipLaunchKernelGGL(chase_pair, dim3(blocks), dim3(256), 0, 0, tab, n - 1, steps, out);
                };
                run();
                hipDeviceSynchronize();
                hipEvent_t a, b;
                hipEventCreate(&a); hipEventCreate(&b);
                hipEventRecord(a);
                for (int r = 0; r < 5; r++) run();
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double recs = 5.0 * blocks * 256.0 * steps;
                std::printf("table %3u MB  waves/SIMD %d  %-5s  %.1f G records/s  (%.2f TB/s of 64-B records)\n", mb, occ,
                            kind ? "pair" : "plain", recs / (ms * 1e-3) / 1e9, recs * 64 / (ms * 1e-3) / 1e12);
            }
        }
        hipFree(tab);
    }
    return 0;
}
