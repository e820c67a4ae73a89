// launch_chain.hip — GPU-side dependent-launch latency vs concurrent streams (round 6 measurement tool).
// S streams each hold a chain of K launches of a tiny kernel.  Every chain is enqueued behind an event that a
// spinning kernel signals only after the host has finished enqueueing, so the time from that event to the end of
// the chains is the GPU's dispatch of the chains alone (no host launch cost).  Prints us per dependent launch of
// one chain for S = 1, 2, 4, 6, 12, 20, with grids of 1 and of 2048 workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

__global__ void tiny(int *p, int n) {
    if (blockIdx.x * blockDim.x + threadIdx.x < n) p[blockIdx.x * blockDim.x + threadIdx.x] += 1;
}
__global__ void spin(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

int main() {
    const int K = 400;
    int *d = nullptr;
    CK(hipMalloc(&d, 1 << 24));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    hipStream_t gate;
    CK(hipStreamCreateWithFlags(&gate, hipStreamNonBlocking));
    std::vector<hipStream_t> st(20);
    std::vector<hipEvent_t> done(20);
    for (int s = 0; s < 20; s++) {
        CK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
        CK(hipEventCreate(&done[s]));
    }
    hipEvent_t go;
    CK(hipEventCreate(&go));
    for (int grid : {1, 2048}) {
        for (int S : {1, 2, 4, 6, 12, 20}) {
            for (int rep = 0; rep < 2; rep++) {
                CK(hipDeviceSynchronize());
                hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, gate, (unsigned long long)khz * 200);   // 200 ms
                CK(hipEventRecord(go, gate));
                for (int s = 0; s < S; s++) CK(hipStreamWaitEvent(st[s], go, 0));
                for (int k = 0; k < K; k++)
                    for (int s = 0; s < S; s++) hipLaunchKernelGGL(tiny, dim3(grid), dim3(256), 0, st[s], d + s * 256, 64);
                for (int s = 0; s < S; s++) CK(hipEventRecord(done[s], st[s]));
                CK(hipDeviceSynchronize());
                float worst = 0;
                for (int s = 0; s < S; s++) {
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, go, done[s]));
                    worst = ms > worst ? ms : worst;
                }
                if (rep) std::printf("grid %4d streams %2d: %.2f ms for %d dependent launches per stream -> %.1f us each "
                                     "(%.0f k launches/s over all streams)\n", grid, S, worst, K, worst * 1e3 / K,
                                     S * K / worst);
            }
        }
    }
    return 0;
}
