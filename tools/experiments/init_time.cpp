// Times the HIP runtime's start-up in a fresh process (hipGetDeviceCount -> ROCr/HSA init), then
// the first stream.  Run it with and without ROCR_VISIBLE_DEVICES to see what device enumeration costs.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
int main() {
    using clk = std::chrono::high_resolution_clock;
    const auto t0 = clk::now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { std::printf("hipGetDeviceCount failed\n"); return 1; }
    const auto t1 = clk::now();
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    const auto t2 = clk::now();
    std::printf("devices %d  init %.1f ms  first stream %.1f ms\n", n,
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(t2 - t1).count());
    (void)hipStreamDestroy(s);
    return 0;
}
