// Cost of the renderer's setup calls on MI355X: hipMalloc/hipFree by size, hipMallocAsync from a
// pool, hipMemset of the allocation, hipStreamCreate, hipEventCreate.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
using clk = std::chrono::high_resolution_clock;
static double ms(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }
int main() {
    auto t = clk::now();
    (void)hipFree(nullptr);
    std::printf("runtime init (hipFree(0)) %.1f ms\n", ms(t));
    for (size_t mb : {64, 1024, 2600, 13000}) {
        void *p = nullptr;
        t = clk::now();
        (void)hipMalloc(&p, mb << 20);
        const double a = ms(t);
        t = clk::now();
        (void)hipMemset(p, 0, 1 << 20);
        (void)hipDeviceSynchronize();
        const double first_touch = ms(t);
        t = clk::now();
        (void)hipFree(p);
        std::printf("hipMalloc %6zu MB %8.2f ms   first memset+sync %6.2f ms   hipFree %8.2f ms\n", mb, a, first_touch, ms(t));
    }
    // the same sizes split into the renderer's 12 buffers per context
    t = clk::now();
    std::vector<void *> bufs;
    for (int k = 0; k < 5 * 12; k++) { void *p; (void)hipMalloc(&p, 220ull << 20); bufs.push_back(p); }
    const double a = ms(t);
    t = clk::now();
    for (void *p : bufs) (void)hipFree(p);
    std::printf("60 x hipMalloc 220 MB %.2f ms, hipFree %.2f ms\n", a, ms(t));
    hipStream_t s;
    (void)hipStreamCreate(&s);
    t = clk::now();
    for (int k = 0; k < 5; k++) { void *p; (void)hipMallocAsync(&p, 2600ull << 20, s); (void)hipFreeAsync(p, s); }
    (void)hipStreamSynchronize(s);
    std::printf("5 x hipMallocAsync/hipFreeAsync 2.6 GB (default pool) %.2f ms\n", ms(t));
    t = clk::now();
    std::vector<hipStream_t> ss(16);
    for (auto &x : ss) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    std::printf("16 x hipStreamCreate %.2f ms\n", ms(t));
    t = clk::now();
    std::vector<hipEvent_t> ev(512);
    for (auto &e : ev) (void)hipEventCreate(&e);
    std::printf("512 x hipEventCreate %.2f ms\n", ms(t));
    t = clk::now();
    for (auto &x : ss) (void)hipStreamDestroy(x);
    for (auto &e : ev) (void)hipEventDestroy(e);
    std::printf("destroy streams+events %.2f ms\n", ms(t));
    return 0;
}
