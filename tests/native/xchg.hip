// xchg.hip — TEST / PROBE INFRASTRUCTURE: device-side implementations of the pixel-tile bucket-byte
// exchange (rt_exchange_fn with on_device = 1, include/rt_abi.h) for hosts that have ONE GPU.
//
//  * xchg_group_*: several tile owners (one rt_renderer each, in their own host threads) on the same
//    device sum their byte arrays device-side, on the pass streams the renderer hands over: the
//    contract RCCL's in-place ncclAllReduce fulfils in the multi-GPU library path.  Per call:
//      1. every owner records an event after its bytes and publishes (pointer, n) at a host barrier;
//      2. every owner's stream waits for all owners' events and sums all arrays into its own scratch;
//      3. a second barrier (everyone has enqueued its reads), then each stream waits for the others'
//         sum kernels and copies its scratch back over its bytes.
//    No host synchronisation with the device: the host threads only meet at the barriers.
//  * xchg_emulate_peers: one owner alone (the 1-GPU "tile share" probe of bench.py).  The global
//    slots of the absent owners (zero bytes) are filled so that the global order has the size a real
//    N-owner run would have: each becomes live (a bucket from a hash of the slot) with the fraction
//    of this owner's own slots that are live, else terminated (65).  The own rays' seeds therefore
//    differ from a real run's, but the global ranking works on a realistic live count.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

namespace {

constexpr int kMaxOwners = 16;

struct Ptrs {
    const uint8_t *p[kMaxOwners];
};

__global__ void sum_kernel(Ptrs in, int owners, uint8_t *__restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t s = 0;
        for (int k = 0; k < owners; k++) s += in.p[k][i];
        out[i] = (uint8_t)s;
    }
}

struct Group;
struct Scratch {
    hipStream_t stream;
    uint8_t *p;
    uint64_t cap;
};
struct Member {
    Group *g;
    int rank;
    // one scratch per pass stream: the calls of different passes in flight run on different streams
    // and must not share a buffer
    std::vector<Scratch> scratch;
    hipEvent_t bytes_ready = nullptr, read_done = nullptr;
};

struct Group {
    int owners;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<Member> mem;
    std::vector<const uint8_t *> ptr;
    std::vector<uint64_t> cnt;
    void barrier() {
        std::unique_lock<std::mutex> l(m);
        const uint64_t my = gen;
        if (++arrived == owners) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != my; });
        }
    }
};

__global__ void own_count_kernel(const uint8_t *__restrict__ b, uint64_t n, unsigned long long *__restrict__ cnt) {
    unsigned own = 0, live = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = b[i];
        own += v != 0;
        live += v >= 1 && v <= 64;
    }
    // one atomic pair per wave (per-lane atomics on two words serialised the whole grid)
    for (int off = 32; off > 0; off >>= 1) {
        own += __shfl_xor(own, off);
        live += __shfl_xor(live, off);
    }
    if ((threadIdx.x & 63) == 0 && own) {
        atomicAdd(&cnt[0], (unsigned long long)own);
        atomicAdd(&cnt[1], (unsigned long long)live);
    }
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void fill_kernel(uint8_t *__restrict__ b, uint64_t n, const unsigned long long *__restrict__ cnt, uint32_t salt) {
    const unsigned long long own = cnt[0], live = cnt[1];     // live <= own < 2^31
    // P(live) = live / own as a 32-bit threshold
    const unsigned long long t = own ? (live << 32) / own : 0ull;
    const uint32_t thr = t > 0xffffffffull ? 0xffffffffu : (uint32_t)t;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (b[i]) continue;
        const uint32_t h = mix((uint32_t)i * 0x9e3779b9u ^ salt);
        b[i] = (uint8_t)((mix(h) < thr) ? 1 + (h & 63u) : 65u);
    }
}

// Counter pairs in a ring: each call uses its own pair on its own stream, so the passes in flight
// (one stream each) never wait for each other through the probe (the host runs at most a bounce
// ahead of each stream, far fewer calls than the ring holds).
constexpr int kRing = 1024;
struct Emu {
    unsigned long long *cnt = nullptr;
    uint32_t calls = 0;
};

}  // namespace

extern "C" {

void *xchg_group_create(int owners) {
    if (owners < 1 || owners > kMaxOwners) return nullptr;
    auto *g = new Group();
    g->owners = owners;
    g->mem.resize(owners);
    g->ptr.resize(owners);
    g->cnt.resize(owners);
    for (int k = 0; k < owners; k++) {
        g->mem[k].g = g;
        g->mem[k].rank = k;
        if (hipEventCreateWithFlags(&g->mem[k].bytes_ready, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->mem[k].read_done, hipEventDisableTiming) != hipSuccess)
            return nullptr;
    }
    return g;
}

void *xchg_group_member(void *group, int rank) {
    auto *g = static_cast<Group *>(group);
    return (g && rank >= 0 && rank < g->owners) ? &g->mem[rank] : nullptr;
}

void xchg_group_destroy(void *group) {
    auto *g = static_cast<Group *>(group);
    if (!g) return;
    for (auto &m : g->mem) {
        for (auto &x : m.scratch) (void)hipFree(x.p);
        if (m.bytes_ready) (void)hipEventDestroy(m.bytes_ready);
        if (m.read_done) (void)hipEventDestroy(m.read_done);
    }
    delete g;
}

// rt_exchange_fn (on_device = 1) for one member of a same-device group
int xchg_group_fn(void *user, uint8_t *bytes, uint64_t n, void *stream) {
    auto *me = static_cast<Member *>(user);
    Group *g = me->g;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Scratch *sc = nullptr;
    for (auto &x : me->scratch)
        if (x.stream == s) sc = &x;
    if (!sc) {
        me->scratch.push_back(Scratch{s, nullptr, 0});
        sc = &me->scratch.back();
    }
    if (n > sc->cap) {                 // the first (largest: bounce 0) call on a stream sizes its scratch
        if (sc->p) {
            if (hipStreamSynchronize(s) != hipSuccess) return -2;
            (void)hipFree(sc->p);
        }
        if (hipMalloc(reinterpret_cast<void **>(&sc->p), n) != hipSuccess) return -2;
        sc->cap = n;
    }
    if (hipEventRecord(me->bytes_ready, s) != hipSuccess) return -3;
    g->ptr[me->rank] = bytes;
    g->cnt[me->rank] = n;
    g->barrier();                      // every owner's bytes are published (and their events recorded)
    Ptrs in{};
    for (int k = 0; k < g->owners; k++) {
        if (g->cnt[k] != n) return -4;  // owners disagree on the global live count
        in.p[k] = g->ptr[k];
        if (k != me->rank && hipStreamWaitEvent(s, g->mem[k].bytes_ready, 0) != hipSuccess) return -5;
    }
    const int grid = (int)std::min<uint64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(sum_kernel, dim3(grid), dim3(256), 0, s, in, g->owners, sc->p, n);
    if (hipGetLastError() != hipSuccess) return -6;
    if (hipEventRecord(me->read_done, s) != hipSuccess) return -7;
    g->barrier();                      // every owner has enqueued its reads of all arrays
    for (int k = 0; k < g->owners; k++)
        if (k != me->rank && hipStreamWaitEvent(s, g->mem[k].read_done, 0) != hipSuccess) return -8;
    if (hipMemcpyAsync(bytes, sc->p, n, hipMemcpyDeviceToDevice, s) != hipSuccess) return -9;
    return 0;
}

void *xchg_emulate_create(void) {
    auto *e = new Emu();
    if (hipMalloc(reinterpret_cast<void **>(&e->cnt), 2 * kRing * sizeof(unsigned long long)) != hipSuccess) {
        delete e;
        return nullptr;
    }
    return e;
}

void xchg_emulate_destroy(void *emu) {
    auto *e = static_cast<Emu *>(emu);
    if (!e) return;
    if (e->cnt) (void)hipFree(e->cnt);
    delete e;
}

// rt_exchange_fn (on_device = 1): one owner alone, the absent owners' slots emulated (see top).
int xchg_emulate_peers(void *emu, uint8_t *bytes, uint64_t n, void *stream) {
    auto *e = static_cast<Emu *>(emu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *cnt = e->cnt + 2 * (e->calls % kRing);
    if (hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned long long), s) != hipSuccess) return -3;
    const int grid = (int)std::min<uint64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(own_count_kernel, dim3(grid), dim3(256), 0, s, bytes, n, cnt);
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, bytes, n, cnt, e->calls * 0x632be5abu);
    if (hipGetLastError() != hipSuccess) return -4;
    e->calls++;
    return 0;
}

}  // extern "C"
