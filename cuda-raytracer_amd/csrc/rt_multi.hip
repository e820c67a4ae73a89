// rt_multi.hip — multi-GPU rendering in one process: pass sharding over the devices of one node,
// framebuffer exchange over RCCL (xGMI).  SURVEY §8b (rt_opts.device_count / device_ids) and §8e
// ("Alternative: pass sharding ... exact with sort on, zero per-bounce traffic").
//
// Replaces gpu_raytrace (reference raytracing.cu:170-284) when rt_opts.device_count >= 1.  The
// reference ran one device; its pass loop (raytracing.cu:222-254) is a sequence of independent
// 20-spp passes, each with its own generate seed, per-bounce process seeds and stable reorder,
// so a pass renders identically on any device.
//
//   * Device k of N renders passes k, k+N, k+2N, ... (round-robin: passes cost the same except a
//     shorter last one), as many in flight as its renderer keeps, into padded pass buffers.
//   * The framebuffer is owned per pixel slice: W*H*3 floats cut into N slices of sl floats.
//     One ncclAllToAll per round sends slice j of each pass buffer to device j (each xGMI link
//     carries 1/N of the data; nothing converges on one GPU), and device j adds the slices it
//     received in pass order, fb_j = ((0 + S_0,j) + S_1,j) + ..., exactly the per-pixel add
//     sequence of one device: the N-device image is bit-identical to the 1-device image with
//     sort on or off.  The exchange of every 4 rounds runs while later passes still render.
//   * One ncclGather of the N finished slices to device_ids[0] (then, if asked, one D2H copy).
//
// Exchange bytes per frame: every pass buffer leaves its device except its own slice,
// P * W*H*3*4 * (N-1)/N in all (1080p teapot, N = 8: 103 passes x 24.9 MB x 7/8 = 2.24 GB over the
// job, ~280 MB per device, 1/7 of it per link), plus the gather's W*H*3*4 * (N-1)/N into device 0.
//
// rt_multi (round 6) is the persistent form: the communicator, one renderer per device (scene
// resident, pass contexts allocated) and the exchange buffers are set up once by rt_multi_create,
// and each rt_multi_run renders the first `pass_count` passes of the frame with one host thread per
// device (RCCL's one-thread-per-device model for a single-process communicator).  rt_render with
// device_count >= 1 is create + run + destroy.  device_count = 1 runs the same code with every
// exchange local.
//
// rt_opts.shard_tiles = 1 (one-shot rt_render only) deals pixel tiles instead (§8e's natural
// shard): device k renders owner k's row stripes of every pass; with sort on the owners all-reduce
// one byte per global live ray after every bounce but the last (nccl_exchange), and the frame is an
// ncclReduce of the owners' framebuffers.
#include "rt_abi.h"
#include "mgpu_protocol.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rtamd {
int fail(int code, const std::string &msg);
}
extern "C" int rtamd_renderer_set_poll(rt_renderer *r, int (*fn)(void *), void *user);   // rt_render.hip
extern "C" int rtamd_renderer_run_pitched(rt_renderer *r, int pass_begin, int count, int stride,
                                          float *d_pass_sums, size_t pitch, rt_stats *stats);   // rt_render.hip
extern "C" int rtamd_renderer_create_inflight(const rt_scene *scene, const rt_opts *opts, rt_renderer **out,
                                              int inflight);                                 // rt_render.hip
extern "C" int rtamd_renderer_run_async_pitched(rt_renderer *r, int pass_begin, int count, int stride,
                                                float *d_pass_sums, size_t pitch);             // rt_render.hip

namespace {

// slice[i] += recv[j][src][i] for the rounds j of the chunk and the ranks src whose pass exists,
// in ascending pass order (pass = src + N * (k0 + j)): one lane per element, ordered adds.
__global__ __launch_bounds__(256) void add_slices_kernel(float *__restrict__ slice, const float *__restrict__ recv,
                                                         size_t sl, int world, int rounds, int k0, int passes) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= sl) return;
    float acc = slice[i];
    for (int j = 0; j < rounds; j++)
        for (int src = 0; src < world; src++)
            if (src + world * (k0 + j) < passes) acc = acc + recv[((size_t)j * world + src) * sl + i];
    slice[i] = acc;
}

const char *nccl_str(ncclResult_t r) { return ncclGetErrorString(r); }

constexpr int kInflightNextToRccl = 16;   // passes in flight of a device's renderer (run_device)

void add_stats(rt_stats &a, const rt_stats &s) {
    a.live_segments += s.live_segments;
    a.generated_rays += s.generated_rays;
    a.sorted_items += s.sorted_items;
    a.nodes_popped += s.nodes_popped;
    a.internal_visits += s.internal_visits;
    a.triangle_tests += s.triangle_tests;
    a.sphere_tests += s.sphere_tests;
    a.hits += s.hits;
    a.misses += s.misses;
    a.hits_sphere += s.hits_sphere;
    a.dead_slots += s.dead_slots;
    a.passes += s.passes;
    a.process_ms += s.process_ms;
    a.sort_ms += s.sort_ms;
    a.trace_ms += s.trace_ms;
    a.trace_launches += s.trace_launches;
    a.kernel_ms += s.kernel_ms;
}

// the devices' stats summed, except the times that overlap: kernel and exchange time are the slowest device's
template <class Dev>
void total_stats(rt_stats *stats, const std::vector<Dev> &devs) {
    std::memset(stats, 0, sizeof(*stats));
    for (auto &d : devs) {
        const double k = stats->kernel_ms;
        add_stats(*stats, d.stats);
        stats->kernel_ms = std::max(k, d.stats.kernel_ms);
        stats->exchange_ms = std::max(stats->exchange_ms, d.exchange_ms);
    }
}

// The abort protocol (setup barrier, shared failure flag, each device aborting only its own
// communicator) lives in mgpu_protocol.h, free of HIP/RCCL types so that it is tested on the CPU.
void comm_abort(ncclComm_t c) { (void)ncclCommAbort(c); }
using Sync = rtamd_mgpu::Sync;
using Link = rtamd_mgpu::LinkT<ncclComm_t, comm_abort>;
using RunGuard = rtamd_mgpu::RunGuardT<Link>;

// the renderer's abort poll (rtamd_renderer_set_poll): a tile exchange waits on this device's collective
int link_poll(void *user) { return static_cast<Link *>(user)->check(); }

int hip_err(hipError_t e, const char *what) {
    return rtamd::fail(e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP,
                       std::string("Error ") + what + " " + hipGetErrorString(e));
}

#ifdef RTAMD_TEST_HOOKS
// ---- Test build only (librtamd_test.so, -DRTAMD_TEST_HOOKS; the product library has neither hook).
// Loopback transport (RTAMD_MULTI_LOOPBACK=1): the "devices" are host threads on ONE GPU (device_ids may
// repeat), and run_device's two collectives become device-to-device copies between the threads' buffers,
// ordered through events the threads swap at host barriers.  It exists so that the multi-device schedule --
// pass dealing, the stale rows of rounds a device has no pass in, the owners' ordered adds, the gather -- runs
// at N > 1 on a one-GPU box (RCCL refuses two ranks on one GPU).  A device that fails releases the others
// from the barrier (fail()), so a failing loopback test returns instead of hanging.
struct Loopback {
    int world = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool failed = false;
    std::vector<hipEvent_t> ev_in, ev_out;    // per rank, re-recorded at every collective
    std::vector<float *> send, recv;          // per rank: the current collective's buffers
    ~Loopback() {
        for (auto e : ev_in) if (e) (void)hipEventDestroy(e);
        for (auto e : ev_out) if (e) (void)hipEventDestroy(e);
    }
    int init(const std::vector<int> &devs) {
        world = (int)devs.size();
        send.assign(world, nullptr);
        recv.assign(world, nullptr);
        ev_in.assign(world, nullptr);
        ev_out.assign(world, nullptr);
        for (int k = 0; k < world; k++)
            if (hipSetDevice(devs[k]) != hipSuccess ||
                hipEventCreateWithFlags(&ev_in[k], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev_out[k], hipEventDisableTiming) != hipSuccess)
                return rtamd::fail(RT_E_HIP, "loopback: hipEventCreate failed");
        return RT_OK;
    }
    void reset() {
        std::lock_guard<std::mutex> l(m);
        arrived = 0;
        failed = false;
    }
    void fail() {
        std::lock_guard<std::mutex> l(m);
        failed = true;
        cv.notify_all();
    }
    bool barrier() {
        std::unique_lock<std::mutex> l(m);
        if (failed) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g || failed; });
        }
        return gen != g;
    }
    // entry: every rank's stream waits for every rank's work so far; exit: for every rank's copies
    int fence(std::vector<hipEvent_t> &ev, int rank, hipStream_t s) {
        if (hipEventRecord(ev[rank], s) != hipSuccess) return RT_E_HIP;
        if (!barrier()) return RT_E_INVALID;
        for (int p = 0; p < world; p++)
            if (p != rank && hipStreamWaitEvent(s, ev[p], 0) != hipSuccess) return RT_E_HIP;
        return RT_OK;
    }
    // ncclAllToAll of rows j0..j1 (sl floats per destination, rows `pitch` floats apart): recv[j][src] =
    // src's buf[j][rank]
    int alltoall(int rank, float *buf, float *rv, int j0, int j1, size_t pitch, size_t sl, hipStream_t s) {
        send[rank] = buf;
        recv[rank] = rv;
        if (int rc = fence(ev_in, rank, s)) return rc;
        for (int j = j0; j < j1; j++)
            for (int src = 0; src < world; src++)
                if (hipMemcpyAsync(rv + (size_t)j * pitch + (size_t)src * sl, send[src] + (size_t)j * pitch + (size_t)rank * sl,
                                   sl * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
                    return RT_E_HIP;
        return fence(ev_out, rank, s);
    }
    // ncclGather of every rank's sl-float slice into root's buffer, block src at src * sl (root's own in place)
    int gather(int rank, float *slice, size_t sl, hipStream_t s) {
        send[rank] = slice;
        if (int rc = fence(ev_in, rank, s)) return rc;
        if (rank == 0)
            for (int src = 1; src < world; src++)
                if (hipMemcpyAsync(slice + (size_t)src * sl, send[src], sl * sizeof(float), hipMemcpyDeviceToDevice, s) !=
                    hipSuccess)
                    return RT_E_HIP;
        return fence(ev_out, rank, s);
    }
};
bool loopback_requested() {
    const char *e = std::getenv("RTAMD_MULTI_LOOPBACK");
    return e && std::atoi(e) != 0;
}
// RTAMD_FAIL_AFTER_SETUP=<rank> makes that device fail right after the setup barrier, the path where its
// peers must not be left inside a collective.
bool injected_failure(int rank) {
    const char *e = std::getenv("RTAMD_FAIL_AFTER_SETUP");
    return e && *e && std::atoi(e) == rank;
}
#define RTAMD_INJECT(rank)                                                                               \
    do {                                                                                                 \
        if (injected_failure(rank)) return rtamd::fail(RT_E_INVALID, "injected failure (RTAMD_FAIL_AFTER_SETUP)"); \
    } while (0)
#else
struct Loopback {
    void fail() {}
    void reset() {}
    int alltoall(int, float *, float *, int, int, size_t, size_t, hipStream_t) { return RT_E_INVALID; }
    int gather(int, float *, size_t, hipStream_t) { return RT_E_INVALID; }
};
constexpr bool loopback_requested() { return false; }
#define RTAMD_INJECT(rank) ((void)(rank))
#endif

}  // namespace

#define MHIP(call)                                              \
    do {                                                        \
        const hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_err(e_, #call);        \
    } while (0)
#define MNCCL(call)                                                                                       \
    do {                                                                                                  \
        if (ln.check()) return rtamd::fail(RT_E_INVALID, "another device of the render failed");         \
        const ncclResult_t r_ = (call);                                                                   \
        if (r_ != ncclSuccess) return rtamd::fail(RT_E_HIP, std::string("Error ") + #call + " " + nccl_str(r_)); \
    } while (0)

namespace {

// Waits for stream s (which holds collectives) while watching the other devices: returns an error
// (and aborts this device's communicator) if one of them failed.
int wait_stream(hipStream_t s, Link &ln) {
    hipError_t err = hipSuccess;
    const rtamd_mgpu::WaitResult w = rtamd_mgpu::wait_watching([&] {
        err = hipStreamQuery(s);
        return err == hipSuccess ? 0 : err == hipErrorNotReady ? 1 : 2;
    }, ln);
    if (w == rtamd_mgpu::kDone) return RT_OK;
    if (w == rtamd_mgpu::kOwnError) return hip_err(err, "hipStreamQuery");
    return rtamd::fail(RT_E_INVALID, "another device of the render failed");
}
#define MWAIT(s)                                   \
    do {                                           \
        if (int rc_ = wait_stream((s), ln)) return rc_; \
    } while (0)

// One device of a persistent multi-device renderer.
struct MDev {
    int device = 0, rank = 0;
    rt_renderer *ren = nullptr;
    float *buf = nullptr, *recv = nullptr, *slice = nullptr;
    int *one = nullptr;               // the create-time rank count (ncclAllReduce of a 1 per device)
    hipStream_t s = nullptr;          // exchange stream
    int rc = 0;
    std::string err;
    rt_stats stats{};
    double exchange_ms = 0;
    void release() {
        if (device >= 0) (void)hipSetDevice(device);
        for (float *b : {buf, recv, slice})
            if (b) (void)hipFree(b);
        if (one) (void)hipFree(one);
        if (s) (void)hipStreamDestroy(s);
        if (ren) rt_renderer_destroy(ren);
        buf = recv = slice = nullptr;
        one = nullptr;
        s = nullptr;
        ren = nullptr;
    }
};

}  // namespace

struct rt_multi {
    int world = 0;
    bool loopback = false;
    bool broken = false;              // a run failed after its setup barrier: communicators may be aborted
    bool events = false;              // per-bounce HIP events in the devices' renderers
    int P = 0;                        // passes of the frame
    int ranks_seen = 0;
    size_t px3 = 0, sl = 0, pitch = 0;
    int chunk_cap = 1;                // rounds of pass buffers allocated per device
    std::vector<MDev> dev;
    std::vector<ncclComm_t> comms;
    std::vector<Link> links;
    std::unique_ptr<Loopback> lb;
    ~rt_multi() {
        for (auto &d : dev) d.release();
        for (size_t k = 0; k < comms.size(); k++)
            if (comms[k] && !(k < links.size() && links[k].aborted)) (void)ncclCommDestroy(comms[k]);   // aborted: freed
    }
};

namespace {

// Device d's share of the first np passes of the frame: render, exchange, add; the root also gathers
// (and copies the frame to fb_out if given).
int run_device(rt_multi &m, MDev &d, Link &ln, Sync &sy, int np, float *fb_out) {
    RunGuard run{sy, ln};
    struct Fail {                     // an error after the setup barrier releases loopback peers too
        RunGuard &run;
        Loopback *lb;
        ~Fail() {
            if (run.arrived && !run.ok && lb) lb->fail();
        }
    } fail_guard{run, m.lb.get()};
    ncclComm_t comm = ln.comm;
    const int world = m.world;
    Loopback *lb = m.lb.get();
    MHIP(hipSetDevice(d.device));
    const size_t sl = m.sl, pitch = m.pitch;
    const int R = (np + world - 1) / world;           // rounds: one pass per device each
    // One device: the all-to-all and the gather are the identity (every slice is its own), so they are skipped
    // and the adds read buf directly, as the torch.distributed path does at N = 1.  RTAMD_XCHG_IDENTITY=0 runs
    // them through RCCL anyway (the N = 1 tests keep the collectives exercised).
    const char *ide = std::getenv("RTAMD_XCHG_IDENTITY");
    const bool identity = world == 1 && !lb && (!ide || std::atoi(ide) != 0);
    // Rounds per renderer call: all of them (up to the buffers allocated at create), so that the renderer
    // keeps its passes in flight across the whole share (between calls it drains: a 26-pass share ran
    // 6.40 ms/pass in calls of 16 passes against 5.91 for one plain run).  The chunk is the same on every
    // device (it fixes the collective sequence): it depends only on R and the image size.
    const int chunk = std::max(1, std::min(R, m.chunk_cap));
    MHIP(hipMemsetAsync(d.slice, 0, sl * sizeof(float), d.s));
    MHIP(hipStreamSynchronize(d.s));
    d.stats = rt_stats{};
    d.exchange_ms = 0;
    if (!run.setup()) return rtamd::fail(RT_E_INVALID, "another device of the render failed");
    RTAMD_INJECT(d.rank);
    using clk = std::chrono::high_resolution_clock;
    const auto loop0 = clk::now();
    rt_renderer *ren = d.ren;
    float *buf = d.buf, *recv = d.recv, *slice = d.slice;
    int rc;
    // Overlapped exchange (the default; RTAMD_XCHG_OVERLAP=0: one exchange after each chunk's render):
    // the chunk's passes are enqueued without waiting (rt_renderer_run_async), and the exchange
    // stream takes the slices of every `xr` rounds as soon as this device's passes of those rounds
    // have written their sums (rt_renderer_wait_pass), while the later passes still render.  The
    // exchange order -- rounds, then the owners' ascending pass order in add_slices_kernel -- is the
    // synchronous one, so the image is the same bit for bit.  Every device issues the same sequence
    // of collectives (it depends only on R, chunk and xr).
    const char *ov = std::getenv("RTAMD_XCHG_OVERLAP");
    const bool overlap = !ov || std::atoi(ov) != 0;
    const char *xre = std::getenv("RTAMD_XCHG_ROUNDS");
    const int xr = overlap ? std::max(1, xre ? std::atoi(xre) : 4) : chunk;
    const bool gtime = std::getenv("RTAMD_TIMING") != nullptr;
    for (int k0 = 0; k0 < R; k0 += chunk) {
        const int mr = std::min(chunk, R - k0);
        // this device's passes of rounds k0 .. k0+mr-1
        const int first = d.rank + world * k0;
        const int mine = first < np ? std::min(mr, (np - 1 - first) / world + 1) : 0;
        if (mine > 0 && overlap) {
            rc = rtamd_renderer_run_async_pitched(ren, first, mine, world, buf, pitch);
            if (rc) return rc;
        }
        if (mine > 0 && !overlap) {
            rt_stats s{};
            rc = rtamd_renderer_run_pitched(ren, first, mine, world, buf, pitch, &s);
            if (rc) return rc;
            add_stats(d.stats, s);
        }
        // rounds of the chunk where this device has no pass send stale rows, which the owners'
        // adds skip (pass src + N*k does not exist)
        auto t0 = clk::now();
        // RTAMD_TIMING: when the exchange groups ran on the device (events around each group's adds)
        struct Events {
            std::vector<hipEvent_t> v;
            ~Events() { for (hipEvent_t e : v) (void)hipEventDestroy(e); }
        } gevs;
        std::vector<hipEvent_t> &gev = gevs.v;
        auto gmark = [&]() -> int {
            if (!gtime) return RT_OK;
            gev.push_back(nullptr);
            MHIP(hipEventCreate(&gev.back()));
            MHIP(hipEventRecord(gev.back(), d.s));
            return RT_OK;
        };
        if (int rc_ = gmark()) return rc_;
        for (int j0 = 0; j0 < mr; j0 += xr) {
            const int j1 = std::min(mr, j0 + xr);
            if (overlap)
                for (int j = j0; j < std::min(j1, mine); j++) {
                    rc = rt_renderer_wait_pass(ren, j, d.s);
                    if (rc) return rc;
                }
            if (int rc_ = gmark()) return rc_;     // the group's passes are done
            if (identity) {
            } else if (lb) {
                if (int rc2 = lb->alltoall(d.rank, buf, recv, j0, j1, pitch, sl, d.s))
                    return rtamd::fail(rc2, "loopback exchange failed");
            } else {
                MNCCL(ncclGroupStart());
                for (int j = j0; j < j1; j++)
                    MNCCL(ncclAllToAll(buf + (size_t)j * pitch, recv + (size_t)j * pitch, sl, ncclFloat32, comm, d.s));
                MNCCL(ncclGroupEnd());
            }
            hipLaunchKernelGGL(add_slices_kernel, dim3((unsigned)((sl + 255) / 256)), dim3(256), 0, d.s, slice,
                               (identity ? buf : recv) + (size_t)j0 * pitch, sl, world, j1 - j0, k0 + j0, np);
            MHIP(hipGetLastError());
            if (int rc_ = gmark()) return rc_;     // its adds are done
        }
        if (mine > 0 && overlap) {
            // the passes render on the renderer's own streams, which no collective waits behind:
            // this wait ends even if a peer device has failed
            rt_stats s{};
            rc = rt_renderer_finish(ren, &s);
            if (rc) return rc;
            add_stats(d.stats, s);
            t0 = clk::now();            // exchange_ms: what the render did not hide
        }
        // the next chunk's render overwrites buf: the exchange must have read it
        const auto tf = clk::now();
        MWAIT(d.s);
        d.exchange_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (gtime) {
            std::string line;
            for (size_t k = 1; k < gev.size(); k++) {
                float ms = 0;
                MHIP(hipEventElapsedTime(&ms, gev[0], gev[k]));
                line += (k % 2 ? " ready " : " added ") + std::to_string(ms);
            }
            std::fprintf(stderr, "rt_multi device %d chunk at round %d: exchange groups (ms after the chunk's enqueue):%s; "
                         "host wait after the render %.2f ms\n", d.rank, k0, line.c_str(),
                         std::chrono::duration<double, std::milli>(clk::now() - tf).count());
        }
    }
    const double loop_ms = std::chrono::duration<double, std::milli>(clk::now() - loop0).count();
    const double unhidden_ms = d.exchange_ms;
    const auto t0 = clk::now();
    // gather the finished slices to the root (in place: the root's own slice is block 0)
    if (lb) {
        if (int rc2 = lb->gather(d.rank, slice, sl, d.s)) return rtamd::fail(rc2, "loopback gather failed");
    } else if (!identity) {
        MNCCL(ncclGather(slice, slice, sl, ncclFloat32, 0, comm, d.s));
    }
    if (d.rank == 0 && fb_out) MHIP(hipMemcpyAsync(fb_out, slice, m.px3 * sizeof(float), hipMemcpyDeviceToHost, d.s));
    MWAIT(d.s);
    d.exchange_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (gtime)
        std::fprintf(stderr, "rt_multi device %d: %d passes rendered and exchanged in %.2f ms (exchange not hidden: %.2f ms, "
                     "%s), then gather%s %.2f ms\n", d.rank, (int)d.stats.passes, loop_ms, unhidden_ms,
                     overlap ? "overlapped" : "after each chunk", fb_out ? " + framebuffer to the host" : "",
                     std::chrono::duration<double, std::milli>(clk::now() - t0).count());
    run.ok = true;
    return RT_OK;
}

// Pixel tiles with the reorder on: the per-bounce bucket bytes summed over the devices in place
// (ncclAllReduce, uint8: every global slot has one owner, no byte exceeds 65), on the pass's stream.
// An aborted run (another device failed) issues no further collective.
int nccl_exchange(void *user, uint8_t *bytes, uint64_t n, void *stream) {
    Link &ln = *static_cast<Link *>(user);
    if (ln.check()) return RT_E_INVALID;
    const ncclResult_t r = ncclAllReduce(bytes, bytes, n, ncclUint8, ncclSum, ln.comm, static_cast<hipStream_t>(stream));
    return r == ncclSuccess ? 0 : -(int)r - 1;
}

struct TileState {
    int device = 0, rank = 0, rc = 0;
    std::string err;
    rt_stats stats{};
    double exchange_ms = 0;
};

// Device `st.rank`'s tiles: owner rank's tile_rows-row stripes of every pass, then an
// ncclReduce of the owners' framebuffers to the root: every pixel has one owner and is 0 elsewhere,
// so the sum is that owner's value bit for bit (x + 0 = x).
int run_device_tiles(const rt_scene *scene, const rt_opts *base, Link &ln, int world, TileState &st,
                     float *fb_out, Sync &sy) {
    RunGuard run{sy, ln};
    ncclComm_t comm = ln.comm;
    MHIP(hipSetDevice(st.device));
    const size_t px3 = (size_t)scene->width * scene->height * 3;
    rt_opts o = *base;
    o.device = st.device;
    o.device_count = 0;
    o.device_ids = nullptr;
    o.shard_tiles = 0;
    o.pass_begin = 0;
    o.pass_count = -1;
    o.pass_stride = 1;
    o.tile_count = world;
    o.tile_index = st.rank;
    rt_renderer *ren = nullptr;
    int rc = rt_renderer_create(scene, &o, &ren);
    if (rc) return rc;
    struct Guard {
        rt_renderer *r;
        RunGuard &run;
        float *d = nullptr;
        hipStream_t s = nullptr;
        ~Guard() {
            run.fail_now();
            if (d) (void)hipFree(d);
            if (s) (void)hipStreamDestroy(s);
            rt_renderer_destroy(r);
        }
    } g{ren, run};
    if (o.sort && world > 1) {
        rc = rt_renderer_set_exchange(ren, nccl_exchange, &ln, 1);
        if (rc) return rc;
        rc = rtamd_renderer_set_poll(ren, link_poll, &ln);
        if (rc) return rc;
    }
    MHIP(hipMalloc(reinterpret_cast<void **>(&g.d), px3 * sizeof(float)));
    MHIP(hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking));
    if (!run.setup()) return rtamd::fail(RT_E_INVALID, "another device of the render failed");
    RTAMD_INJECT(st.rank);
    rt_stats s{};
    using clk = std::chrono::high_resolution_clock;
    rc = rtamd_renderer_run_pitched(ren, 0, -1, 1, nullptr, 0, &s);
    if (rc) return rc;
    st.stats = s;
    rc = rt_renderer_copy_framebuffer(ren, g.d);
    if (rc) return rc;
    const auto t0 = clk::now();
    MNCCL(ncclReduce(g.d, g.d, px3, ncclFloat32, ncclSum, 0, comm, g.s));
    if (st.rank == 0) MHIP(hipMemcpyAsync(fb_out, g.d, px3 * sizeof(float), hipMemcpyDeviceToHost, g.s));
    MWAIT(g.s);
    st.exchange_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    run.ok = true;
    return RT_OK;
}

// The device list of a multi-device render (opts->device_ids or 0..N-1; with the loopback test
// transport every "device" is device 0 unless listed).
int device_list(const rt_opts *opts, bool loopback, std::vector<int> &devs) {
    const int world = opts->device_count;
    if (world < 1) return rtamd::fail(RT_E_INVALID, "device_count must be at least 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    devs.assign(world, 0);
    for (int k = 0; k < world; k++) {
        devs[k] = opts->device_ids ? opts->device_ids[k] : (loopback ? 0 : k);
        if (devs[k] < 0 || devs[k] >= ndev)
            return rtamd::fail(RT_E_NODEVICE, "device_ids: no such HIP device (" + std::to_string(devs[k]) + "; " +
                                                  std::to_string(ndev) + " visible)");
        for (int j = 0; j < k && !loopback; j++)
            if (devs[j] == devs[k]) return rtamd::fail(RT_E_INVALID, "device_ids: a device is listed twice");
    }
    return RT_OK;
}

int render_tiles(const rt_scene *scene, const rt_opts *opts, float *fb_out, rt_stats *stats) {
    using clk = std::chrono::high_resolution_clock;
    const auto w0 = clk::now();
    if (loopback_requested())
        return rtamd::fail(RT_E_INVALID, "RTAMD_MULTI_LOOPBACK covers pass sharding only (not shard_tiles)");
    std::vector<int> devs;
    if (int rc = device_list(opts, false, devs)) return rc;
    const int world = opts->device_count;
    std::vector<ncclComm_t> comms(world, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), world, devs.data());
    if (r != ncclSuccess) return rtamd::fail(RT_E_HIP, std::string("Error ncclCommInitAll ") + nccl_str(r));
    std::vector<TileState> st(world);
    Sync sy;
    sy.world = world;
    std::vector<Link> links(world);
    for (int k = 0; k < world; k++) {
        links[k].comm = comms[k];
        links[k].sy = &sy;
    }
    std::vector<std::thread> th;
    for (int k = 0; k < world; k++) {
        st[k].device = devs[k];
        st[k].rank = k;
        th.emplace_back([&, k]() {
            st[k].rc = run_device_tiles(scene, opts, links[k], world, st[k], fb_out, sy);
            if (st[k].rc) st[k].err = rt_last_error();
        });
    }
    for (auto &t : th) t.join();
    for (auto &l : links)
        if (!l.aborted && l.comm) (void)ncclCommDestroy(l.comm);   // ncclCommAbort already freed the others
    // report the device that failed first-hand, not a peer that returned because of it
    for (auto &s : st)
        if (s.rc && s.err.find("another device") == std::string::npos) return rtamd::fail(s.rc, s.err);
    for (auto &s : st)
        if (s.rc) return rtamd::fail(s.rc, s.err);
    if (stats) {
        total_stats(stats, st);
        stats->render_ms = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    }
    return RT_OK;
}

// first-hand error of a set of devices (not a peer that returned because of it)
int first_error(const std::vector<MDev> &dev) {
    for (auto &d : dev)
        if (d.rc && d.err.find("another device") == std::string::npos) return rtamd::fail(d.rc, d.err);
    for (auto &d : dev)
        if (d.rc) return rtamd::fail(d.rc, d.err);
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(const rt_scene *scene, const rt_opts *opts, rt_multi **out) {
    if (!out) return rtamd::fail(RT_E_INVALID, "null output");
    *out = nullptr;
    if (!scene || !opts) return rtamd::fail(RT_E_INVALID, "null argument");
    if (opts->shard_tiles) return rtamd::fail(RT_E_INVALID, "rt_multi: pass sharding only (shard_tiles is rt_render's)");
    if (opts->tile_count > 1) return rtamd::fail(RT_E_INVALID, "device_count and tile_count are exclusive "
                                                              "(shard_tiles = 1 deals the tiles over the devices)");
    if (opts->pass_begin != 0 || (opts->pass_count != -1 && opts->pass_count != (scene->ray_count + 19) / 20) ||
        opts->pass_stride > 1)
        return rtamd::fail(RT_E_INVALID, "multi-device rt_render renders the whole frame (pass_begin 0, all passes)");
    std::unique_ptr<rt_multi> m(new rt_multi());
    m->loopback = loopback_requested();
    std::vector<int> devs;
    if (int rc = device_list(opts, m->loopback, devs)) return rc;
    const int world = m->world = opts->device_count;
    m->P = (scene->ray_count + 19) / 20;
    m->px3 = (size_t)scene->width * scene->height * 3;
    m->sl = (m->px3 + world - 1) / world;            // floats per owner slice (last one padded)
    m->pitch = m->sl * world;                        // pass buffer rows padded to N equal slices
    // Pass buffers for all of a frame's rounds, up to 16 GB (buf + recv; 1080p: 320 rounds); the cap depends
    // only on the frame and the image, so it is the same on every device.  RTAMD_XCHG_CHUNK forces fewer
    // (the tests' multi-call cases).
    const int R = (m->P + world - 1) / world;
    const size_t round_bytes = m->pitch * sizeof(float) * 2;
    m->chunk_cap = std::max(1, std::min<int>(R, (int)std::min<size_t>((size_t)1 << 30, ((size_t)16 << 30) / round_bytes)));
    if (const char *ce = std::getenv("RTAMD_XCHG_CHUNK")) m->chunk_cap = std::max(1, std::min(m->chunk_cap, std::atoi(ce)));
    const char *mev = std::getenv("RTAMD_MULTI_EVENTS");
    m->events = mev && std::atoi(mev) != 0;
    m->comms.assign(world, nullptr);
#ifdef RTAMD_TEST_HOOKS
    if (m->loopback) {
        m->lb.reset(new Loopback());
        if (int rc = m->lb->init(devs)) return rc;
    }
#endif
    if (!m->loopback) {
        const ncclResult_t r = ncclCommInitAll(m->comms.data(), world, devs.data());
        if (r != ncclSuccess) {
            m->comms.clear();
            return rtamd::fail(RT_E_HIP, std::string("Error ncclCommInitAll ") + nccl_str(r));
        }
    }
    m->links.assign(world, Link{});
    for (int k = 0; k < world; k++) m->links[k].comm = m->comms[k];
    m->dev.assign(world, MDev{});
    // Per device, in parallel: the exchange buffers first (so that the renderer sizes its pass contexts on the
    // memory that is left), then the renderer.  No collective runs here, so a failure needs no abort.
    std::vector<std::thread> th;
    for (int k = 0; k < world; k++) {
        MDev &d = m->dev[k];
        d.device = devs[k];
        d.rank = k;
        const bool identity_only = world == 1 && !m->loopback;
        th.emplace_back([&m, &d, scene, opts, identity_only]() {
            auto body = [&]() -> int {
                MHIP(hipSetDevice(d.device));
                const size_t rows = (size_t)m->chunk_cap * m->pitch * sizeof(float);
                MHIP(hipMalloc(reinterpret_cast<void **>(&d.buf), rows));
                // recv: skipped only where the exchange is always the identity (one device, RTAMD_XCHG_IDENTITY
                // read per run: keep it when that may turn the exchange on)
                const char *ide = std::getenv("RTAMD_XCHG_IDENTITY");
                if (!identity_only || (ide && std::atoi(ide) == 0)) MHIP(hipMalloc(reinterpret_cast<void **>(&d.recv), rows));
                MHIP(hipMalloc(reinterpret_cast<void **>(&d.slice), (d.rank == 0 ? m->pitch : m->sl) * sizeof(float)));
                MHIP(hipMalloc(reinterpret_cast<void **>(&d.one), sizeof(int)));
                MHIP(hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking));
                MHIP(hipMemsetAsync(d.buf, 0, rows, d.s));   // row padding stays 0
                if (d.recv) MHIP(hipMemsetAsync(d.recv, 0, rows, d.s));
                const int one = 1;
                MHIP(hipMemcpyAsync(d.one, &one, sizeof(int), hipMemcpyHostToDevice, d.s));
                MHIP(hipStreamSynchronize(d.s));
                rt_opts o = *opts;
                o.device = d.device;
                o.device_count = 0;
                o.device_ids = nullptr;
                o.pass_begin = 0;
                o.pass_count = -1;
                o.pass_stride = 1;
                o.tile_count = 0;
                // Passes in flight next to RCCL: each pass's stream needs a hardware queue of its own -- two
                // streams on one in-order queue run their passes one after the other -- and the communicator's
                // streams take queues too (one-GPU probe, 26 passes: 7.07 ms/pass at 16 in flight, 7.50 at 20;
                // DESIGN §7).  bench.py's torch.distributed path uses the same 16.
                int rc = rtamd_renderer_create_inflight(scene, &o, &d.ren, kInflightNextToRccl);
                if (rc) return rc;
                // the owners add the pass slices themselves: no framebuffer add chain across the pass streams
                if ((rc = rt_renderer_set_accumulate(d.ren, 0))) return rc;
                // no per-bounce HIP events (four marker packets per bounce in every pass's stream, ~2 %), as in
                // bench.py's timed steps (rt_multi_set_event_timing / RTAMD_MULTI_EVENTS=1 turn them on)
                return rt_renderer_set_event_timing(d.ren, m->events);
            };
            d.rc = body();
            if (d.rc) d.err = rt_last_error();
        });
    }
    for (auto &t : th) t.join();
    if (int rc = first_error(m->dev)) return rc;
    // Every communicator rank answers: one in-place ncclAllReduce of a 1 per device (the loopback transport
    // has no communicator: its device count stands in).
    if (m->loopback) {
        m->ranks_seen = world;
    } else {
        ncclResult_t r = ncclGroupStart();
        for (int k = 0; k < world && r == ncclSuccess; k++) {
            if (hipSetDevice(m->dev[k].device) != hipSuccess) return rtamd::fail(RT_E_HIP, "hipSetDevice failed");
            r = ncclAllReduce(m->dev[k].one, m->dev[k].one, 1, ncclInt32, ncclSum, m->comms[k], m->dev[k].s);
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r != ncclSuccess || e != ncclSuccess)
            return rtamd::fail(RT_E_HIP, std::string("Error ncclAllReduce (rank count) ") + nccl_str(r != ncclSuccess ? r : e));
        int seen = 0;
        for (int k = 0; k < world; k++) {
            MDev &d = m->dev[k];
            MHIP(hipSetDevice(d.device));
            MHIP(hipMemcpyAsync(&seen, d.one, sizeof(int), hipMemcpyDeviceToHost, d.s));
            MHIP(hipStreamSynchronize(d.s));
            if (k == 0) m->ranks_seen = seen;
            if (seen != world)
                return rtamd::fail(RT_E_HIP, "rt_multi: the communicator counted " + std::to_string(seen) + " of " +
                                                 std::to_string(world) + " devices");
        }
    }
    *out = m.release();
    return RT_OK;
}

int rt_multi_run(rt_multi *m, int32_t pass_count, float *fb_out, rt_stats *stats) {
    using clk = std::chrono::high_resolution_clock;
    const auto w0 = clk::now();
    if (!m) return rtamd::fail(RT_E_INVALID, "null rt_multi");
    if (m->broken) return rtamd::fail(RT_E_INVALID, "rt_multi: an earlier run failed on a device (destroy and recreate)");
    if (pass_count < -1 || pass_count > m->P)
        return rtamd::fail(RT_E_INVALID, "rt_multi_run: pass_count outside [-1, passes of the frame]");
    const int np = pass_count < 0 ? m->P : pass_count;
    const int world = m->world;
    Sync sy;
    sy.world = world;
    for (auto &l : m->links) l.sy = &sy;
    if (m->lb) m->lb->reset();
    std::vector<std::thread> th;
    for (int k = 0; k < world; k++) {
        MDev &d = m->dev[k];
        d.rc = 0;
        d.err.clear();
        th.emplace_back([m, &d, &sy, np, fb_out, k]() {
            d.rc = run_device(*m, d, m->links[k], sy, np, fb_out);
            if (d.rc) d.err = rt_last_error();
        });
    }
    for (auto &t : th) t.join();
    for (auto &l : m->links) l.sy = nullptr;
    bool any = false;
    for (auto &d : m->dev) any = any || d.rc;
    if (any) {
        // collectives may have been aborted mid-run: the communicators are not reused
        m->broken = sy.failed.load() || std::any_of(m->links.begin(), m->links.end(), [](const Link &l) { return l.aborted; });
        return first_error(m->dev);
    }
    if (stats) {
        total_stats(stats, m->dev);
        stats->render_ms = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    }
    return RT_OK;
}

int rt_multi_read_framebuffer(rt_multi *m, float *fb_out) {
    if (!m || !fb_out) return rtamd::fail(RT_E_INVALID, "null argument");
    if (m->broken) return rtamd::fail(RT_E_INVALID, "rt_multi: an earlier run failed on a device");
    MDev &d = m->dev[0];
    MHIP(hipSetDevice(d.device));
    MHIP(hipMemcpyAsync(fb_out, d.slice, m->px3 * sizeof(float), hipMemcpyDeviceToHost, d.s));
    MHIP(hipStreamSynchronize(d.s));
    return RT_OK;
}

int rt_multi_set_event_timing(rt_multi *m, int32_t enable) {
    if (!m) return rtamd::fail(RT_E_INVALID, "null rt_multi");
    for (auto &d : m->dev)
        if (int rc = rt_renderer_set_event_timing(d.ren, enable)) return rc;
    m->events = enable != 0;
    return RT_OK;
}

int rt_multi_set_counters(rt_multi *m, int32_t enable) {
    if (!m) return rtamd::fail(RT_E_INVALID, "null rt_multi");
    for (auto &d : m->dev)
        if (int rc = rt_renderer_set_counters(d.ren, enable)) return rc;
    return RT_OK;
}

int rt_multi_ranks(const rt_multi *m) { return m ? m->ranks_seen : 0; }

void rt_multi_destroy(rt_multi *m) { delete m; }

}  // extern "C"

// rt_render with device_count >= 1: the persistent multi-device renderer used once (pass sharding), or the
// one-shot pixel-tile render.
int rtamd_render_multi(const rt_scene *scene, const rt_opts *opts, float *fb_out, rt_stats *stats) {
    using clk = std::chrono::high_resolution_clock;
    const auto w0 = clk::now();
    if (opts->shard_tiles) return render_tiles(scene, opts, fb_out, stats);
    rt_multi *m = nullptr;
    int rc = rt_multi_create(scene, opts, &m);
    if (rc) return rc;
    rc = rt_multi_run(m, -1, fb_out, stats);
    rt_multi_destroy(m);
    if (!rc && stats) stats->render_ms = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    return rc;
}
