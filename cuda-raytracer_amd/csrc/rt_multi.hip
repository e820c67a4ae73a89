// rt_multi.hip — multi-GPU rt_render in one process: pass sharding over the devices of one node,
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
//     After a chunk of rounds, one ncclAllToAll per round sends slice j of each pass buffer to
//     device j (each xGMI link carries 1/N of the data; nothing converges on one GPU), and device
//     j adds the slices it received in pass order, fb_j = ((0 + S_0,j) + S_1,j) + ..., exactly
//     the per-pixel add sequence of one device: the N-device image is bit-identical to the
//     1-device image with sort on or off.
//   * One ncclGather of the N finished slices to device_ids[0], then one D2H copy to fb_out.
//
// Exchange bytes per frame: every pass buffer leaves its device except its own slice,
// P * W*H*3*4 * (N-1)/N in all (1080p teapot, N = 8: 103 passes x 24.9 MB x 7/8 = 2.24 GB over the
// job, ~280 MB per device, 1/7 of it per link), plus the gather's W*H*3*4 * (N-1)/N into device 0.
// One host thread per device (RCCL's one-thread-per-device model for a single-process
// communicator); device_count = 1 runs the same code with every exchange local.
//
// rt_opts.shard_tiles = 1 deals pixel tiles instead (§8e's natural shard): device k renders owner
// k's row stripes of every pass; with sort on the owners all-reduce one byte per global live ray
// after every bounce but the last (nccl_exchange), and the frame is an ncclReduce of the owners'
// framebuffers.
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

struct DevState {
    int device = 0, rank = 0;
    int rc = 0;
    std::string err;
    rt_stats stats{};
    double exchange_ms = 0;
};

// Test transport (RTAMD_MULTI_LOOPBACK=1): the "devices" are host threads on ONE GPU (device_ids may repeat),
// and run_device's two collectives become device-to-device copies between the threads' buffers, ordered through
// events the threads swap at host barriers.  It exists so that the multi-device schedule -- pass dealing, the
// stale rows of rounds a device has no pass in, the owners' ordered adds, the gather -- runs at N > 1 on a
// one-GPU box (RCCL refuses two ranks on one GPU); the product path is RCCL.  No abort handling: tests only.
struct Loopback {
    int world = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<hipEvent_t> ev_in, ev_out;    // per rank, re-recorded at every collective
    std::vector<float *> send, recv;          // per rank: the current collective's buffers
    void barrier() {
        std::unique_lock<std::mutex> l(m);
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g; });
        }
    }
    // entry: every rank's stream waits for every rank's work so far; exit: for every rank's copies
    int fence(std::vector<hipEvent_t> &ev, int rank, hipStream_t s) {
        if (hipEventRecord(ev[rank], s) != hipSuccess) return RT_E_HIP;
        barrier();
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

void add_stats(DevState &st, const rt_stats &s) {
    st.stats.live_segments += s.live_segments;
    st.stats.generated_rays += s.generated_rays;
    st.stats.sorted_items += s.sorted_items;
    st.stats.nodes_popped += s.nodes_popped;
    st.stats.internal_visits += s.internal_visits;
    st.stats.triangle_tests += s.triangle_tests;
    st.stats.sphere_tests += s.sphere_tests;
    st.stats.hits += s.hits;
    st.stats.misses += s.misses;
    st.stats.hits_sphere += s.hits_sphere;
    st.stats.dead_slots += s.dead_slots;
    st.stats.passes += s.passes;
    st.stats.kernel_ms += s.kernel_ms;
    st.stats.process_ms += s.process_ms;
    st.stats.sort_ms += s.sort_ms;
    st.stats.trace_ms += s.trace_ms;
    st.stats.trace_launches += s.trace_launches;
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

// Test hook: RTAMD_FAIL_AFTER_SETUP=<rank> makes that device fail right after the setup barrier, the
// path where its peers must not be left inside a collective.
bool injected_failure(int rank) {
    const char *e = std::getenv("RTAMD_FAIL_AFTER_SETUP");
    return e && *e && std::atoi(e) == rank;
}

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

// Device `st.rank`'s share of the frame: render, exchange, add; the root also gathers.
int run_device(const rt_scene *scene, const rt_opts *base, Link &ln, int world, DevState &st, float *fb_out,
               Sync &sy, Loopback *lb) {
    RunGuard run{sy, ln};
    ncclComm_t comm = ln.comm;
    MHIP(hipSetDevice(st.device));
    const int P = (scene->ray_count + 19) / 20;
    const size_t px3 = (size_t)scene->width * scene->height * 3;
    const size_t sl = (px3 + world - 1) / world;      // floats per owner slice (last one padded)
    const size_t pitch = sl * world;                  // pass buffer rows padded to N equal slices
    const int R = (P + world - 1) / world;            // rounds: one pass per device each
    // One device: the all-to-all and the gather are the identity (every slice is its own), so they are skipped
    // and the adds read buf directly, as the torch.distributed path does at N = 1.  RTAMD_XCHG_IDENTITY=0 runs
    // them through RCCL anyway (the N = 1 tests keep the collectives exercised).
    const char *ide = std::getenv("RTAMD_XCHG_IDENTITY");
    const bool identity = world == 1 && !lb && (!ide || std::atoi(ide) != 0);
    // Rounds per renderer call: all of them, so that the renderer keeps its passes in flight across the whole
    // share (between calls it drains: a 26-pass share ran 6.40 ms/pass in calls of 16 passes against 5.91 for
    // one plain run), up to 16 GB of pass buffers (buf + recv: 1080p, 320 rounds).  The chunk must be the same
    // on every device (it fixes the collective sequence): it depends only on R and the image size.
    // RTAMD_XCHG_CHUNK forces a smaller one (the tests' multi-call cases).
    const size_t round_bytes = pitch * sizeof(float) * 2;
    int chunk = std::max(1, std::min<int>(R, (int)std::min<size_t>((size_t)1 << 30, ((size_t)16 << 30) / round_bytes)));
    if (const char *ce = std::getenv("RTAMD_XCHG_CHUNK")) chunk = std::max(1, std::min(chunk, std::atoi(ce)));
    rt_opts o = *base;
    o.device = st.device;
    o.device_count = 0;
    o.device_ids = nullptr;
    o.pass_begin = 0;
    o.pass_count = -1;
    o.pass_stride = 1;
    o.tile_count = 0;
    rt_renderer *ren = nullptr;
    // Passes in flight next to RCCL: each pass's stream needs a hardware queue of its own -- two
    // streams on one in-order queue run their passes one after the other -- and the communicator's
    // streams take queues too (one-GPU probe, 26 passes: 7.07 ms/pass at 16 in flight, 7.50 at 20;
    // DESIGN §7).  bench.py's torch.distributed path uses the same 16.
    int rc = rtamd_renderer_create_inflight(scene, &o, &ren, kInflightNextToRccl);
    if (rc) return rc;
    struct Guard {
        rt_renderer *r;
        RunGuard &run;
        float *bufs[3] = {nullptr, nullptr, nullptr};
        hipStream_t s = nullptr;
        ~Guard() {
            run.fail_now();
            for (float *b : bufs)
                if (b) (void)hipFree(b);
            if (s) (void)hipStreamDestroy(s);
            rt_renderer_destroy(r);
        }
    } g{ren, run};
    // the owners add the pass slices themselves: no framebuffer add chain across the pass streams
    rc = rt_renderer_set_accumulate(ren, 0);
    if (rc) return rc;
    // no per-bounce HIP events (four marker packets per bounce in every pass's stream, ~2 %), as in bench.py's
    // timed steps: the multi-device stats carry no process_ms / sort_ms / trace_ms (RTAMD_MULTI_EVENTS=1 keeps them)
    const char *mev = std::getenv("RTAMD_MULTI_EVENTS");
    rc = rt_renderer_set_event_timing(ren, mev && std::atoi(mev) != 0);
    if (rc) return rc;
    float *&buf = g.bufs[0], *&recv = g.bufs[1], *&slice = g.bufs[2];
    MHIP(hipMalloc(reinterpret_cast<void **>(&buf), (size_t)chunk * pitch * sizeof(float)));
    if (!identity) MHIP(hipMalloc(reinterpret_cast<void **>(&recv), (size_t)chunk * pitch * sizeof(float)));
    MHIP(hipMalloc(reinterpret_cast<void **>(&slice), (st.rank == 0 ? pitch : sl) * sizeof(float)));
    MHIP(hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking));
    MHIP(hipMemsetAsync(buf, 0, (size_t)chunk * pitch * sizeof(float), g.s));   // padding stays 0
    MHIP(hipMemsetAsync(slice, 0, sl * sizeof(float), g.s));
    MHIP(hipStreamSynchronize(g.s));
    if (!run.setup()) return rtamd::fail(RT_E_INVALID, "another device of the render failed");
    if (injected_failure(st.rank)) return rtamd::fail(RT_E_INVALID, "injected failure (RTAMD_FAIL_AFTER_SETUP)");
    using clk = std::chrono::high_resolution_clock;
    const auto loop0 = clk::now();
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
    for (int k0 = 0; k0 < R; k0 += chunk) {
        const int m = std::min(chunk, R - k0);
        // this device's passes of rounds k0 .. k0+m-1
        const int first = st.rank + world * k0;
        const int mine = first < P ? std::min(m, (P - 1 - first) / world + 1) : 0;
        if (mine > 0 && overlap) {
            rc = rtamd_renderer_run_async_pitched(ren, first, mine, world, buf, pitch);
            if (rc) return rc;
        }
        if (mine > 0 && !overlap) {
            rt_stats s{};
            rc = rtamd_renderer_run_pitched(ren, first, mine, world, buf, pitch, &s);
            if (rc) return rc;
            add_stats(st, s);
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
        const bool gtime = std::getenv("RTAMD_TIMING") != nullptr;
        auto gmark = [&]() -> int {
            if (!gtime) return RT_OK;
            gev.push_back(nullptr);
            MHIP(hipEventCreate(&gev.back()));
            MHIP(hipEventRecord(gev.back(), g.s));
            return RT_OK;
        };
        if (int rc_ = gmark()) return rc_;
        for (int j0 = 0; j0 < m; j0 += xr) {
            const int j1 = std::min(m, j0 + xr);
            if (overlap)
                for (int j = j0; j < std::min(j1, mine); j++) {
                    rc = rt_renderer_wait_pass(ren, j, g.s);
                    if (rc) return rc;
                }
            if (int rc_ = gmark()) return rc_;     // the group's passes are done
            if (identity) {
            } else if (lb) {
                if (int rc2 = lb->alltoall(st.rank, buf, recv, j0, j1, pitch, sl, g.s))
                    return rtamd::fail(rc2, "loopback exchange failed");
            } else {
                MNCCL(ncclGroupStart());
                for (int j = j0; j < j1; j++)
                    MNCCL(ncclAllToAll(buf + (size_t)j * pitch, recv + (size_t)j * pitch, sl, ncclFloat32, comm, g.s));
                MNCCL(ncclGroupEnd());
            }
            hipLaunchKernelGGL(add_slices_kernel, dim3((unsigned)((sl + 255) / 256)), dim3(256), 0, g.s, slice,
                               (identity ? buf : recv) + (size_t)j0 * pitch, sl, world, j1 - j0, k0 + j0, P);
            MHIP(hipGetLastError());
            if (int rc_ = gmark()) return rc_;     // its adds are done
        }
        if (mine > 0 && overlap) {
            // the passes render on the renderer's own streams, which no collective waits behind:
            // this wait ends even if a peer device has failed
            rt_stats s{};
            rc = rt_renderer_finish(ren, &s);
            if (rc) return rc;
            add_stats(st, s);
            t0 = clk::now();            // exchange_ms: what the render did not hide
        }
        // the next chunk's render overwrites buf: the exchange must have read it
        const auto tf = clk::now();
        MWAIT(g.s);
        st.exchange_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (gtime) {
            std::string line;
            for (size_t k = 1; k < gev.size(); k++) {
                float ms = 0;
                MHIP(hipEventElapsedTime(&ms, gev[0], gev[k]));
                line += (k % 2 ? " ready " : " added ") + std::to_string(ms);
            }
            std::fprintf(stderr, "rt_multi device %d chunk at round %d: exchange groups (ms after the chunk's enqueue):%s; "
                         "host wait after the render %.2f ms\n", st.rank, k0, line.c_str(),
                         std::chrono::duration<double, std::milli>(clk::now() - tf).count());
        }
    }
    const double loop_ms = std::chrono::duration<double, std::milli>(clk::now() - loop0).count();
    const double unhidden_ms = st.exchange_ms;
    const auto t0 = clk::now();
    // gather the finished slices to the root (in place: the root's own slice is block 0)
    if (lb) {
        if (int rc2 = lb->gather(st.rank, slice, sl, g.s)) return rtamd::fail(rc2, "loopback gather failed");
    } else if (!identity) {
        MNCCL(ncclGather(slice, slice, sl, ncclFloat32, 0, comm, g.s));
    }
    if (st.rank == 0) MHIP(hipMemcpyAsync(fb_out, slice, px3 * sizeof(float), hipMemcpyDeviceToHost, g.s));
    MWAIT(g.s);
    st.exchange_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (std::getenv("RTAMD_TIMING"))
        std::fprintf(stderr, "rt_multi device %d: %d passes rendered and exchanged in %.2f ms (exchange not hidden: %.2f ms, "
                     "%s), then gather + framebuffer to the host %.2f ms\n", st.rank, (int)st.stats.passes, loop_ms,
                     unhidden_ms, overlap ? "overlapped" : "after each chunk",
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

// Device `st.rank`'s tiles: owner rank's tile_rows-row stripes of every pass, then an
// ncclReduce of the owners' framebuffers to the root: every pixel has one owner and is 0 elsewhere,
// so the sum is that owner's value bit for bit (x + 0 = x).
int run_device_tiles(const rt_scene *scene, const rt_opts *base, Link &ln, int world, DevState &st,
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
    if (injected_failure(st.rank)) return rtamd::fail(RT_E_INVALID, "injected failure (RTAMD_FAIL_AFTER_SETUP)");
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

}  // namespace

int rtamd_render_multi(const rt_scene *scene, const rt_opts *opts, float *fb_out, rt_stats *stats) {
    using clk = std::chrono::high_resolution_clock;
    const auto w0 = clk::now();
    const int world = opts->device_count;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    const bool loopback = loopback_requested();
    if (loopback && opts->shard_tiles)
        return rtamd::fail(RT_E_INVALID, "RTAMD_MULTI_LOOPBACK covers pass sharding only (not shard_tiles)");
    std::vector<int> devs(world);
    for (int k = 0; k < world; k++) {
        devs[k] = opts->device_ids ? opts->device_ids[k] : (loopback ? 0 : k);
        if (devs[k] < 0 || devs[k] >= ndev) return rtamd::fail(RT_E_NODEVICE, "device_ids: no such HIP device");
        for (int j = 0; j < k && !loopback; j++)
            if (devs[j] == devs[k]) return rtamd::fail(RT_E_INVALID, "device_ids: a device is listed twice");
    }
    if (opts->tile_count > 1) return rtamd::fail(RT_E_INVALID, "device_count and tile_count are exclusive "
                                                              "(shard_tiles = 1 deals the tiles over the devices)");
    if (opts->pass_begin != 0 || (opts->pass_count != -1 && opts->pass_count != (scene->ray_count + 19) / 20) ||
        opts->pass_stride > 1)
        return rtamd::fail(RT_E_INVALID, "multi-device rt_render renders the whole frame (pass_begin 0, all passes)");
    std::vector<ncclComm_t> comms(world, nullptr);
    Loopback lb;
    struct LbEvents {
        Loopback &lb;
        ~LbEvents() {
            for (auto e : lb.ev_in) if (e) (void)hipEventDestroy(e);
            for (auto e : lb.ev_out) if (e) (void)hipEventDestroy(e);
        }
    } lb_events{lb};
    if (loopback) {
        lb.world = world;
        lb.send.assign(world, nullptr);
        lb.recv.assign(world, nullptr);
        lb.ev_in.assign(world, nullptr);
        lb.ev_out.assign(world, nullptr);
        for (int k = 0; k < world; k++)
            if (hipSetDevice(devs[k]) != hipSuccess ||
                hipEventCreateWithFlags(&lb.ev_in[k], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&lb.ev_out[k], hipEventDisableTiming) != hipSuccess)
                return rtamd::fail(RT_E_HIP, "loopback: hipEventCreate failed");
    } else {
        const ncclResult_t r = ncclCommInitAll(comms.data(), world, devs.data());
        if (r != ncclSuccess) return rtamd::fail(RT_E_HIP, std::string("Error ncclCommInitAll ") + nccl_str(r));
    }
    std::vector<DevState> st(world);
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
            st[k].rc = opts->shard_tiles ? run_device_tiles(scene, opts, links[k], world, st[k], fb_out, sy)
                                         : run_device(scene, opts, links[k], world, st[k], fb_out, sy,
                                                      loopback ? &lb : nullptr);
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
        std::memset(stats, 0, sizeof(*stats));
        for (auto &s : st) {
            const rt_stats &x = s.stats;
            stats->generated_rays += x.generated_rays;
            stats->live_segments += x.live_segments;
            stats->sorted_items += x.sorted_items;
            stats->nodes_popped += x.nodes_popped;
            stats->internal_visits += x.internal_visits;
            stats->triangle_tests += x.triangle_tests;
            stats->sphere_tests += x.sphere_tests;
            stats->hits += x.hits;
            stats->misses += x.misses;
            stats->hits_sphere += x.hits_sphere;
            stats->dead_slots += x.dead_slots;
            stats->passes += x.passes;
            stats->process_ms += x.process_ms;
            stats->sort_ms += x.sort_ms;
            stats->trace_ms += x.trace_ms;
            stats->trace_launches += x.trace_launches;
            stats->kernel_ms = std::max(stats->kernel_ms, x.kernel_ms);
            stats->exchange_ms = std::max(stats->exchange_ms, s.exchange_ms);
        }
        stats->render_ms = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    }
    return RT_OK;
}
