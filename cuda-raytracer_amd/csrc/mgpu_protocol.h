// mgpu_protocol.h — the multi-device abort protocol of rt_multi.hip, free of HIP and RCCL types so
// that it can be tested on the CPU (tests/native/mgpu_protocol_test.cpp, tests/test_mgpu_protocol.py).
//
// A device that fails must not leave its peers blocked in a collective.  Every device first builds
// its renderer and buffers (where nearly every failure happens: out of memory, a bad scene) and
// meets the others; if any failed, all return before the first collective.  A failure after that
// sets `failed`; every device aborts only its OWN communicator (its thread is the only one that
// uses it, so no call can race the abort), when it fails itself or when it sees the flag: before
// each collective and while it polls a stream or event that waits on one.  The aborted
// communicator's pending work ends, and its peers' polls see the flag and abort theirs.
#pragma once
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "rt_abi.h"

namespace rtamd_mgpu {

struct Sync {
    std::mutex m;
    std::condition_variable cv;
    int world = 0, arrived = 0;
    bool setup_failed = false;
    std::atomic<bool> failed{false};
    bool setup_done(bool ok) {   // false if any device's setup failed
        std::unique_lock<std::mutex> l(m);
        if (!ok) setup_failed = true;
        if (++arrived == world) cv.notify_all();
        else cv.wait(l, [&] { return arrived == world; });
        return !setup_failed;
    }
};

// One device's communicator and its abort state (touched by that device's thread only).  Comm is
// the communicator handle, AbortFn aborts one (ncclCommAbort in the library).
template <class Comm, void (*AbortFn)(Comm)>
struct LinkT {
    Comm comm{};
    bool aborted = false;
    Sync *sy = nullptr;
    void abort() {
        if (!aborted && comm) AbortFn(comm);
        aborted = true;
    }
    // nonzero (and the communicator aborted) once any device has failed
    int check() {
        if (!sy->failed.load()) return 0;
        abort();
        return RT_E_INVALID;
    }
};

// Scope guard of one device's run: arrives at the setup barrier as failed if the run ends before
// setup(), and on an error after it raises the flag and aborts this device's communicator.
template <class Link>
struct RunGuardT {
    Sync &sy;
    Link &ln;
    bool arrived = false, ok = false;
    bool setup() {
        arrived = true;
        return sy.setup_done(true);
    }
    // an error after setup: raise the flag and abort this device's communicator now, before the
    // renderer and buffers are torn down (their teardown must not wait on a collective a peer is
    // still blocked in); called by the resource guards' destructors, and again (a no-op) at scope exit
    void fail_now() {
        if (arrived && !ok) {
            sy.failed = true;
            ln.abort();
        }
    }
    ~RunGuardT() {
        if (!arrived) (void)sy.setup_done(false);
        else fail_now();
    }
};

// Waits until query() reports completion while watching the other devices.  query() returns 0 when
// done, 1 while not ready, anything else on an error of its own.  kPeerFailed: another device
// failed (this device's communicator is aborted).
enum WaitResult { kDone = 0, kPeerFailed = 1, kOwnError = 2 };
template <class Query, class Link>
WaitResult wait_watching(Query query, Link &ln) {
    for (;;) {
        const int q = query();
        if (q == 0) return kDone;
        if (q != 1) return kOwnError;
        if (ln.check()) return kPeerFailed;
        std::this_thread::yield();
    }
}

}  // namespace rtamd_mgpu
