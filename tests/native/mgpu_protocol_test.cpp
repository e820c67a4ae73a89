// CPU test of the multi-device abort protocol (cuda-raytracer_amd/csrc/mgpu_protocol.h) that
// rt_multi.hip runs over RCCL: N device threads with fake communicators whose "collective" only
// completes when every device has entered it, or ends when the device's own communicator is
// aborted -- what a pending RCCL collective does.  Built and run by tests/test_mgpu_protocol.py.
//
//   scenario ok          every device completes its collectives; nothing is aborted
//   scenario setup R     device R fails before the setup barrier: every device returns before any
//                        collective; the others then abort their unused communicators at scope exit
//                        (rt_multi.hip skips ncclCommDestroy for those)
//   scenario after R     device R fails right after the barrier while the others are blocked in a
//                        collective that can never complete: all of them return, with an error,
//                        every communicator aborted (the case ADVICE r03 asked to exercise)
#include "mgpu_protocol.h"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct FakeComm {
    std::atomic<bool> aborted{false};
};
void fake_abort(FakeComm *c) { c->aborted = true; }
using Link = rtamd_mgpu::LinkT<FakeComm *, fake_abort>;
using RunGuard = rtamd_mgpu::RunGuardT<Link>;

// a collective all devices must enter: done once `entered` reaches the world size
struct Collective {
    std::atomic<int> entered{0};
};

int run_device(int rank, int world, int fail_rank, bool fail_before_setup, Link &ln, rtamd_mgpu::Sync &sy,
               Collective *colls, int ncoll) {
    RunGuard run{sy, ln};
    if (rank == fail_rank && fail_before_setup) return RT_E_OOM;   // e.g. out of memory building buffers
    if (!run.setup()) return RT_E_INVALID;                          // a peer failed: no collective at all
    if (rank == fail_rank) return RT_E_HIP;                          // fails after the barrier
    for (int k = 0; k < ncoll; k++) {
        if (ln.check()) return RT_E_INVALID;                         // MNCCL's check before each call
        colls[k].entered++;
        // the stream holding the collective: complete when all entered, error once aborted
        const rtamd_mgpu::WaitResult w = rtamd_mgpu::wait_watching([&] {
            if (ln.comm->aborted) return 2;                          // the aborted collective errors out
            return colls[k].entered.load() == world ? 0 : 1;
        }, ln);
        if (w == rtamd_mgpu::kOwnError) return RT_E_HIP;
        if (w == rtamd_mgpu::kPeerFailed) return RT_E_INVALID;
    }
    run.ok = true;
    return RT_OK;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s WORLD ok|setup|after [RANK]\n", argv[0]);
        return 2;
    }
    const int world = std::atoi(argv[1]);
    const std::string mode = argv[2];
    const int fail_rank = mode == "ok" ? -1 : std::atoi(argv[3]);
    rtamd_mgpu::Sync sy;
    sy.world = world;
    std::vector<FakeComm> comms(world);
    std::vector<Link> links(world);
    for (int r = 0; r < world; r++) {
        links[r].comm = &comms[r];
        links[r].sy = &sy;
    }
    const int ncoll = 3;
    Collective colls[ncoll];
    std::vector<int> rc(world, 12345);
    std::atomic<int> finished{0};
    std::vector<std::thread> th;
    for (int r = 0; r < world; r++)
        th.emplace_back([&, r] {
            rc[r] = run_device(r, world, fail_rank, mode == "setup", links[r], sy, colls, ncoll);
            finished++;
        });
    // every device must return: a thread left blocked in a collective is the failure this guards
    const auto t0 = std::chrono::steady_clock::now();
    while (finished.load() < world) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) {
            std::printf("HANG: %d of %d devices returned\n", finished.load(), world);
            std::fflush(stdout);
            std::_Exit(3);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    for (auto &t : th) t.join();
    int aborted = 0;
    for (auto &c : comms) aborted += c.aborted ? 1 : 0;
    std::printf("rc");
    for (int r = 0; r < world; r++) std::printf(" %d", rc[r]);
    int entered = 0;
    for (auto &c : colls) entered += c.entered.load();
    std::printf(" aborted %d failed %d entered %d\n", aborted, sy.failed.load() ? 1 : 0, entered);
    return 0;
}
