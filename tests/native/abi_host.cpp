// abi_host.cpp — a C++ host of librtamd.so bound the way the reference's own main would bind the
// drop-in (load_scene -> rt_scene_load, gpu_raytrace -> rt_render), with nothing
// set in the environment: no GPU_MAX_HW_QUEUES, no RTAMD_* knob.  It checks that the library is fast
// without the host's help (the library's constructor asks HIP for the hardware queues its pass
// streams need; rt_abi.h) and writes pass 0's framebuffer for the image check.
//
//   abi_host <scene> <asset_root> W H spp bounces passes reps <pass0_fb.bin>
//
// stdout: one JSON line per rt_render of `passes` passes (reps of them; each creates and frees its
// renderer like gpu_raytrace, raytracing.cu:170-284), then one for the pass-0 render.
#include "rt_abi.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
    if (argc < 10) {
        std::fprintf(stderr, "usage: %s scene asset_root W H spp bounces passes reps pass0_fb.bin\n", argv[0]);
        return 1;
    }
    rt_load_opts lo;
    rt_default_load_opts(&lo);
    lo.quiet = 1;
    lo.asset_root = argv[2];
    lo.image_override = 1;
    lo.width = std::atoi(argv[3]);
    lo.height = std::atoi(argv[4]);
    lo.ray_count = std::atoi(argv[5]);
    lo.bounces = std::atoi(argv[6]);
    const int passes = std::atoi(argv[7]), reps = std::atoi(argv[8]);
    rt_scene_host *h = nullptr;
    if (rt_scene_load(argv[1], &lo, &h)) {
        std::printf("Error rt_scene_load %s\n", rt_last_error());
        return 1;
    }
    const rt_scene *s = rt_scene_view(h);
    std::vector<float> fb((size_t)s->width * s->height * 3);
    const char *q = std::getenv("GPU_MAX_HW_QUEUES");   // as the library's constructor left it
    for (int rep = 0; rep < reps; rep++) {
        rt_opts o;
        rt_default_opts(&o);
        o.pass_count = passes;
        rt_stats st;
        if (rt_render(s, &o, fb.data(), &st)) {
            std::printf("Error rt_render %s\n", rt_last_error());
            return 1;
        }
        std::printf("{\"rep\": %d, \"passes\": %u, \"render_ms\": %.3f, \"kernel_ms\": %.3f, \"ms_per_pass\": %.4f, "
                    "\"live_segments\": %llu, \"gpu_max_hw_queues\": \"%s\"}\n",
                    rep, st.passes, st.render_ms, st.kernel_ms, st.kernel_ms / st.passes,
                    (unsigned long long)st.live_segments, q ? q : "unset");
        std::fflush(stdout);
    }
    // the same passes on one persistent renderer, three runs back to back (what a host rendering several frames
    // would do): the first run pays what a fresh renderer pays, the later ones show the steady state
    {
        rt_opts o;
        rt_default_opts(&o);
        rt_renderer *r = nullptr;
        if (rt_renderer_create(s, &o, &r) || rt_renderer_set_event_timing(r, 0)) {
            std::printf("Error rt_renderer_create %s\n", rt_last_error());
            return 1;
        }
        for (int k = 0; k < 3; k++) {
            rt_stats st;
            if (rt_renderer_run(r, 0, passes, 1, nullptr, &st)) {
                std::printf("Error rt_renderer_run %s\n", rt_last_error());
                return 1;
            }
            std::printf("{\"persistent_run\": %d, \"passes\": %u, \"kernel_ms\": %.3f, \"ms_per_pass\": %.4f}\n", k,
                        st.passes, st.kernel_ms, st.kernel_ms / st.passes);
            std::fflush(stdout);
        }
        rt_renderer_destroy(r);
    }
    rt_opts o;
    rt_default_opts(&o);
    o.pass_count = 1;
    rt_stats st;
    if (rt_render(s, &o, fb.data(), &st)) {
        std::printf("Error rt_render %s\n", rt_last_error());
        return 1;
    }
    FILE *f = std::fopen(argv[9], "wb");
    if (!f || std::fwrite(fb.data(), sizeof(float), fb.size(), f) != fb.size()) return 1;
    std::fclose(f);
    std::printf("{\"pass0\": true, \"live_segments\": %llu}\n", (unsigned long long)st.live_segments);
    rt_scene_free(h);
    return 0;
}
