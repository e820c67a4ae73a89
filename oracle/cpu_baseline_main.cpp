// cpu_baseline_main.cpp — TEST INFRASTRUCTURE ONLY: times the oracle's restatement of the
// reference `cpu` path (raytracing.cu:122-163) for bench.py's cpu_baseline leg.  Built with the
// reference's host flags (-O3 -ffast-math -fopenmp, build.sh:2) in its own process, so the
// fast-math FTZ mode never leaks into the strict parity oracle.
//   cpu_baseline <scene> <asset_root> <W> <H> <spp> <bounces> <pass_limit> <threads>
#include "oracle.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

int main(int argc, char **argv) {
    if (argc < 9) {
        std::printf("usage: %s scene asset_root W H spp bounces pass_limit threads\n", argv[0]);
        return 1;
    }
    const int32_t image[4] = {std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6])};
    const int pass_limit = std::atoi(argv[7]);
    int threads = std::atoi(argv[8]);
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#endif
    orc_scene *s = orc_load_scene(argv[1], 1, argv[2], image, nullptr);
    if (!s) { std::printf("Error %s\n", orc_last_error()); return 1; }
    orc_info info;
    orc_get_info(s, &info);
    std::vector<float> fb((size_t)info.width * info.height * 3);
    double secs = 0;
    uint64_t live = 0;
    const int passes = orc_render_cpu_path_counted(s, fb.data(), pass_limit, threads, &secs, &live);
    double mean = 0;
    for (float v : fb) mean += v;
    mean /= fb.size();
    std::printf("CPU Took %gs\n", secs);
    std::printf("{\"seconds\": %.6f, \"passes\": %d, \"threads\": %d, \"width\": %d, \"height\": %d, "
                "\"spp\": %d, \"bounces\": %d, \"live_segments\": %llu, \"fb_mean\": %.6g}\n",
                secs, passes, threads, info.width, info.height, info.ray_count, info.bounces,
                (unsigned long long)live, mean);
    orc_free_scene(s);
    return 0;
}
