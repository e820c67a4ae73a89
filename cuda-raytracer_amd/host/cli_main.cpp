// cli_main.cpp — `raytracing`, the drop-in for the reference executable (raytracing.cu:305-398).
//
//   raytracing <scene file> [no_sort] [cpu] [no_gpu] [no_bvh]
//              [--image W H spp bounces exposure] [--devices N] [--device K]
//              [--asset-root DIR] [--out FILE] [--stats FILE] [--gpu-bvh]
//
// Reference behaviour kept: usage line + exit 1 without a scene, "No raytracing hardware
// specified" + exit 2 for no_gpu without cpu, unknown words ignored, asset paths relative to
// the CWD, the same stdout lines, CPU image stacked above the GPU image, output
// raytracing.png.  Added: the --options above (all optional).  --devices N renders whole
// 20-spp passes round-robin on GPUs 0..N-1 inside the library (rt_opts.device_count: one
// RCCL communicator, pass-sum slices exchanged over xGMI and added in pass order by their
// owner, then gathered to GPU 0), so the image is identical to the 1-GPU image.
#include "rt_abi.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

namespace {

int die(const char *what) {
    std::printf("Error %s %s\n", what, rt_last_error());
    return 1;
}

}  // namespace

int main(int argc, char **argv) {
    // Up to 20 passes in flight per device on their own streams: give HIP enough hardware queues
    // (read when HIP initialises).
    if (const char *q = std::getenv("GPU_MAX_HW_QUEUES"); !q || std::atoi(q) < 24) setenv("GPU_MAX_HW_QUEUES", "24", 1);
    if (argc < 2) {
        std::printf("Usage: %s <scene>\n", argv[0]);
        return 1;
    }
    bool sort = true, cpu = false, gpu = true, bvh = true, gpu_bvh = false;
    int devices = 0, device = 0;          // devices 0: not given (the single device `device`)
    const char *asset_root = nullptr, *out_path = "raytracing.png", *stats_path = nullptr;
    rt_load_opts lo;
    rt_default_load_opts(&lo);
    for (int i = 2; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "no_sort") sort = false;
        else if (a == "cpu") cpu = true;
        else if (a == "no_bvh") bvh = false;
        else if (a == "no_gpu") gpu = false;
        else if (a == "--image" && i + 5 < argc) {
            lo.image_override = 1;
            lo.width = std::atoi(argv[++i]);
            lo.height = std::atoi(argv[++i]);
            lo.ray_count = std::atoi(argv[++i]);
            lo.bounces = std::atoi(argv[++i]);
            lo.exposure_override = 1;
            lo.exposure = (float)std::atof(argv[++i]);
        } else if (a == "--devices" && i + 1 < argc) devices = std::max(1, std::atoi(argv[++i]));
        else if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (a == "--asset-root" && i + 1 < argc) asset_root = argv[++i];
        else if (a == "--out" && i + 1 < argc) out_path = argv[++i];
        else if (a == "--stats" && i + 1 < argc) stats_path = argv[++i];
        else if (a == "--gpu-bvh") gpu_bvh = true;
        // unknown words are ignored, like the reference
    }
    if (!cpu && !gpu) {
        std::printf("No raytracing hardware specified\n");
        return 2;
    }
    // HIP runtime, queue and code-object initialisation (~0.2 s per process) runs on a thread of
    // its own while the scene loads and the BVH builds; the GPU Took span below starts before the
    // wait for it, so whatever is left of it is still counted.
    const auto t_start = std::chrono::high_resolution_clock::now();
    auto ms_since = [](std::chrono::high_resolution_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t).count();
    };
    const bool timing = std::getenv("RTAMD_TIMING") != nullptr;
    double warm_ms = 0;
    struct Warmup {
        std::thread t;
        ~Warmup() { if (t.joinable()) t.join(); }
    } warm;
    if (gpu)
        warm.t = std::thread([=, &warm_ms] {
            const auto w0 = std::chrono::high_resolution_clock::now();
            for (int k = 0; k < (devices > 0 ? devices : 1); k++) (void)rt_device_warmup(devices > 0 ? k : device);
            warm_ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - w0).count();
        });
    lo.use_bvh = bvh ? 1 : 0;
    lo.asset_root = asset_root;
    if (gpu_bvh) lo.bvh_device = device;          // GPU binned-SAH build, same node array
    rt_scene_host *host = nullptr;
    if (rt_scene_load(argv[1], &lo, &host)) return die("load_scene");
    const rt_scene *s = rt_scene_view(host);
    const size_t px3 = (size_t)s->width * s->height * 3;
    std::vector<uint8_t> image;
    std::vector<float> fb(px3);
    rt_stats gst{};
    double cpu_s = 0;
    if (cpu) {
        if (rt_cpu_render(s, fb.data(), 0, &cpu_s) < 0) return die("cpu_raytrace");
        std::printf("CPU Took %gs\n", cpu_s);
        std::vector<uint8_t> part(px3);
        rt_tonemap(fb.data(), s->width, s->height, s->exposure, s->ray_count, part.data());
        image.insert(image.end(), part.begin(), part.end());
    }
    if (gpu) {
        const auto g0 = std::chrono::high_resolution_clock::now();
        const double load_ms = ms_since(t_start);
        if (warm.t.joinable()) warm.t.join();
        if (timing)
            std::fprintf(stderr, "cli: scene loaded at %.1f ms, HIP warm-up took %.1f ms, waited %.1f ms for it\n", load_ms,
                         warm_ms, ms_since(g0));
        rt_opts o;
        rt_default_opts(&o);
        o.sort = sort ? 1 : 0;
        o.device = device;
        if (devices > 0) o.device_count = devices;   // devices 0..N-1, RCCL inside rt_render
        if (rt_render(s, &o, fb.data(), &gst)) return die("gpu_raytrace");
        std::printf("GPU Took %gs\n",
                    std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - g0).count());
        if (rt_bloom(fb.data(), s->width, s->height, (float)(0.7 * s->ray_count), 5, device)) return die("bloom");
        std::vector<uint8_t> part(px3);
        rt_tonemap(fb.data(), s->width, s->height, s->exposure, s->ray_count, part.data());
        image.insert(image.end(), part.begin(), part.end());
    }
    if (rt_write_png(out_path, image.data(), s->width, (int)(image.size() / s->width / 3))) return die("stbi_write_png");
    if (stats_path) {
        if (FILE *f = std::fopen(stats_path, "w")) {
            const double secs = gst.render_ms / 1000.0;
            std::fprintf(f,
                         "{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"bounces\": %d, "
                         "\"sort\": %d, \"devices\": %d, \"render_ms\": %.3f, \"kernel_ms\": %.3f, "
                         "\"live_segments\": %llu, \"generated_rays\": %llu, \"live_mrays_per_s\": %.3f, "
                         "\"cpu_s\": %.6f, \"bvh_ms\": %.3f}\n",
                         argv[1], s->width, s->height, s->ray_count, s->bounces, sort ? 1 : 0, devices > 0 ? devices : 1, gst.render_ms,
                         gst.kernel_ms, (unsigned long long)gst.live_segments, (unsigned long long)gst.generated_rays,
                         secs > 0 ? gst.live_segments / secs / 1e6 : 0.0, cpu_s, rt_scene_bvh_ms(host));
            std::fclose(f);
        }
    }
    rt_scene_free(host);
    return 0;
}
