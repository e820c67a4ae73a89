// cpu_render.hip — the reference's `cpu` path (raytracing.cu:122-163), host-only.
//
// Keeps the CLI's `cpu` option working: same pass loop, the bounce-invariant seed of the
// reference's OpenMP loop (its inner `i` shadows the bounce index, raytracing.cu:142-149),
// no sort, no bloom, sequential accumulation (:114-120).  The per-ray arithmetic is the
// shared __host__ __device__ code in rt_device.h; traversal walks the reference node layout
// with the reference's explicit (index, distance) stack (scene.cu:134-241).  Work is split
// over std::threads in chunks of 1000 rays, like `schedule(dynamic, 1000)`.
#include "rt_abi.h"
#include "rt_device.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#pragma clang fp contract(off)

namespace rtamd {
int fail(int code, const std::string &msg);
}

using namespace rtd;

namespace {

struct RayState { V3 o, d, T, C; };

V3 vec(const rt_vec3 &v) { return v3(v.x, v.y, v.z); }

void trace_bvh(const rt_scene &s, V3 o, V3 d, float &closest, int &index) {
    const float ix = 1 / d.x, iy = 1 / d.y, iz = 1 / d.z;
    uint32_t idx_stack[32];
    float dist_stack[32];
    int sc = 1;
    idx_stack[0] = 0;
    dist_stack[0] = 0;
    while (sc) {
        sc--;
        if (dist_stack[sc] >= closest) continue;
        const rt_bvh_node &nd = s.bvh[idx_stack[sc]];
        if (nd.child2 <= nd.child1) {
            for (int i = nd.child2; i < nd.child1; i++) {
                const rt_triangle &t = s.triangles[i];
                float th;
                if (ray_triangle(o, d, vec(t.p1), vec(t.p2p1), vec(t.p3p1), closest, th)) {
                    closest = th;
                    index = s.sphere_count + i;
                }
            }
        } else {
            const rt_bvh_node &a = s.bvh[nd.child1], &b = s.bvh[nd.child2];
            float d1, d2;
            const bool h1 = slab(a.min_bound.x, a.min_bound.y, a.min_bound.z, a.max_bound.x, a.max_bound.y,
                                 a.max_bound.z, o, ix, iy, iz, closest, d1);
            const bool h2 = slab(b.min_bound.x, b.min_bound.y, b.min_bound.z, b.max_bound.x, b.max_bound.y,
                                 b.max_bound.z, o, ix, iy, iz, closest, d2);
            if (h1 && h2) {
                const bool near1 = d1 < d2;
                idx_stack[sc] = near1 ? nd.child1 : nd.child2;
                dist_stack[sc++] = near1 ? d1 : d2;
                idx_stack[sc] = near1 ? nd.child2 : nd.child1;
                dist_stack[sc++] = near1 ? d2 : d1;
            } else if (h1) {
                idx_stack[sc] = nd.child1;
                dist_stack[sc++] = d1;
            } else if (h2) {
                idx_stack[sc] = nd.child2;
                dist_stack[sc++] = d2;
            }
        }
    }
}

void process(const rt_scene &s, RayState &r, Rng rng) {
    if (is_black(r.T)) return;                       // scene.cu:326 (host branch)
    float closest = 1e30f;
    int index = -1;
    for (int i = 0; i < s.sphere_count; i++) {
        float t;
        if (ray_sphere(r.o, r.d, vec(s.spheres[i].center), s.spheres[i].radius, closest, t)) {
            closest = t;
            index = i;
        }
    }
    trace_bvh(s, r.o, r.d, closest, index);
    if (index == -1) {
        r.C = r.C + sky_color(&s.environment_map[0].x, s.environment_map_width, s.environment_map_height, r.d) * r.T;
        r.T = v3(0, 0, 0);
        return;
    }
    const V3 hit = r.o + closest * r.d;
    V3 normal;
    if (index < s.sphere_count) {
        normal = (1 / s.spheres[index].radius) * (hit - vec(s.spheres[index].center));
    } else {
        normal = vec(s.triangles[index - s.sphere_count].normal);
    }
    const rt_material &m = s.materials[s.material_indices[index]];
    const Mat mat{vec(m.diffuse_albedo), m.metallicity, vec(m.specular_albedo), m.roughness, vec(m.emitted),
                  m.index_of_refraction};
    V3 nd = r.d;
    scatter(r.d, normal, mat, rng, r.T, r.C, nd);
    r.o = hit;
    r.d = nd;
}

template <class F>
void parallel_chunks(int total, int threads, F &&body) {
    std::atomic<int> next{0};
    auto worker = [&]() {
        for (int b; (b = next.fetch_add(1000)) < total;) {
            const int e = std::min(total, b + 1000);
            for (int i = b; i < e; i++) body(i);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(worker);
    worker();
    for (auto &th : pool) th.join();
}

}  // namespace

extern "C" int rt_cpu_render(const rt_scene *s, float *fb, int32_t threads, double *seconds) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    if (!s || !fb) return rtamd::fail(RT_E_INVALID, "rt_cpu_render: null argument");
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    const int64_t pixels = (int64_t)s->width * s->height;
    if (pixels * 20 > 0x7fffffff) return rtamd::fail(RT_E_INVALID, "image too large");
    std::vector<RayState> rays((size_t)pixels * 20);
    std::fill(fb, fb + pixels * 3, 0.0f);
    int remaining = s->ray_count, passes = 0;
    const V3 cam = vec(s->camera_position), tl = vec(s->near_plane_top_left);
    const V3 sr = vec(s->scaled_right), su = vec(s->scaled_up);
    while (remaining) {
        const int rtc = std::min(remaining, 20);
        remaining -= rtc;
        const int total = (int)(rtc * pixels);
        parallel_chunks(total, threads, [&](int i) {   // generate_initial_rays, scene.cu:78-105
            Rng rng = pcg_seed((uint32_t)i * 0x85810BEAu + 709579u * (uint32_t)remaining);
            const int pixel = i / rtc;
            const int x = pixel % s->width, y = pixel / s->width;
            const float xc = (x + random01(rng)) * s->inv_width;
            const float yc = (y + random01(rng)) * s->inv_height;
            rays[i] = RayState{cam, normalise(tl + xc * sr - yc * su), v3(1, 1, 1), v3(0, 0, 0)};
        });
        for (int b = 0; b < s->bounces; b++) {
            parallel_chunks(total, threads, [&](int i) {
                process(*s, rays[i], pcg_seed(1905678123u * (uint32_t)i + 345903u * (uint32_t)(remaining * 20 + i)));
            });
        }
        for (int i = 0; i < total; i++) {
            float *p = fb + (size_t)(i / rtc) * 3;
            p[0] = p[0] + rays[i].C.x;
            p[1] = p[1] + rays[i].C.y;
            p[2] = p[2] + rays[i].C.z;
        }
        passes++;
    }
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
    return passes;
}
