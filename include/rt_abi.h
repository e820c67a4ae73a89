/*
 * rt_abi.h — C ABI of the MI355X-native path tracer (librtamd.so).
 *
 * Drop-in boundary for isaac-chandler/cuda-raytracer's GPU render path.  Plain C types,
 * pointers and sizes only; no HIP or torch types cross this boundary.  Every entry point
 * names the reference interface it replaces (file:line in the reference checkout).
 *
 * Byte layouts of the scene arrays are the reference's (scene.cuh:9-100):
 *   rt_sphere 16 B, rt_triangle 48 B (ray-tracing representation: p1, p2-p1, p3-p1,
 *   normalise(cross(p3-p1, p2-p1))), rt_material 48 B, rt_bvh_node 32 B,
 *   uint16 material indices (spheres first, then triangles), env map float[h][w][3].
 *
 * Errors: every int-returning call returns 0 on success or a negative RT_E_* code and
 * records a message readable with rt_last_error() (thread-local).  The reference printed
 * "Error <expr> <msg>" and exit(1) instead (common.cuh:10-18); the CLI keeps that.
 * Hardware queues: loading the library sets GPU_MAX_HW_QUEUES=24 unless the host has set it (HIP
 * reads it at initialisation; 4 by default), and a renderer keeps at most that many passes in flight,
 * one stream each (up to 20).
 * Threading: calls are blocking.  One rt_renderer is bound to one device and must not be
 * used from two threads at once; distinct renderers may run concurrently.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

enum {
    RT_OK = 0,
    RT_E_INVALID = -1,   /* bad argument / scene */
    RT_E_IO = -2,        /* file could not be read or written */
    RT_E_HIP = -3,       /* HIP runtime error (message has the HIP error string) */
    RT_E_NODEVICE = -4,  /* no HIP device / HIP kernels not loadable */
    RT_E_OOM = -5        /* device allocation failed */
};

typedef struct { float x, y, z; } rt_vec3;
typedef struct { rt_vec3 center; float radius; } rt_sphere;                          /* scene.cuh:9  */
typedef struct { rt_vec3 p1, p2p1, p3p1, normal; } rt_triangle;                      /* scene.cuh:27 */
typedef struct {                                                                      /* scene.cuh:42 */
    rt_vec3 diffuse_albedo; float metallicity;
    rt_vec3 specular_albedo; float roughness;
    rt_vec3 emitted; float index_of_refraction;
} rt_material;
typedef struct { rt_vec3 min_bound, max_bound; int32_t child1, child2; } rt_bvh_node; /* scene.cuh:82 */

/* Host view of a loaded scene; mirrors `struct Scene` (scene.cuh:102-152). All pointers are
 * borrowed host memory. */
typedef struct {
    const rt_sphere *spheres;         int32_t sphere_count;
    const rt_triangle *triangles;     int32_t triangle_count;
    const uint16_t *material_indices;
    const rt_material *materials;     int32_t material_count;
    const rt_bvh_node *bvh;           int32_t bvh_node_count;
    int32_t width, height;
    const rt_vec3 *environment_map;   int32_t environment_map_width, environment_map_height;
    rt_vec3 camera_position, forward, up;
    float vertical_fov, exposure;
    rt_vec3 min_coord, inv_dimensions;
    rt_vec3 scaled_right, scaled_up, near_plane_top_left;
    float inv_width, inv_height;
    int32_t bounces, ray_count;
} rt_scene;

/* ------------------------------------------------------------------ scene loading (host)
 * Replaces load_scene(Scene*, const char*, bool use_bvh) (scene.cu:569-831) including
 * load_ply (:491), load_pfm (:548), precompute_camera_data (:62) and the binned-SAH
 * generate_bvh (:1002-1036).  CRLF scene files are accepted (the reference read them in
 * Windows text mode).  Prints the reference's stdout lines unless opts->quiet. */
typedef struct {
    int32_t use_bvh;          /* 1 = BVH depth 30 (default); 0 = `no_bvh` (single leaf)      */
    int32_t quiet;            /* 1 = suppress "Triangle count"/"BVH Took"/... stdout lines      */
    const char *asset_root;   /* directory relative asset paths resolve against; NULL = CWD  */
    int32_t image_override;   /* 1 = replace the scene's `image` W H spp bounces with below   */
    int32_t width, height, ray_count, bounces;
    int32_t exposure_override;
    float exposure;
    int32_t bvh_device;       /* -1 = build the BVH on the host (default); >= 0 = on that HIP device
                                 (same node array, triangle and material-index order)          */
} rt_load_opts;

typedef struct rt_scene_host rt_scene_host;   /* owns the arrays a rt_scene points into */

int rt_scene_load(const char *path, const rt_load_opts *opts, rt_scene_host **out);
const rt_scene *rt_scene_view(const rt_scene_host *scene);
double rt_scene_bvh_ms(const rt_scene_host *scene);          /* "BVH Took" (scene.cu:1026) */
void rt_scene_free(rt_scene_host *scene);

/* ------------------------------------------------------------------ GPU render
 * Pass p (0-based) of a render casts rtc = min(spp - 20p, 20) rays per pixel with
 * generate-seed `remaining` = spp - 20p - rtc (raytracing.cu:222-229). */
typedef struct {
    int32_t sort;         /* 1 = ray reordering after each bounce but the last (default);
                             0 = `no_sort` (raytracing.cu:238)                             */
    int32_t device;       /* HIP device ordinal                                          */
    int32_t pass_begin;   /* first pass to render (0)                                    */
    int32_t pass_count;   /* passes to render; -1 = all remaining                        */
    int32_t pass_stride;  /* render passes pass_begin, +stride, ... (multi-GPU pass shard) */
    int32_t collect_counters; /* 1 = also count traversal work (Pn/Iv/Tt) for the byte model */
    /* Pixel-tile sharding: the image is cut into stripes of tile_rows rows, dealt
     * round-robin to tile_count owners; this render casts only the rays of owner tile_index's
     * stripes, with their global ray indices (so seeds are the 1-GPU ones), and leaves the other
     * pixels 0.  With sort = 1 the process seeds follow the global post-sort slot
     * (raytracing.cu:89, :238-247), which needs the per-bounce exchange of
     * rt_renderer_set_exchange.  tile_count 0 or 1 = the whole image (default). */
    int32_t tile_count;
    int32_t tile_index;
    int32_t tile_rows;    /* stripe height in rows; 0 = 8 */
    /* Multi-GPU in one process (rt_render only): device_count > 1 renders whole
     * passes round-robin over device_ids[0..device_count) (NULL = devices 0..device_count-1), one
     * host thread and renderer per device, in one RCCL communicator (ncclCommInitAll).  Pass
     * framebuffers are exchanged as pixel slices (ncclAllToAll over xGMI: slice j goes to device
     * j, which adds the slices in pass order, bit-identical to one device) and the finished
     * slices are gathered to device_ids[0] (ncclGather), then copied to fb_out.  0 or 1 = the
     * single device `device`.  The reference ran one device (raytracing.cu:170-284). */
    int32_t device_count;
    const int32_t *device_ids;
    /* With device_count >= 1: 0 = pass sharding (above, the default); 1 = pixel tiles: device k
     * renders owner k's tile_rows-row stripes of every pass, with sort on through the
     * per-bounce bucket-byte ncclAllReduce (rt_renderer_set_exchange), and an ncclReduce of the
     * owners' framebuffers (disjoint pixels, the rest 0) to device_ids[0]. */
    int32_t shard_tiles;
} rt_opts;

typedef struct {
    uint64_t generated_rays;   /* rays generated (sum of n over passes)                    */
    uint64_t live_segments;    /* process_ray invocations on live slots                    */
    uint64_t sorted_items;     /* slots moved by the reorder                               */
    uint64_t nodes_popped;     /* Pn, only with collect_counters                           */
    uint64_t internal_visits;  /* Iv, only with collect_counters                           */
    uint64_t triangle_tests;   /* Tt, only with collect_counters                           */
    uint64_t sphere_tests;     /* S x live segments                                        */
    uint64_t hits, misses;     /* closest-hit outcomes over live segments                  */
    uint64_t hits_sphere;      /* subset of hits on spheres (the rest hit triangles)       */
    uint64_t dead_slots;       /* slots skipped by the terminated-key early-out            */
    uint32_t passes, reserved;
    double render_ms;          /* host wall time of the call (the "GPU Took" span)         */
    double kernel_ms;          /* HIP-event time of the whole pass loop on the stream      */
    double process_ms;         /* HIP-event time summed over the process (traversal) launches */
    double sort_ms;            /* HIP-event time summed over the reorder launches          */
    double trace_ms;           /* trace_kernel launches, summed: each launch's span on the device
                                  wall clock from its first wave's start to its last wave's end
                                  (event timing on; 0 for scenes without triangles, which have
                                  no trace launch)                                          */
    uint64_t trace_launches;   /* trace_kernel launches timed in trace_ms                  */
    /* rt_render runs without per-bounce events (like the benchmark's timed passes): its process_ms,
       sort_ms and trace_ms stay 0 unless RTAMD_EVENTS=1; rt_renderer_run has them by default */
    double exchange_ms;        /* multi-GPU rt_render: host wall time of the RCCL slice exchange
                                  and gather (max over devices).  The multi-GPU render runs
                                  without per-bounce events: process_ms, sort_ms and trace_ms
                                  stay 0 there unless RTAMD_MULTI_EVENTS=1                  */
} rt_stats;

void rt_default_opts(rt_opts *opts);
void rt_default_load_opts(rt_load_opts *opts);
int rt_device_count(void);
/* Initialises the HIP runtime, the device's queues and the kernel code object on `device`
 * (what the first render would otherwise pay, ~0.2 s per process).  Thread-safe; a host can call
 * it on a thread of its own while it loads the scene, as the CLI does.  No reference
 * counterpart: the reference pays CUDA context creation inside gpu_raytrace (raytracing.cu:174). */
int rt_device_warmup(int32_t device);

/* Replaces `Vec3 *gpu_raytrace(const Scene *scene, bool sort)` (raytracing.cu:170-284):
 * uploads the scene, renders every pass selected by opts, and writes the accumulated
 * framebuffer (W*H*3 floats, raw radiance sums, caller-owned) to fb_out. */
int rt_render(const rt_scene *scene, const rt_opts *opts, float *fb_out, rt_stats *stats);

/* Persistent renderer: scene resident in HBM, ray buffers sized for 20 rays/pixel per pass,
 * up to 20 passes in flight on separate streams (each with its own buffer set) so one pass's
 * latency-bound last bounces overlap another's throughput-bound first bounces.  The framebuffer
 * adds stay in pass order.  Used by rt_render, the benchmark and the multi-GPU drivers. */
typedef struct rt_renderer rt_renderer;
int rt_renderer_create(const rt_scene *scene, const rt_opts *opts, rt_renderer **out);
/* Renders passes pass_begin, pass_begin+stride, ... (count passes) and adds each pass's
 * per-pixel sum into the renderer's device framebuffer (ordered: fb += pass_sum, pass
 * order).  If d_pass_sums != NULL (device pointer, count*W*H*3 floats) the pass sums are
 * also stored there.  Blocking. */
int rt_renderer_run(rt_renderer *r, int32_t pass_begin, int32_t count, int32_t stride,
                    float *d_pass_sums, rt_stats *stats);
/* The same passes enqueued without waiting (d_pass_sums required, not for pixel tiles with sort
 * on): rt_renderer_wait_pass makes a caller's HIP stream (a hipStream_t on r's device) wait until
 * the k-th pass of the run (0-based) has written its sums, so the caller can exchange finished
 * passes while later ones render (the multi-GPU slice exchange); rt_renderer_finish waits for the
 * whole run and fills stats.  The framebuffer adds and every other rule are those of
 * rt_renderer_run.  Until rt_renderer_finish returns, every other call on r that runs passes,
 * touches the framebuffer or changes the run's settings (run, run_host, read/copy_framebuffer,
 * clear, set_event_timing, set_counters, launch_profile) fails with RT_E_INVALID and changes
 * nothing.  No reference counterpart (the reference's gpu_raytrace returned at the end). */
int rt_renderer_run_async(rt_renderer *r, int32_t pass_begin, int32_t count, int32_t stride, float *d_pass_sums);
int rt_renderer_wait_pass(rt_renderer *r, int32_t k, void *hip_stream);
int rt_renderer_finish(rt_renderer *r, rt_stats *stats);
/* Same, with the per-pass sums returned in host memory (count*W*H*3 floats). */
int rt_renderer_run_host(rt_renderer *r, int32_t pass_begin, int32_t count, int32_t stride,
                         float *host_pass_sums, rt_stats *stats);
int rt_renderer_read_framebuffer(rt_renderer *r, float *fb_out);   /* device fb -> host     */
int rt_renderer_copy_framebuffer(rt_renderer *r, float *d_out);    /* device fb -> device ptr on
                                                                       r's device (W*H*3 floats) */
int rt_renderer_clear(rt_renderer *r);                               /* zero the device fb    */
/* Pixel tiles with the reorder on (tile_count > 1, sort = 1).  The process seed is the
 * ray's GLOBAL post-sort slot (raytracing.cu:89 after :238-247), so after every bounce but the
 * last the owners exchange one byte per global live ray: each writes bucket + 1 at the global slot
 * of each of its live rays into a zeroed array of n bytes, and `exchange` must sum the arrays of
 * all owners in place (an all-reduce: every slot has one owner, no byte exceeds 65) and return 0.
 * Each owner then ranks its rays as the stable sort of all keys would; rays never migrate.
 * on_device = 1: `bytes` is a device pointer on the renderer's device and the exchange is enqueued
 * on (or completed before returning from) `hip_stream`, a hipStream_t; 0: `bytes` is host memory
 * and the exchange completes before returning.  Calls come in the same order on every owner
 * (pass by pass of a group in flight, bounce by bounce).  Without an exchange such a render fails. */
typedef int (*rt_exchange_fn)(void *user, uint8_t *bytes, uint64_t n, void *hip_stream);
int rt_renderer_set_exchange(rt_renderer *r, rt_exchange_fn fn, void *user, int32_t on_device);
/* The same exchange over RCCL for one process per GPU (torchrun-style hosts): the renderer joins
 * an RCCL communicator of nranks owners (ncclCommInitRank; blocks until every rank has joined) and
 * sums the bytes with an in-place ncclAllReduce(uint8) on the pass's stream, so no byte leaves
 * the device.  Every rank passes the same RT_RCCL_ID_BYTES-byte id: rank 0 makes it with
 * rt_rccl_unique_id and the host hands it to the others (e.g. a torch.distributed broadcast).
 * The communicator is the renderer's and is destroyed with it.  No reference counterpart: the
 * reference ran one device (raytracing.cu:170-284). */
#define RT_RCCL_ID_BYTES 128
int rt_rccl_unique_id(uint8_t *id_out);
int rt_renderer_set_exchange_rccl(rt_renderer *r, const uint8_t *id, int32_t nranks, int32_t rank);
int rt_renderer_set_counters(rt_renderer *r, int32_t enable);
/* Framebuffer accumulation (default on).  Off, a run must be given d_pass_sums and only writes them:
 * no pass is added into the renderer's framebuffer, so no pass's stream waits for another's (the
 * in-order add chain is what the multi-GPU drivers, which add the pass slices themselves, turn off).
 * No reference counterpart. */
int rt_renderer_set_accumulate(rt_renderer *r, int32_t enable);
/* Per-bounce HIP events behind rt_stats.process_ms / sort_ms (default on).  Off, those stay 0 and
 * a pass's stream carries no marker packets between its kernels (~2 % faster frames). */
int rt_renderer_set_event_timing(rt_renderer *r, int32_t enable);
/* Per trace launch of the last run's first pass (event timing on): trace_ms_out[b] = the launch's
 * device wall-clock span (first wave start to last wave end) and live_out[b] = the live rays it
 * traced, for bounce b < cap.  Returns the number of launches written (0 without event timing or
 * for scenes without triangles).  Live counts are known only for runs of at most as many passes
 * as are in flight (the benchmark's one-pass exclusive run); in a longer run live_out[b] is 0.
 * Measurement only; no reference counterpart. */
int rt_renderer_launch_profile(rt_renderer *r, int32_t cap, double *trace_ms_out, uint32_t *live_out);
void rt_renderer_destroy(rt_renderer *r);

/* Persistent multi-GPU renderer (one process): rt_render's device_count >= 1 pass sharding
 * with its set-up kept between renders -- one RCCL communicator over device_ids[0..device_count)
 * (ncclCommInitAll; NULL = devices 0..device_count-1), one renderer per device (scene resident, 16
 * passes in flight each) and the slice-exchange buffers.  opts as for rt_render (sort,
 * collect_counters, device_count, device_ids; pass sharding only: shard_tiles and tile_count are
 * refused).  rt_multi_create fails with RT_E_NODEVICE when a listed device does not exist, and checks
 * that every communicator rank answers (an all-reduce of one int per device; rt_multi_ranks returns the
 * count).  rt_multi_run renders passes 0..pass_count-1 of the frame (-1 = all) round-robin over the
 * devices (pass p on device p mod N), exchanges the pass sums as pixel slices while later passes
 * render (ncclAllToAll; each owner adds its slice in pass order, so the image is bit-identical to one
 * device's) and gathers the frame on device_ids[0]; fb_out (host, W*H*3 floats) receives it unless
 * NULL, and rt_multi_read_framebuffer copies the last run's frame later.  A run that fails after its
 * devices started leaves the object unusable (its communicators may be aborted): destroy it.
 * Blocking; one call at a time per object.  No reference counterpart: the reference ran one device
 * and allocated per call (raytracing.cu:170-284). */
typedef struct rt_multi rt_multi;
int rt_multi_create(const rt_scene *scene, const rt_opts *opts, rt_multi **out);
int rt_multi_run(rt_multi *m, int32_t pass_count, float *fb_out, rt_stats *stats);
int rt_multi_read_framebuffer(rt_multi *m, float *fb_out);
int rt_multi_set_event_timing(rt_multi *m, int32_t enable);   /* per-bounce events (default off) */
int rt_multi_set_counters(rt_multi *m, int32_t enable);       /* traversal counters (Pn/Iv/Tt)   */
int rt_multi_ranks(const rt_multi *m);
void rt_multi_destroy(rt_multi *m);

/* Closest hit of n caller rays: rays = n x {o.x o.y o.z d.x d.y d.z} (d unit length, as every
 * ray the render traces).  The sphere loop (scene.cu:338-372) then bvh_closest_hit_distance
 * (scene.cu:134-241) -- one bounce of process_ray up to the hit (scene.cu:320-374) -- through
 * the render's traversal kernel.  t_out[i] = closest distance (1e30 when nothing is hit),
 * index_out[i] = primitive index (spheres first, then sphere_count + triangle; -1 = miss).
 * With opts->collect_counters the traversal counters are returned in stats. */
int rt_trace_rays(const rt_scene *scene, const rt_opts *opts, const float *rays, int32_t n,
                  float *t_out, int32_t *index_out, rt_stats *stats);

/* Replaces the bloom block of main (raytracing.cu:356-393, kernels :21-74): high-pass
 * (luminance > threshold), clamped box blur of `radius` horizontally then vertically,
 * add back.  fb is a host W*H*3 buffer, updated in place. */
int rt_bloom(float *fb, int32_t width, int32_t height, float threshold, int32_t radius, int32_t device);
/* Same on a device-resident framebuffer (device pointer). */
int rt_bloom_device(float *d_fb, int32_t width, int32_t height, float threshold, int32_t radius,
                    int32_t device);

/* Replaces write_framebuffer_to_output_image (raytracing.cu:286-303). rgb_out: W*H*3. */
void rt_tonemap(const float *fb, int32_t width, int32_t height, float exposure, int32_t ray_count,
                uint8_t *rgb_out);
/* Replaces stbi_write_png (raytracing.cu:395): 8-bit RGB PNG, own encoder (lossless). */
int rt_write_png(const char *path, const uint8_t *rgb, int32_t width, int32_t height);

/* Replaces `Vec3 *cpu_raytrace(Scene *scene)` (raytracing.cu:122-163): the reference's
 * OpenMP CPU path with its bounce-invariant seed; fb_out W*H*3 (overwritten).  Returns the
 * number of passes rendered; seconds = the "CPU Took" span. */
int rt_cpu_render(const rt_scene *scene, float *fb_out, int32_t threads, double *seconds);

const char *rt_last_error(void);
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_ABI_H */
