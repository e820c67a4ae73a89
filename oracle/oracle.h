/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of isaac-chandler/cuda-raytracer's render path, used as the
 * parity checker for the MI355X HIP path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product
 * (cuda-raytracer_amd/, include/rt_abi.h) never links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference has no tests or golden
 * vectors and compiling/running it is denied for every session
 * (SURVEY.md §8c).  Anchors used instead: BVH node/triangle counts from the
 * survey probe (cornell: 32 tris / 21 nodes), primitive counts from REPORT.pdf
 * p.7 (teapot 126,050), and per-channel statistics of renders/<scene>.png
 * (tests/golden/reference_render_stats.json).  Everything else is
 * "parity unpinned": a restatement written from the reference source text.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

typedef struct {
    int32_t width, height, ray_count, bounces;
    float exposure;
    int32_t sphere_count, triangle_count, material_count, bvh_node_count;
    int32_t env_width, env_height;
} orc_info;

/* Per-render counters.  Pn/Iv/Tt are the §8(d) byte-model inputs. */
typedef struct {
    uint64_t generated_rays;
    uint64_t live_segments;     /* process_ray calls on a live slot           */
    uint64_t dead_slots;        /* slots skipped by the key early-out         */
    uint64_t nodes_popped;      /* Pn: node loads at scene.cu:155             */
    uint64_t internal_visits;   /* Iv: child pair slab tests, scene.cu:201-202 */
    uint64_t triangle_tests;    /* Tt: Möller–Trumbore bodies, scene.cu:162    */
    uint64_t sphere_tests;      /* S per live segment                          */
    uint64_t hits_triangle, hits_sphere, misses;
    uint64_t sorted_items;
    uint32_t max_stack;
    uint32_t passes;
    uint32_t max_ray_nodes;     /* largest Pn of a single segment                */
    uint32_t reserved;
} orc_stats;

/* Scene loading (restates scene.cu:491-831 + generate_bvh 1002-1036).
 * asset_root: directory asset paths resolve against (NULL = CWD, as the reference).
 * image: optional {W,H,spp,bounces} override (NULL = scene file); exposure: optional. */
orc_scene *orc_load_scene(const char *path, int use_bvh, const char *asset_root,
                          const int32_t *image, const float *exposure);
void orc_free_scene(orc_scene *s);
const char *orc_last_error(void);
void orc_get_info(const orc_scene *s, orc_info *out);
/* Copy out the flat arrays (reference byte layouts: Sphere 16, Triangle 48,
 * Material 48, BvhNode 32, uint16 material indices, env float[h*w*3]) and the
 * 17-float camera block {camera_position, forward, up, vertical_fov,
 * min_coord, inv_dimensions, scaled_right, scaled_up, near_plane_top_left,
 * inv_width, inv_height} (see orc_camera_floats). Any pointer may be NULL. */
void orc_get_arrays(const orc_scene *s, void *spheres, void *triangles,
                    uint16_t *material_indices, void *materials, void *bvh,
                    float *env, float *camera);
int orc_camera_floats(void);

/* GPU-path semantics (raytracing.cu:170-284): passes [pass_begin, pass_begin+pass_count)
 * (pass_count < 0 = all), slot-seeded RNG, keys, stable sort after every bounce but the
 * last, ordered per-pixel accumulation: fb += (c_0 + c_1 + ... ) per pass.
 * fb_inout: W*H*3 floats, accumulated into.  bucket_hist (optional):
 * [passes][bounces][65] counts of post-process buckets (64 = terminated). */
int orc_render_gpu_semantics(const orc_scene *s, int sort, int pass_begin, int pass_count,
                             float *fb_inout, orc_stats *stats, uint64_t *bucket_hist,
                             int threads);
/* Per-pass sums instead of the running framebuffer: out[pass][W*H*3]. */
/* Pixel-tile sharding with the per-bounce bucket exchange (SURVEY §8e "sort on"): this owner's
 * stripes only; `exchange` must sum `n` bytes in place over all owners (an all-reduce) and return
 * 0.  fb_inout += this owner's pass sums, pass by pass (other pixels untouched). */
typedef int (*orc_exchange_fn)(void *user, uint8_t *bytes, int64_t n);
int orc_render_tiled(const orc_scene *s, int sort, int tile_count, int tile_index, int tile_rows,
                     int pass_begin, int pass_count, orc_exchange_fn exchange, void *user,
                     float *fb_inout, orc_stats *stats, int threads);
int orc_render_pass_sums(const orc_scene *s, int sort, int pass_begin, int pass_count,
                         float *out, int threads);
/* Per bounce b of pass `pass`: max_steps[b] = the longest ray's internal visits + triangle tests
 * (the HIP trace kernel's steps), live[b] = live rays.  Arrays of `bounces` entries. */
int orc_pass_bounce_profile(const orc_scene *s, int sort, int pass, uint32_t *max_steps, uint64_t *live,
                            int threads);
/* Analysis only: the longest ray's dependent record fetches per bounce under the chain models
 * (tools/chain_models.py), and the distinct scene bytes one XCD's rays in flight touch under three ways of
 * dealing the live slots to the XCDs (tools/route_model.py); see oracle.cpp. */
int orc_pass_chain_profile(const orc_scene *s, int sort, int pass, uint64_t *out, int threads);
int orc_bounce_working_set(const orc_scene *s, int sort, int pass, int bounce, int window, int depth,
                           int windows_per_xcd, double *out, int threads);
int orc_bounce_wave_model(const orc_scene *s, int sort, int pass, int bounce, int tile, int obits, int dbits,
                          int refill, double *out, int threads);

/* CPU-path semantics (raytracing.cu:122-163): bounce-invariant seed quirk, no keys,
 * no sort, sequential accumulate.  fb_out: W*H*3 (overwritten). pass_limit < 0 = all. */
int orc_render_cpu_path(const orc_scene *s, float *fb_out, int pass_limit, int threads,
                        double *seconds);
/* Same, also counting live ray segments (process_ray calls past the early-out). */
int orc_render_cpu_path_counted(const orc_scene *s, float *fb_out, int pass_limit, int threads,
                                double *seconds, uint64_t *live_segments);

/* Closest hit of n rays {o.xyz, d.xyz}: the sphere loop (scene.cu:338-372) then
 * bvh_closest_hit_distance (scene.cu:134-241).  t_out = closest (1e30 if nothing is hit),
 * index_out = primitive index or -1; stats (optional) gets Pn / Iv / Tt / sphere tests. */
void orc_closest_hit(const orc_scene *s, const float *rays, int n, float *t_out, int32_t *index_out,
                     orc_stats *stats);

/* Post-process (raytracing.cu:21-74, 286-303). */
void orc_bloom(float *fb, int width, int height, float threshold, int radius);
void orc_tonemap(const float *fb, int width, int height, float exposure, int ray_count,
                 uint8_t *out_rgb);

/* Known-answer helpers for golden vectors. */
void orc_pcg_stream(uint32_t seed, int n, uint32_t *out);
void orc_random_draws(uint32_t seed, int n, float *r01, float *r02, float *rad);
void orc_random_on_sphere(uint32_t seed, int n, float *out_xyz);
void orc_sincos(const float *x, int n, float *s, float *c);
float orc_atan01(float x);
uint32_t orc_generate_seed(int32_t ray_index, int32_t seed);
uint32_t orc_process_seed(int32_t slot, int32_t seed);
uint32_t orc_cpu_seed(int32_t i, int32_t remaining);
uint16_t orc_interleave_5(uint16_t x);
uint32_t orc_morton(float x, float y, float z);
int orc_key_bucket(uint32_t key);
int orc_ray_aabb(const float *bmin, const float *bmax, const float *origin, const float *dir,
                 float tmax, float *tmin_out);
int orc_ray_triangle(const float *tri12, const float *origin, const float *dir,
                     float closest, float *t_out);
int orc_ray_sphere(const float *sphere4, const float *origin, const float *dir, float closest,
                   float *t_out);
void orc_env_project(const float *dir, float *uv);
int orc_env_texel(const float *dir, int env_w, int env_h);

#ifdef __cplusplus
}
#endif
#endif
