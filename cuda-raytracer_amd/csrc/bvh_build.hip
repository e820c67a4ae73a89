// bvh_build.hip — the reference's binned-SAH BVH build (scene.cu:866-1036) on the GPU, emitting
// the same node array, triangle order and material-index order as the serial build.
//
// Level-synchronous: every node of a level is one workgroup.
//   * bounds_kernel: the node's box (the reference grows it triangle by triangle with a min/max
//     that keeps the earlier of equal values, so a -0/+0 tie keeps the first triangle's zero:
//     reduced here as (value, index) pairs), the centroid range per axis, the 8 bins per axis
//     (counts and boxes: only their areas reach a decision, and those do not depend on the order
//     the min/max run in), and the split decision, evaluated by one lane with the reference's
//     float expressions in the reference's order;
//   * partition_kernel: the reference's two-pointer loop (scene.cu:960-975) as a closed form.
//     With L = #left (centroid < position) and a = L if A[L] is left (or L = n) else L + 1, the
//     loop examines A[0..a) from the front and A[n-1..a] from the back; front lefts stay, the
//     k-th front right and the k-th back left trade places, and the rights are stacked from the
//     end in the order examined: front right k at rank k + (#back rights before back left k-1),
//     back right y at rank (#back lefts before y) + 1 + (#back rights before y).  A node whose
//     partition is degenerate (L = 0 or n) becomes a leaf, but its range is permuted all the
//     same, as in the reference.
// The host keeps the node list between levels, numbers the nodes as the reference's recursion
// allocates them (children of the k-th split node in depth-first order get 2k+1 and 2k+2), and
// applies the final triangle permutation.
#include "rt_abi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#pragma clang fp contract(off)

namespace rtamd {
int fail(int code, const std::string &msg);
}

namespace {

constexpr int kBins = 8;              // scene.cu:896
constexpr int kBig = 1024;              // workgroup per node above kBigMin triangles: 16 waves
constexpr int kSmall = 64;             // one wave per smaller node
constexpr int kBigMin = 4096;
#ifndef RT_BVH_HUGE
#define RT_BVH_HUGE 32768
#endif
#ifndef RT_BVH_CHUNK
#define RT_BVH_CHUNK 8192
#endif
constexpr int kHuge = RT_BVH_HUGE;     // nodes above this: box, bins and partition over chunks of kChunk
constexpr int kChunk = RT_BVH_CHUNK;   // triangles, one workgroup each, then combined

struct NodeRange {                     // one node of the current level
    int begin, end;
};

struct Chunk {                         // a huge node's triangle sub-range
    int node;                          // the node's index in the level (huge nodes come first)
    int lo, hi;
    int first, n;                      // the node's chunks: [first, first + n)
    int count;                         // the node's triangle count
};

struct BoxPartial {                    // a chunk's box (value, index) extremes and centroid range
    float v[6];
    int vi[6];
    float c[6];
};

struct BinPartial {                    // a chunk's bin counts and bin bound keys
    int cnt[3][8];
    int key[3][8][6];
};

struct NodeOut {                       // per node of the level, written by the kernels
    float lo[3], hi[3];                // the node's box (min_bound, max_bound)
    int axis;                          // -1: no partition (leaf by count, depth or cost)
    float pos;                         // split position
    int left;                          // # triangles left of the split (partition_kernel)
};

// The reference's float min/max (math.cuh): a NaN argument yields the other one; ties keep the
// first argument.
__device__ __forceinline__ float ref_min(float a, float b) { return a != a ? b : (b != b ? a : (b < a ? b : a)); }
__device__ __forceinline__ float ref_max(float a, float b) { return a != a ? b : (b != b ? a : (b > a ? b : a)); }

// (value, index) min/max with the sequential rule: the smaller (larger) value; among equal
// values (==, so -0 and +0 tie) the smaller index.  NaN values never win.
__device__ __forceinline__ void arg_min(float &v, int &i, float v2, int i2) {
    if (v2 != v2) return;
    if (v != v || v2 < v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void arg_max(float &v, int &i, float v2, int i2) {
    if (v2 != v2) return;
    if (v != v || v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

// Float -> int key that orders like the float (for LDS integer atomics on bin bounds).
__device__ __forceinline__ int fkey(float f) {
    const int b = __float_as_int(f);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float funkey(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

__device__ __forceinline__ float half_area(const float lo[3], const float hi[3]) {   // scene.cu:853-858
    const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return x * y + x * z + y * z;
}

// Node box, centroid ranges, bins and the split decision (scene.cu:868-955).
// MODE 0: one workgroup per node does everything.  Huge nodes are spread over workgroups:
// MODE 1: per chunk, the box/centroid extremes -> pbox;  MODE 2: per chunk, the node's box from
// its chunks' pbox, then the chunk's bins -> pbin;  MODE 3: per node, box and bins combined from
// the chunks, then the decision.  (value, index) extremes, integer counts and min/max keys
// combine in any order, so every mode yields the same NodeOut.
template <int kThreads, int MODE>
__global__ __launch_bounds__(kThreads) void bounds_kernel(const NodeRange *__restrict__ nodes,
                                                          const Chunk *__restrict__ chunks,
                                                          const int2 *__restrict__ huge, int depth_left,
                                                          const float4 *__restrict__ blo, const float4 *__restrict__ bhi,
                                                          const float4 *__restrict__ cen, NodeOut *__restrict__ out,
                                                          BoxPartial *__restrict__ pbox, BinPartial *__restrict__ pbin) {
    constexpr int kWaves = kThreads / 64;
    int lo, hi, count, first = 0, nch = 0;
    if (MODE == 1 || MODE == 2) {
        const Chunk ch = chunks[blockIdx.x];
        lo = ch.lo; hi = ch.hi; count = ch.count; first = ch.first; nch = ch.n;
    } else {
        const NodeRange nr = nodes[blockIdx.x];
        lo = nr.begin; hi = nr.end; count = hi - lo;
        if (MODE == 3) { first = huge[blockIdx.x].x; nch = huge[blockIdx.x].y; }
    }
    const int t = threadIdx.x;
    __shared__ float s_v[6][kWaves];
    __shared__ int s_i[6][kWaves];
    __shared__ float s_c[6][kWaves];
    __shared__ int s_cnt[3][kBins];
    __shared__ int s_key[3][kBins][6];
    __shared__ int s_wcnt[kWaves][3][kBins];
    __shared__ int s_wkey[kWaves][3][kBins][6];

    // box (exact first-occurrence semantics) and centroid ranges
    float v[6] = {1e30f, 1e30f, 1e30f, -1e30f, -1e30f, -1e30f};
    int vi[6] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
    float c[6] = {1e30f, 1e30f, 1e30f, -1e30f, -1e30f, -1e30f};
    if (MODE >= 2) {                    // combine the node's chunk extremes (every thread)
        for (int q = first; q < first + nch; q++) {
            const BoxPartial &pb = pbox[q];
            for (int k = 0; k < 6; k++) {
                if (k < 3) arg_min(v[k], vi[k], pb.v[k], pb.vi[k]); else arg_max(v[k], vi[k], pb.v[k], pb.vi[k]);
                c[k] = k < 3 ? ref_min(c[k], pb.c[k]) : ref_max(c[k], pb.c[k]);
            }
        }
    } else {
#pragma unroll 4
    for (int i = lo + t; i < hi; i += kThreads) {
        const float4 l = blo[i], h = bhi[i], ce = cen[i];
        arg_min(v[0], vi[0], l.x, i); arg_min(v[1], vi[1], l.y, i); arg_min(v[2], vi[2], l.z, i);
        arg_max(v[3], vi[3], h.x, i); arg_max(v[4], vi[4], h.y, i); arg_max(v[5], vi[5], h.z, i);
        c[0] = ref_min(c[0], ce.x); c[1] = ref_min(c[1], ce.y); c[2] = ref_min(c[2], ce.z);
        c[3] = ref_max(c[3], ce.x); c[4] = ref_max(c[4], ce.y); c[5] = ref_max(c[5], ce.z);
    }
    // within the wave by shuffles, then across the 16 waves through LDS
    for (int off = 32; off > 0; off >>= 1) {
        for (int k = 0; k < 6; k++) {
            const float ov = __shfl_xor(v[k], off);
            const int oi = __shfl_xor(vi[k], off);
            if (k < 3) arg_min(v[k], vi[k], ov, oi); else arg_max(v[k], vi[k], ov, oi);
            const float oc = __shfl_xor(c[k], off);
            c[k] = k < 3 ? ref_min(c[k], oc) : ref_max(c[k], oc);
        }
    }
    const int wv = t >> 6;
    if ((t & 63) == 0)
        for (int k = 0; k < 6; k++) { s_v[k][wv] = v[k]; s_i[k][wv] = vi[k]; s_c[k][wv] = c[k]; }
    __syncthreads();
    for (int k = 0; k < 6; k++) {
        float a = s_v[k][0], cc = s_c[k][0];
        int ai = s_i[k][0];
        for (int q = 1; q < kWaves; q++) {
            if (k < 3) arg_min(a, ai, s_v[k][q], s_i[k][q]); else arg_max(a, ai, s_v[k][q], s_i[k][q]);
            cc = k < 3 ? ref_min(cc, s_c[k][q]) : ref_max(cc, s_c[k][q]);
        }
        v[k] = a;
        c[k] = cc;
    }
    }
    if (MODE == 1) {
        if (t == 0) {
            BoxPartial &pb = pbox[blockIdx.x];
            for (int k = 0; k < 6; k++) { pb.v[k] = v[k]; pb.vi[k] = vi[k]; pb.c[k] = c[k]; }
        }
        return;
    }
    // The reference starts from the fresh node's (1e30, -1e30) box: a range reduced to those
    // (empty, or only NaN-free sentinels) leaves them as they are.
    float box_lo[3], box_hi[3], cmin[3], cmax[3];
    for (int k = 0; k < 3; k++) {
        box_lo[k] = ref_min(1e30f, v[k]);
        box_hi[k] = ref_max(-1e30f, v[k + 3]);
        cmin[k] = ref_min(1e30f, c[k]);
        cmax[k] = ref_max(-1e30f, c[k + 3]);
    }
    const bool may_split = count > 4 && depth_left > 0;
    if (MODE == 2 && !may_split) return;
    if (may_split && MODE == 3) {        // the chunks' bins
        for (int k = t; k < 3 * kBins; k += kThreads) {
            const int a = k / kBins, b = k % kBins;
            int cnt = 0, key[6] = {fkey(1e30f), fkey(1e30f), fkey(1e30f), fkey(-1e30f), fkey(-1e30f), fkey(-1e30f)};
            for (int q = first; q < first + nch; q++) {
                cnt += pbin[q].cnt[a][b];
                for (int z = 0; z < 3; z++) {
                    key[z] = min(key[z], pbin[q].key[a][b][z]);
                    key[z + 3] = max(key[z + 3], pbin[q].key[a][b][z + 3]);
                }
            }
            s_cnt[a][b] = cnt;
            for (int z = 0; z < 6; z++) s_key[a][b][z] = key[z];
        }
        __syncthreads();
    } else if (may_split) {
        // Bins per wave in LDS (integer atomics on keys that order like the floats; only 64 lanes
        // contend for a wave's bins), then combined over the waves.
        const int w = t >> 6, lane = t & 63;
        for (int k = lane; k < 3 * kBins; k += 64) {
            const int a = k / kBins, b = k % kBins;
            s_wcnt[w][a][b] = 0;
            for (int q = 0; q < 3; q++) s_wkey[w][a][b][q] = fkey(1e30f);
            for (int q = 3; q < 6; q++) s_wkey[w][a][b][q] = fkey(-1e30f);
        }
        __syncthreads();
        float scale[3];
        for (int a = 0; a < 3; a++) scale[a] = kBins / (cmax[a] - cmin[a]);   // scene.cu:911
        // Neighbouring triangles mostly share a bin, so per-lane atomics would serialise 64 ways on
        // one LDS word: in the 16-wave (big-node) variant the lanes holding the same bin are found
        // by ballot, reduced across the wave by shuffles, and one lane per (wave, bin) does the
        // atomics (lamp root: 5.4 -> ~2 ms).  Small nodes' bins vary more across a wave, and there
        // the per-lane atomics are cheaper.  The loop is wave-uniform (ballots need every lane).
        for (int i0 = lo + (t & ~63); i0 < hi; i0 += kThreads) {
            const int i = i0 + lane;
            const bool valid = i < hi;
            float4 l = make_float4(0, 0, 0, 0), h = l, ce = l;
            if (valid) { l = blo[i]; h = bhi[i]; ce = cen[i]; }
            const float cc[3] = {ce.x, ce.y, ce.z};
            const int kl[3] = {fkey(l.x), fkey(l.y), fkey(l.z)}, kh[3] = {fkey(h.x), fkey(h.y), fkey(h.z)};
            for (int a = 0; a < 3; a++) {
                if (cmin[a] == cmax[a]) continue;
                const int b = min(kBins - 1, (int)((cc[a] - cmin[a]) * scale[a]));   // scene.cu:918
                if (kWaves == 1) {      // one-wave nodes (<= 4096 triangles): plain per-lane atomics
                    if (valid) {
                        atomicAdd(&s_wcnt[w][a][b], 1);
                        for (int q = 0; q < 3; q++) {
                            atomicMin(&s_wkey[w][a][b][q], kl[q]);
                            atomicMax(&s_wkey[w][a][b][q + 3], kh[q]);
                        }
                    }
                    continue;
                }
                unsigned long long rem = __ballot(valid);
                while (rem) {
                    const int leader = __ffsll((long long)rem) - 1;
                    const int b0 = __shfl(b, leader);
                    const bool in = valid && b == b0;
                    const unsigned long long m = __ballot(in);
                    int r[6];
                    for (int q = 0; q < 3; q++) {
                        r[q] = in ? kl[q] : 0x7fffffff;
                        r[q + 3] = in ? kh[q] : (int)0x80000000;
                    }
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1)
                        for (int q = 0; q < 3; q++) {
                            r[q] = min(r[q], __shfl_xor(r[q], off));
                            r[q + 3] = max(r[q + 3], __shfl_xor(r[q + 3], off));
                        }
                    if (lane == leader) {
                        atomicAdd(&s_wcnt[w][a][b0], __popcll(m));
                        for (int q = 0; q < 3; q++) {
                            atomicMin(&s_wkey[w][a][b0][q], r[q]);
                            atomicMax(&s_wkey[w][a][b0][q + 3], r[q + 3]);
                        }
                    }
                    rem &= ~m;
                }
            }
        }
        __syncthreads();
        for (int k = t; k < 3 * kBins; k += kThreads) {
            const int a = k / kBins, b = k % kBins;
            int cnt = 0, key[6];
            for (int q = 0; q < 6; q++) key[q] = s_wkey[0][a][b][q];
            for (int v2 = 0; v2 < kWaves; v2++) {
                cnt += s_wcnt[v2][a][b];
                for (int q = 0; q < 3; q++) {
                    key[q] = min(key[q], s_wkey[v2][a][b][q]);
                    key[q + 3] = max(key[q + 3], s_wkey[v2][a][b][q + 3]);
                }
            }
            s_cnt[a][b] = cnt;
            for (int q = 0; q < 6; q++) s_key[a][b][q] = key[q];
        }
        __syncthreads();
        if (MODE == 2) {
            for (int k = t; k < 3 * kBins; k += kThreads) {
                const int a = k / kBins, b = k % kBins;
                pbin[blockIdx.x].cnt[a][b] = s_cnt[a][b];
                for (int q = 0; q < 6; q++) pbin[blockIdx.x].key[a][b][q] = s_key[a][b][q];
            }
            return;
        }
    }
    if (t != 0) return;
    NodeOut o;
    for (int k = 0; k < 3; k++) { o.lo[k] = box_lo[k]; o.hi[k] = box_hi[k]; }
    o.axis = -1;
    o.pos = 0.0f;
    o.left = 0;
    if (may_split) {
        const float own_cost = half_area(box_lo, box_hi) * count;
        float best_cost = own_cost, best_pos = 0.0f;
        int best_axis = -1;
        for (int a = 0; a < 3; a++) {
            if (cmin[a] == cmax[a]) continue;
            float larea[kBins - 1], rarea[kBins - 1];
            int lcount[kBins - 1];
            float llo[3] = {1e30f, 1e30f, 1e30f}, lhi[3] = {-1e30f, -1e30f, -1e30f};
            float rlo[3] = {1e30f, 1e30f, 1e30f}, rhi[3] = {-1e30f, -1e30f, -1e30f};
            int lsum = 0;
            for (int i = 0; i + 1 < kBins; i++) {                              // scene.cu:928-937
                lsum += s_cnt[a][i];
                lcount[i] = lsum;
                const int r = kBins - 1 - i;
                for (int q = 0; q < 3; q++) {
                    llo[q] = ref_min(llo[q], funkey(s_key[a][i][q]));
                    lhi[q] = ref_max(lhi[q], funkey(s_key[a][i][q + 3]));
                    rlo[q] = ref_min(rlo[q], funkey(s_key[a][r][q]));
                    rhi[q] = ref_max(rhi[q], funkey(s_key[a][r][q + 3]));
                }
                larea[i] = half_area(llo, lhi);
                rarea[kBins - 2 - i] = half_area(rlo, rhi);
            }
            const float step = (cmax[a] - cmin[a]) / kBins;                    // scene.cu:940
            for (int i = 0; i + 1 < kBins; i++) {                              // scene.cu:942-953
                const float cost = lcount[i] * larea[i] + (count - lcount[i]) * rarea[i];
                if (cost != 0 && cost < best_cost) {
                    best_axis = a;
                    best_pos = cmin[a] + step * (i + 1);
                    best_cost = cost;
                }
            }
        }
        if (best_axis >= 0 && best_cost < own_cost) {
            o.axis = best_axis;
            o.pos = best_pos;
        }
    }
    out[blockIdx.x] = o;
}

// Block-wide exclusive scan of one small int per thread (wave: shuffles; across waves: LDS);
// *total = the block's sum.
template <int kWaves>
__device__ __forceinline__ int block_scan(int x, int *total, int *s_wave) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    const int wave_total = __shfl(incl, 63);
    if (kWaves == 1) {
        *total = wave_total;
        return incl - x;
    }
    if (lane == 63) s_wave[w] = wave_total;
    __syncthreads();
    int before = 0, sum = 0;
#pragma unroll
    for (int k = 0; k < kWaves; k++) {
        const int c = s_wave[k];
        before += k < w ? c : 0;
        sum += c;
    }
    __syncthreads();                    // s_wave is reused by the next call
    *total = sum;
    return before + incl - x;
}

// The reference's partition of a node's range (scene.cu:960-975) in closed form (see the top).
// Pass 0 stores each element's side as a byte; the scans then walk the front (positions
// [0, a) ascending) and the back (positions [a, n) descending) kPer elements per thread at a
// time.  Element order within the range moves to tmp and back; idx/blo/bhi/cen move together.
constexpr int kPer = 4;
template <int kThreads>
__global__ __launch_bounds__(kThreads) void partition_kernel(const NodeRange *__restrict__ nodes,
                                                             NodeOut *__restrict__ out, uint32_t *__restrict__ idx,
                                                             float4 *__restrict__ blo, float4 *__restrict__ bhi,
                                                             float4 *__restrict__ cen, uint32_t *__restrict__ t_idx,
                                                             float4 *__restrict__ t_blo, float4 *__restrict__ t_bhi,
                                                             float4 *__restrict__ t_cen, int *__restrict__ xk,
                                                             int *__restrict__ rk, uint8_t *__restrict__ side) {
    const NodeOut no = out[blockIdx.x];
    if (no.axis < 0) return;
    const NodeRange nr = nodes[blockIdx.x];
    const int base = nr.begin, n = nr.end - nr.begin;
    const int t = threadIdx.x;
    const float pos = no.pos;
    const int axis = no.axis;
    constexpr int kWaves = kThreads / 64, kTile = kThreads * kPer;
    __shared__ int s_scan[kWaves];
    uint8_t *S = side + base;               // 1 = left (centroid < position)
    int cnt = 0;
    for (int p = t; p < n; p += kThreads) {
        const float4 c = cen[base + p];
        const float v = axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
        const bool l = v < pos;
        S[p] = l ? 1 : 0;
        cnt += l;
    }
    int L;
    (void)block_scan<kWaves>(cnt, &L, s_scan);
    __syncthreads();                                 // the side bytes are read by other lanes below
    const int a = (L == n || S[L]) ? L : L + 1;
    int *X = xk + base, *R = rk + base;
    auto move = [&](int from, int to) {
        t_idx[base + to] = idx[base + from];
        t_blo[base + to] = blo[base + from];
        t_bhi[base + to] = bhi[base + from];
        t_cen[base + to] = cen[base + from];
    };
    // front A[0..a): the k-th right records X[k] = its position
    int run = 0;
    for (int p0 = 0; p0 < a; p0 += kTile) {
        uint8_t f[kPer];
        int c = 0;
        for (int j = 0; j < kPer; j++) {
            const int p = p0 + t * kPer + j;
            f[j] = p < a ? (uint8_t)(S[p] ? 0 : 1) : 0;     // 1 = right
            c += f[j];
        }
        int tot;
        int k = run + block_scan<kWaves>(c, &tot, s_scan);
        for (int j = 0; j < kPer; j++)
            if (f[j]) X[k++] = p0 + t * kPer + j;
        run += tot;
    }
    __syncthreads();
    // back A[n-1..a] (B-index y = n-1-p): lefts record R[k] = # back rights before them;
    // back rights go to their final place
    const int nb = n - a;
    int run_l = 0, run_r = 0;
    for (int y0 = 0; y0 < nb; y0 += kTile) {
        uint8_t f[kPer];                    // 0 none, 1 left, 2 right
        int cl = 0, cr = 0;
        for (int j = 0; j < kPer; j++) {
            const int y = y0 + t * kPer + j;
            f[j] = y < nb ? (S[n - 1 - y] ? 1 : 2) : 0;
            cl += f[j] == 1;
            cr += f[j] == 2;
        }
        int tot;
        const int packed = block_scan<kWaves>(cl | (cr << 16), &tot, s_scan);
        int kl = run_l + (packed & 0xffff), kr = run_r + (packed >> 16);
        for (int j = 0; j < kPer; j++) {
            const int y = y0 + t * kPer + j;
            if (f[j] == 1) R[kl++] = kr;
            else if (f[j] == 2) { move(n - 1 - y, n - 1 - (kl + 1 + kr)); kr++; }
        }
        run_l += tot & 0xffff;
        run_r += tot >> 16;
    }
    __syncthreads();
    // back lefts take the places of the front rights
    run_l = 0;
    for (int y0 = 0; y0 < nb; y0 += kTile) {
        uint8_t f[kPer];
        int c = 0;
        for (int j = 0; j < kPer; j++) {
            const int y = y0 + t * kPer + j;
            f[j] = y < nb ? S[n - 1 - y] : 0;
            c += f[j];
        }
        int tot;
        int kl = run_l + block_scan<kWaves>(c, &tot, s_scan);
        for (int j = 0; j < kPer; j++)
            if (f[j]) move(n - 1 - (y0 + t * kPer + j), X[kl++]);
        run_l += tot;
    }
    // front lefts stay; the k-th front right goes to rank k + (# back rights before back left k-1)
    run = 0;
    for (int p0 = 0; p0 < a; p0 += kTile) {
        uint8_t f[kPer];                    // 0 none, 1 left, 2 right
        int c = 0;
        for (int j = 0; j < kPer; j++) {
            const int p = p0 + t * kPer + j;
            f[j] = p < a ? (S[p] ? 1 : 2) : 0;
            c += f[j] == 2;
        }
        int tot;
        int k = run + block_scan<kWaves>(c, &tot, s_scan);
        for (int j = 0; j < kPer; j++) {
            const int p = p0 + t * kPer + j;
            if (f[j] == 1) move(p, p);
            else if (f[j] == 2) { move(p, n - 1 - (k + (k >= 1 ? R[k - 1] : 0))); k++; }
        }
        run += tot;
    }
    __syncthreads();
    for (int p = t; p < n; p += kThreads) {
        idx[base + p] = t_idx[base + p];
        blo[base + p] = t_blo[base + p];
        bhi[base + p] = t_bhi[base + p];
        cen[base + p] = t_cen[base + p];
    }
    if (t == 0) out[blockIdx.x].left = L;
}


// The closed-form partition of a huge node over its chunks (one workgroup per chunk; the same
// moves as partition_kernel, with the ranks made global by the chunks' counts):
//   P1 side bytes and lefts per chunk; P2 front rights / back lefts / back rights per chunk
//   (front = positions [0, a), back = [a, n)); P3 X[k] for the front rights, R[j] for the back
//   lefts, back rights to their places; P4 back lefts to X[j], front rights to
//   n-1-(k + R[k-1]), front lefts in place; P5 the node's range back from tmp.
// Back ranks count in the reference's examination order from the end (descending positions).
struct PartCounts { int l, fr, bl, br; };

__device__ __forceinline__ void huge_node_split(const Chunk &ch, const PartCounts *cnt, const uint8_t *S, int n,
                                                int &L, int &a) {
    L = 0;
    for (int q = ch.first; q < ch.first + ch.n; q++) L += cnt[q].l;
    a = (L == n || S[L]) ? L : L + 1;
}

template <int kThreads, int PHASE>
__global__ __launch_bounds__(kThreads) void partition_huge_kernel(const NodeRange *__restrict__ nodes,
                                                                  const Chunk *__restrict__ chunks,
                                                                  NodeOut *__restrict__ out, uint32_t *__restrict__ idx,
                                                                  float4 *__restrict__ blo, float4 *__restrict__ bhi,
                                                                  float4 *__restrict__ cen, uint32_t *__restrict__ t_idx,
                                                                  float4 *__restrict__ t_blo, float4 *__restrict__ t_bhi,
                                                                  float4 *__restrict__ t_cen, int *__restrict__ xk,
                                                                  int *__restrict__ rk, uint8_t *__restrict__ side,
                                                                  PartCounts *__restrict__ cnt) {
    const Chunk ch = chunks[blockIdx.x];
    const NodeOut no = out[ch.node];
    if (no.axis < 0) return;
    const int base = nodes[ch.node].begin, n = ch.count;
    const int c0 = ch.lo - base, c1 = ch.hi - base;         // this chunk's positions in the node
    const int t = threadIdx.x;
    constexpr int kWaves = kThreads / 64, kTile = kThreads * kPer;
    __shared__ int s_scan[kWaves];
    uint8_t *S = side + base;
    int *X = xk + base, *R = rk + base;
    auto move = [&](int from, int to) {
        t_idx[base + to] = idx[base + from];
        t_blo[base + to] = blo[base + from];
        t_bhi[base + to] = bhi[base + from];
        t_cen[base + to] = cen[base + from];
    };
    if (PHASE == 1) {
        int c = 0;
        for (int p = c0 + t; p < c1; p += kThreads) {
            const float4 ce = cen[base + p];
            const float v = no.axis == 0 ? ce.x : (no.axis == 1 ? ce.y : ce.z);
            const bool l = v < no.pos;
            S[p] = l ? 1 : 0;
            c += l;
        }
        int tot;
        (void)block_scan<kWaves>(c, &tot, s_scan);
        if (t == 0) cnt[blockIdx.x].l = tot;
        return;
    }
    if (PHASE == 5) {
        for (int p = c0 + t; p < c1; p += kThreads) {
            idx[base + p] = t_idx[base + p];
            blo[base + p] = t_blo[base + p];
            bhi[base + p] = t_bhi[base + p];
            cen[base + p] = t_cen[base + p];
        }
        if (blockIdx.x == (unsigned)ch.first && t == 0) {
            int L, a;
            huge_node_split(ch, cnt, S, n, L, a);
            out[ch.node].left = L;
        }
        return;
    }
    int L, a;
    huge_node_split(ch, cnt, S, n, L, a);
    const int f0 = c0, f1 = min(c1, a);                      // front part of the chunk: [f0, f1)
    const int b0 = max(c0, a), b1 = c1;                      // back part: [b0, b1), walked b1-1 down to b0
    if (PHASE == 2) {
        int fr = 0, bl = 0, br = 0;
        for (int p = f0 + t; p < f1; p += kThreads) fr += S[p] ? 0 : 1;
        for (int p = b0 + t; p < b1; p += kThreads) { bl += S[p]; br += S[p] ? 0 : 1; }
        int tfr, tbl, tbr;
        (void)block_scan<kWaves>(fr, &tfr, s_scan);
        (void)block_scan<kWaves>(bl, &tbl, s_scan);
        (void)block_scan<kWaves>(br, &tbr, s_scan);
        if (t == 0) { cnt[blockIdx.x].fr = tfr; cnt[blockIdx.x].bl = tbl; cnt[blockIdx.x].br = tbr; }
        return;
    }
    // global rank offsets: front rights of earlier chunks; back lefts / rights of later chunks
    int fr_before = 0, bl_after = 0, br_after = 0;
    for (int q = ch.first; q < (int)blockIdx.x; q++) fr_before += cnt[q].fr;
    for (int q = blockIdx.x + 1; q < ch.first + ch.n; q++) { bl_after += cnt[q].bl; br_after += cnt[q].br; }
    // back part, descending positions (the reference's order from the end)
    const int nb = b1 - b0;
    int run_l = bl_after, run_r = br_after;
    for (int y0 = 0; y0 < nb; y0 += kTile) {
        uint8_t f[kPer];                    // 0 none, 1 left, 2 right
        int cl = 0, cr = 0;
        for (int j = 0; j < kPer; j++) {
            const int y = y0 + t * kPer + j;
            f[j] = y < nb ? (S[b1 - 1 - y] ? 1 : 2) : 0;
            cl += f[j] == 1;
            cr += f[j] == 2;
        }
        int tot;
        const int packed = block_scan<kWaves>(cl | (cr << 16), &tot, s_scan);
        int kl = run_l + (packed & 0xffff), kr = run_r + (packed >> 16);
        for (int j = 0; j < kPer; j++) {
            const int p = b1 - 1 - (y0 + t * kPer + j);
            if (f[j] == 1) {
                if (PHASE == 3) R[kl] = kr;
                else move(p, X[kl]);
                kl++;
            } else if (f[j] == 2) {
                if (PHASE == 3) move(p, n - 1 - (kl + 1 + kr));
                kr++;
            }
        }
        run_l += tot & 0xffff;
        run_r += tot >> 16;
    }
    // front part, ascending positions
    int run = fr_before;
    for (int p0 = f0; p0 < f1; p0 += kTile) {
        uint8_t f[kPer];                    // 0 none, 1 left, 2 right
        int c = 0;
        for (int j = 0; j < kPer; j++) {
            const int p = p0 + t * kPer + j;
            f[j] = p < f1 ? (S[p] ? 1 : 2) : 0;
            c += f[j] == 2;
        }
        int tot;
        int k = run + block_scan<kWaves>(c, &tot, s_scan);
        for (int j = 0; j < kPer; j++) {
            const int p = p0 + t * kPer + j;
            if (f[j] == 2) {
                if (PHASE == 3) X[k] = p;
                else move(p, n - 1 - (k + (k >= 1 ? R[k - 1] : 0)));
                k++;
            } else if (f[j] == 1 && PHASE == 4) {
                move(p, p);
            }
        }
        run += tot;
    }
}

#define BCHK(call)                                                                                 \
    do {                                                                                           \
        const hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) return rtamd::fail(RT_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
struct Buf {
    T *p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t n) { return hipMalloc(reinterpret_cast<void **>(&p), std::max<size_t>(n, 1) * sizeof(T)); }
};

struct TreeNode {                       // host-side node of the build
    float lo[3], hi[3];
    int begin, end;
    int child = -1;                     // first of the two children in `tree` (-1: leaf)
};

}  // namespace

namespace rtamd {

// The reference's generate_bvh (scene.cu:1002-1036) up to the triangle post-processing: tris in
// build representation (p1, p2, p3, centroid) and their material indices are permuted in place,
// nodes receives the node array.  max_depth 30 (BVH) or 0 (no_bvh).
int gpu_build_bvh(std::vector<rt_triangle> &tris, uint16_t *tri_mats, std::vector<rt_bvh_node> &nodes,
                  int max_depth, int device) {
    const int n = (int)tris.size();
    using clk = std::chrono::high_resolution_clock;
    const bool timing = std::getenv("RTAMD_TIMING") != nullptr;
    auto t_mark = clk::now();
    std::string report;
    auto mark = [&](const char *what) {
        if (!timing) return;
        const auto now = clk::now();
        char buf[96];
        std::snprintf(buf, sizeof(buf), " %s %.2f ms,", what, std::chrono::duration<double, std::milli>(now - t_mark).count());
        report += buf;
        t_mark = now;
    };
    BCHK(hipSetDevice(device));
    // per-triangle boxes as the reference grows them (p1, p2, p3 in turn), centroids
    std::vector<float4> h_lo(std::max(n, 1)), h_hi(std::max(n, 1)), h_cen(std::max(n, 1));
    auto mn = [](float a, float b) { return a != a ? b : (b != b ? a : (b < a ? b : a)); };
    auto mx = [](float a, float b) { return a != a ? b : (b != b ? a : (b > a ? b : a)); };
    for (int i = 0; i < n; i++) {
        const rt_triangle &t = tris[i];
        const rt_vec3 v[3] = {t.p1, t.p2p1, t.p3p1};
        float l[3] = {1e30f, 1e30f, 1e30f}, h[3] = {-1e30f, -1e30f, -1e30f};
        for (const rt_vec3 &p : v) {
            const float c[3] = {p.x, p.y, p.z};
            for (int k = 0; k < 3; k++) { l[k] = mn(l[k], c[k]); h[k] = mx(h[k], c[k]); }
        }
        h_lo[i] = make_float4(l[0], l[1], l[2], 0.0f);
        h_hi[i] = make_float4(h[0], h[1], h[2], 0.0f);
        h_cen[i] = make_float4(t.normal.x, t.normal.y, t.normal.z, 0.0f);
    }
    std::vector<uint32_t> h_idx(std::max(n, 1));
    for (int i = 0; i < n; i++) h_idx[i] = (uint32_t)i;
    Buf<float4> blo, bhi, cen, t_blo, t_bhi, t_cen;
    Buf<uint32_t> idx, t_idx;
    Buf<int> xk, rk;
    Buf<uint8_t> side;
    Buf<NodeRange> d_nodes;
    Buf<NodeOut> d_out;
    Buf<Chunk> d_chunks;
    Buf<int2> d_huge;
    Buf<BoxPartial> pbox;
    Buf<BinPartial> pbin;
    Buf<PartCounts> pcnt;
    const size_t m = std::max(n, 1);
    BCHK(blo.alloc(m)); BCHK(bhi.alloc(m)); BCHK(cen.alloc(m));
    BCHK(t_blo.alloc(m)); BCHK(t_bhi.alloc(m)); BCHK(t_cen.alloc(m));
    BCHK(idx.alloc(m)); BCHK(t_idx.alloc(m)); BCHK(xk.alloc(m)); BCHK(rk.alloc(m)); BCHK(side.alloc(m));
    // a level holds at most n / 1 nodes (ranges are disjoint and non-empty below the root)
    BCHK(d_nodes.alloc(m)); BCHK(d_out.alloc(m));
    // chunks of the huge nodes of a level: disjoint ranges of > kHuge triangles, so fewer than
    // n / kChunk + n / kHuge of them
    const size_t max_chunks = (size_t)n / kChunk + (size_t)n / kHuge + 1;
    BCHK(d_chunks.alloc(max_chunks)); BCHK(d_huge.alloc(max_chunks));
    BCHK(pbox.alloc(max_chunks)); BCHK(pbin.alloc(max_chunks)); BCHK(pcnt.alloc(max_chunks));
    std::vector<Chunk> h_chunks;
    std::vector<int2> h_huge;
    // the per-thread default stream: the build is synchronous, and a stream costs ~3.6 ms to create
    hipStream_t s = hipStreamPerThread;
    BCHK(hipMemcpyAsync(blo.p, h_lo.data(), m * sizeof(float4), hipMemcpyHostToDevice, s));
    BCHK(hipMemcpyAsync(bhi.p, h_hi.data(), m * sizeof(float4), hipMemcpyHostToDevice, s));
    BCHK(hipMemcpyAsync(cen.p, h_cen.data(), m * sizeof(float4), hipMemcpyHostToDevice, s));
    BCHK(hipMemcpyAsync(idx.p, h_idx.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice, s));

    BCHK(hipStreamSynchronize(s));
    mark("setup+upload");
    std::vector<TreeNode> tree(1);
    tree[0].begin = 0;
    tree[0].end = n;
    std::vector<int> level{0};                   // tree indices of the current level
    std::vector<NodeRange> h_ranges;
    std::vector<NodeOut> h_out;
    std::string levels_report;
    for (int depth = 0; !level.empty(); depth++) {
        const auto t_level = clk::now();
        const int cnt = (int)level.size();
        // huge nodes first (box and bins over many workgroups), then big ones (a 16-wave
        // workgroup each), then the rest (one wave each)
        auto len_of = [&](int x) { return tree[x].end - tree[x].begin; };
        std::stable_partition(level.begin(), level.end(), [&](int x) { return len_of(x) > kBigMin; });
        std::stable_partition(level.begin(), level.end(), [&](int x) { return len_of(x) > kHuge; });
        int nbig = 0, nhuge = 0;
        h_ranges.resize(cnt);
        h_chunks.clear();
        h_huge.clear();
        for (int k = 0; k < cnt; k++) {
            h_ranges[k] = {tree[level[k]].begin, tree[level[k]].end};
            const int len = h_ranges[k].end - h_ranges[k].begin;
            nbig += len > kBigMin;
            if (len > kHuge) {
                nhuge++;
                const int first = (int)h_chunks.size(), nch = (len + kChunk - 1) / kChunk;
                for (int j = 0; j < nch; j++)
                    h_chunks.push_back(Chunk{k, h_ranges[k].begin + j * kChunk,
                                             std::min(h_ranges[k].end, h_ranges[k].begin + (j + 1) * kChunk), first, nch,
                                             len});
                h_huge.push_back(make_int2(first, nch));
            }
        }
        BCHK(hipMemcpyAsync(d_nodes.p, h_ranges.data(), cnt * sizeof(NodeRange), hipMemcpyHostToDevice, s));
        const int left_depth = max_depth - depth;
        if (nhuge) {
            const int nch = (int)h_chunks.size();
            BCHK(hipMemcpyAsync(d_chunks.p, h_chunks.data(), nch * sizeof(Chunk), hipMemcpyHostToDevice, s));
            BCHK(hipMemcpyAsync(d_huge.p, h_huge.data(), nhuge * sizeof(int2), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL((bounds_kernel<kBig, 1>), dim3(nch), dim3(kBig), 0, s, d_nodes.p, d_chunks.p, d_huge.p,
                               left_depth, blo.p, bhi.p, cen.p, d_out.p, pbox.p, pbin.p);
            hipLaunchKernelGGL((bounds_kernel<kBig, 2>), dim3(nch), dim3(kBig), 0, s, d_nodes.p, d_chunks.p, d_huge.p,
                               left_depth, blo.p, bhi.p, cen.p, d_out.p, pbox.p, pbin.p);
            hipLaunchKernelGGL((bounds_kernel<kSmall, 3>), dim3(nhuge), dim3(kSmall), 0, s, d_nodes.p, d_chunks.p,
                               d_huge.p, left_depth, blo.p, bhi.p, cen.p, d_out.p, pbox.p, pbin.p);
        }
        if (nbig > nhuge)
            hipLaunchKernelGGL((bounds_kernel<kBig, 0>), dim3(nbig - nhuge), dim3(kBig), 0, s, d_nodes.p + nhuge,
                               d_chunks.p, d_huge.p, left_depth, blo.p, bhi.p, cen.p, d_out.p + nhuge, pbox.p, pbin.p);
        if (nhuge) {
            const int nch = (int)h_chunks.size();
#define RT_PART_HUGE(PH)                                                                                         \
    hipLaunchKernelGGL((partition_huge_kernel<kBig, PH>), dim3(nch), dim3(kBig), 0, s, d_nodes.p, d_chunks.p,     \
                       d_out.p, idx.p, blo.p, bhi.p, cen.p, t_idx.p, t_blo.p, t_bhi.p, t_cen.p, xk.p, rk.p, side.p, \
                       pcnt.p)
            RT_PART_HUGE(1); RT_PART_HUGE(2); RT_PART_HUGE(3); RT_PART_HUGE(4); RT_PART_HUGE(5);
#undef RT_PART_HUGE
        }
        if (nbig > nhuge)
            hipLaunchKernelGGL(partition_kernel<kBig>, dim3(nbig - nhuge), dim3(kBig), 0, s, d_nodes.p + nhuge,
                               d_out.p + nhuge, idx.p, blo.p, bhi.p, cen.p, t_idx.p, t_blo.p, t_bhi.p, t_cen.p, xk.p,
                               rk.p, side.p);
        if (cnt > nbig) {
            hipLaunchKernelGGL((bounds_kernel<kSmall, 0>), dim3(cnt - nbig), dim3(kSmall), 0, s, d_nodes.p + nbig,
                               d_chunks.p, d_huge.p, left_depth, blo.p, bhi.p, cen.p, d_out.p + nbig, pbox.p, pbin.p);
            hipLaunchKernelGGL(partition_kernel<kSmall>, dim3(cnt - nbig), dim3(kSmall), 0, s, d_nodes.p + nbig,
                               d_out.p + nbig, idx.p, blo.p, bhi.p, cen.p, t_idx.p, t_blo.p, t_bhi.p, t_cen.p, xk.p, rk.p, side.p);
        }
        BCHK(hipGetLastError());
        h_out.resize(cnt);
        BCHK(hipMemcpyAsync(h_out.data(), d_out.p, cnt * sizeof(NodeOut), hipMemcpyDeviceToHost, s));
        BCHK(hipStreamSynchronize(s));
        std::vector<int> next;
        for (int k = 0; k < cnt; k++) {
            const NodeOut &o = h_out[k];
            TreeNode &tn = tree[level[k]];
            std::memcpy(tn.lo, o.lo, sizeof(tn.lo));
            std::memcpy(tn.hi, o.hi, sizeof(tn.hi));
            const int len = tn.end - tn.begin;
            if (o.axis < 0 || o.left == 0 || o.left == len) continue;   // leaf (scene.cu:977-980)
            const int c = (int)tree.size();
            const int b = tn.begin, e = tn.end, mid = tn.begin + o.left;
            tree[level[k]].child = c;
            tree.push_back(TreeNode{});
            tree.push_back(TreeNode{});
            tree[c].begin = b; tree[c].end = mid;
            tree[c + 1].begin = mid; tree[c + 1].end = e;
            next.push_back(c);
            next.push_back(c + 1);
        }
        level.swap(next);
        if (timing) {
            char buf[64];
            std::snprintf(buf, sizeof(buf), " %d:%d/%d/%.2f", depth, cnt, nbig,
                          std::chrono::duration<double, std::milli>(clk::now() - t_level).count());
            levels_report += buf;
        }
    }
    mark("levels");
    if (timing) std::fprintf(stderr, "gpu_build_bvh levels (depth:nodes/big/ms):%s\n", levels_report.c_str());
    BCHK(hipMemcpyAsync(h_idx.data(), idx.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    BCHK(hipStreamSynchronize(s));
    // node numbering of the reference's recursion: a split allocates its two children at the
    // end of the array, then its first child's subtree is split, then the second's
    std::vector<int> final_of(tree.size(), -1);
    final_of[0] = 0;
    int next_index = 1;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int x = stack.back();
        stack.pop_back();
        if (tree[x].child < 0) continue;
        final_of[tree[x].child] = next_index;
        final_of[tree[x].child + 1] = next_index + 1;
        next_index += 2;
        stack.push_back(tree[x].child + 1);    // second child's subtree after the first's
        stack.push_back(tree[x].child);
    }
    nodes.assign(tree.size(), rt_bvh_node{});
    for (size_t x = 0; x < tree.size(); x++) {
        const TreeNode &tn = tree[x];
        rt_bvh_node &nd = nodes[final_of[x]];
        nd.min_bound = {tn.lo[0], tn.lo[1], tn.lo[2]};
        nd.max_bound = {tn.hi[0], tn.hi[1], tn.hi[2]};
        if (tn.child >= 0) {
            nd.child1 = final_of[tn.child];
            nd.child2 = final_of[tn.child + 1];
        } else {
            nd.child2 = tn.begin;
            nd.child1 = tn.end;
        }
    }
    std::vector<rt_triangle> t2(tris.size());
    std::vector<uint16_t> m2(tris.size());
    for (int i = 0; i < n; i++) {
        t2[i] = tris[h_idx[i]];
        m2[i] = tri_mats[h_idx[i]];
    }
    tris.swap(t2);
    if (n) std::memcpy(tri_mats, m2.data(), n * sizeof(uint16_t));
    mark("numbering+permute");
    if (timing) std::fprintf(stderr, "gpu_build_bvh (%d triangles, %zu nodes):%s\n", n, nodes.size(), report.c_str());
    return RT_OK;
}

}  // namespace rtamd
