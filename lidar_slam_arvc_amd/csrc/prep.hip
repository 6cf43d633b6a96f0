// prep.hip -- KeyFrame.pre_process on the device (keyframe.py:113-124), batched over keyframes.
//
//   filter_radius_height  (keyframe.py:74-94)        : f64 strict mask + order-preserving compaction
//   voxel_down_sample     (keyframe.py:150-151)      : f64 Open3D voxel keys, stable sort, per-voxel
//                                                      sequential f64 mean (bit-exact with Open3D)
//   spatial index (replaces KDTreeFlann)             : cell keys -> radix sort -> dense CSR table
//   estimate_normals      (keyframe.py:160-162)      : hybrid radius / kNN-300 neighbourhoods,
//                                                      exact f64 distances, FastEigen3x3
//
// All kernels of a stage run over every keyframe of the batch in one launch (block tables map
// workgroups to (keyframe, first point)); the host synchronises only to learn data-dependent
// point counts (filter, voxel) and grid extents.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <type_traits>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <vector>

#include "fasteigen.h"
#include "lsm_ctx.h"

namespace {

constexpr int FILTER_THREADS = 256;
constexpr int FILTER_PER_THREAD = 4;
constexpr int FILTER_CHUNK = FILTER_THREADS * FILTER_PER_THREAD;
constexpr int PT_THREADS = 256;
constexpr int64_t MAX_CELLS_PER_CLOUD = int64_t(1) << 24;
// Default cell edge of the keyframe grid in x and z (m; y cells are half of it). With cubic cells
// (rounds 1-5) 0.375 m was best (round 1: 0.3 4136, 0.36 4308, 0.4 4336, 0.45 4177, 0.5 4028
// pairs/s); with the anisotropic cells of round 6 (profiles/r06/gridcell_ysub_sweep.txt) C3 runs
// 8727 / 9328 / 9445 pairs/s at 0.33 / 0.375 / 0.42 m and C4 6270 / 6995 / 7168 -- larger cells
// cost the walks (wider row windows), smaller ones push far queries into the fallback (its
// virtual blocks, 4 x-cells wide, shrink with the cell).
constexpr float LSM_DEFAULT_GRID_CELL = 0.42f;
constexpr float LSM_VOXEL_GRID_CELL_MIN = 0.75f;   // voxelised clouds (lsm_prep_batch)

struct Seg {           // (keyframe, first point) of one workgroup
    int32_t cloud;
    int32_t start;
};

// ------------------------------------------------------------------------------------------
// filter_radius_height: keep iff x^2+y^2 < maxr^2, > minr^2, z > minh, z < maxh (all strict,
// float64, no FMA contraction -- numpy evaluates x**2 + y**2 as two rounded products and a sum).
// ------------------------------------------------------------------------------------------
struct FilterParams {
    double maxr2, minr2, minh, maxh;
};

__device__ __forceinline__ bool keep_point(float x, float y, float z, const FilterParams &f) {
    double dx = x, dy = y, dz = z;
    double r2 = lsm_dadd(lsm_dmul(dx, dx), lsm_dmul(dy, dy));
    return (r2 < f.maxr2) & (r2 > f.minr2) & (dz > f.minh) & (dz < f.maxh);
}

__global__ void __launch_bounds__(FILTER_THREADS)
filter_count(const Seg *segs, const float *const *raw, const int32_t *nraw, FilterParams f,
             uint32_t *bcount) {
    const Seg s = segs[blockIdx.x];
    const float *p = raw[s.cloud];
    const int n = nraw[s.cloud];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < FILTER_PER_THREAD; ++k) {
        int i = s.start + k * FILTER_THREADS + threadIdx.x;
        if (i < n) c += keep_point(p[3 * i], p[3 * i + 1], p[3 * i + 2], f) ? 1u : 0u;
    }
    // wave sum then LDS across 4 waves
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, LSM_WAVE);
    __shared__ uint32_t ws[FILTER_THREADS / LSM_WAVE];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < FILTER_THREADS / LSM_WAVE; ++w) t += ws[w];
        bcount[blockIdx.x] = t;
    }
}

// Order-preserving compaction: within a block, points are handled in index order (k-major
// chunks of 256), ranks from wave ballots + LDS prefix of wave totals.
__global__ void __launch_bounds__(FILTER_THREADS)
filter_write(const Seg *segs, const float *const *raw, const int32_t *nraw, FilterParams f,
             const uint32_t *boff, float4 *out, uint32_t *src_index) {
    const Seg s = segs[blockIdx.x];
    const float *p = raw[s.cloud];
    const int n = nraw[s.cloud];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t wtot[FILTER_THREADS / LSM_WAVE];
    uint32_t base = boff[blockIdx.x];
    for (int k = 0; k < FILTER_PER_THREAD; ++k) {
        int i = s.start + k * FILTER_THREADS + threadIdx.x;
        float x = 0.f, y = 0.f, z = 0.f;
        bool keep = false;
        if (i < n) {
            x = p[3 * i];
            y = p[3 * i + 1];
            z = p[3 * i + 2];
            keep = keep_point(x, y, z, f);
        }
        uint64_t m = __ballot(keep);
        uint32_t below = __popcll(m & ((uint64_t(1) << lane) - 1));
        if (lane == 0) wtot[wave] = __popcll(m);
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (int w = 0; w < FILTER_THREADS / LSM_WAVE; ++w) {
            woff += (w < wave) ? wtot[w] : 0u;
            tot += wtot[w];
        }
        if (keep) {
            uint32_t o = base + woff + below;
            out[o] = make_float4(x, y, z, 0.f);
            src_index[o] = uint32_t(i);
        }
        base += tot;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// bounding boxes (f64 for the voxel grid, f32 values are exact in f64)
// ------------------------------------------------------------------------------------------
// Several workgroups per cloud (one workgroup per cloud left the GPU mostly idle: 0.22 ms per
// 257-cloud batch): wave min / max in f32, then one atomic per wave on order-preserving u32 keys
// (bbk: 6 per cloud, min slots start at ~0, max slots at 0); bbox_final turns them into the f64
// box (f32 values are exact in f64). Min / max are order-independent, so the box is the same.
constexpr int BBOX_BLOCKS = 16;   // workgroups per cloud
__device__ __forceinline__ uint32_t f32_key(float v) {
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_f32(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void __launch_bounds__(256)
bbox_kernel(const float4 *pts, const uint32_t *cloud_off, const uint32_t *cloud_n, uint32_t *bbk) {
    const int c = blockIdx.x;
    const uint32_t off = cloud_off[c], n = cloud_n[c];
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = blockIdx.y * blockDim.x + threadIdx.x; i < n; i += gridDim.y * blockDim.x) {
        const float4 p = pts[off + i];
        mn[0] = fminf(mn[0], p.x);
        mn[1] = fminf(mn[1], p.y);
        mn[2] = fminf(mn[2], p.z);
        mx[0] = fmaxf(mx[0], p.x);
        mx[1] = fmaxf(mx[1], p.y);
        mx[2] = fmaxf(mx[2], p.z);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], o, LSM_WAVE));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], o, LSM_WAVE));
        }
    if ((threadIdx.x & 63) == 0 && mn[0] <= mx[0]) {
        for (int k = 0; k < 3; ++k) {
            atomicMin(bbk + 6 * c + k, f32_key(mn[k]));
            atomicMax(bbk + 6 * c + 3 + k, f32_key(mx[k]));
        }
    }
}

__global__ void bbox_init(uint32_t *bbk, int K) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 6 * K) bbk[i] = (i % 6) < 3 ? 0xffffffffu : 0u;
}

// an empty cloud keeps (+inf, -inf) as the one-workgroup kernel left it
__global__ void bbox_final(const uint32_t *bbk, int K, double *bb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 6 * K) return;
    const uint32_t k = bbk[i];
    const bool lo = (i % 6) < 3;
    bb[i] = (lo && k == 0xffffffffu) ? INFINITY : ((!lo && k == 0u) ? -INFINITY : double(key_f32(k)));
}

// per-cloud (off, cnt) of the filter's output from its block offsets (no host round trip)
__global__ void filter_cloud_ranges(const uint32_t *boff, const int32_t *first_block,
                                    const int32_t *nblocks, int K, uint32_t *off, uint32_t *cnt) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int f = first_block[k], nb = nblocks[k];
    off[k] = nb ? boff[f] : 0u;
    cnt[k] = nb ? boff[f + nb] - boff[f] : 0u;
}

// per-cloud (off, cnt) of the voxel centroids from the clouds' first voxel ids vb[0 .. K]
__global__ void vox_cloud_ranges(const uint32_t *vb, int K, uint32_t *off, uint32_t *cnt) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    off[k] = vb[k] - vb[0];
    cnt[k] = vb[k + 1] - vb[k];
}

// bb[6 k .. 6 k + 6) = (min xyz, max xyz) of cloud k
int run_bbox(lsm_ctx *ctx, const float4 *pts, const uint32_t *d_off, const uint32_t *d_cnt, int K,
             double *d_bb, const char *name) {
    hipStream_t st = ctx->stream;
    uint32_t *bbk = (uint32_t *)ctx->buf(name, size_t(K) * 24 + 4);
    if (!bbk) return LSM_ENOMEM;
    const int g = (6 * K + 255) / 256;
    bbox_init<<<g, 256, 0, st>>>(bbk, K);
    bbox_kernel<<<dim3(K, BBOX_BLOCKS), 256, 0, st>>>(pts, d_off, d_cnt, bbk);
    bbox_final<<<g, 256, 0, st>>>(bbk, K, d_bb);
    return LSM_OK;
}

// ------------------------------------------------------------------------------------------
// voxel_down_sample ([O3D] PointCloud::VoxelDownSample)
// ------------------------------------------------------------------------------------------
struct VoxGeo {         // per cloud, computed on the host from the f64 bbox
    double ox, oy, oz;  // voxel_min_bound = min_bound - v/2
    int64_t dx, dy, dz; // key extents
    uint64_t key_off;   // offset of this cloud in the global key space
};

// ref_coord = (p - voxel_min_bound) / voxel_size ; voxel_index = int(floor(ref_coord)), as a key in
// the batch's key space
__device__ __forceinline__ uint64_t voxel_key(float4 p, const VoxGeo &G, double v) {
    const int64_t kx = (int64_t)(int)floor(lsm_ddiv(lsm_dsub((double)p.x, G.ox), v));
    const int64_t ky = (int64_t)(int)floor(lsm_ddiv(lsm_dsub((double)p.y, G.oy), v));
    const int64_t kz = (int64_t)(int)floor(lsm_ddiv(lsm_dsub((double)p.z, G.oz), v));
    return G.key_off + uint64_t((kx * G.dy + ky) * G.dz + kz);
}

// Per point: its voxel key, and whether it starts a run -- a maximal stretch of consecutive points
// (index order) in one voxel. A scan's consecutive points are neighbours on the sensor's rings, so
// runs are long (Ouster-128 at 0.4 / 0.2 / 0.1 m: 7.3 / 3.6 / 2.2 points on average) and the
// grouping sorts runs, not points. A cloud's first point starts a run (key spaces are disjoint).
// KeyT: uint32_t when the batch's key space fits 32 bits (4 radix passes over 4-byte keys)
template <typename KeyT>
__global__ void __launch_bounds__(PT_THREADS)
voxel_keys(const Seg *segs, const float4 *pts, const uint32_t *cloud_off, const uint32_t *cloud_n,
           const VoxGeo *geo, double v, KeyT *keys, uint32_t *run_head) {
    __shared__ KeyT sk[PT_THREADS];
    const Seg s = segs[blockIdx.x];
    const int t = threadIdx.x, i = s.start + t;
    const bool valid = i < int(cloud_n[s.cloud]);
    const uint32_t g = cloud_off[s.cloud] + i;
    const VoxGeo G = geo[s.cloud];
    KeyT key = 0;
    if (valid) {
        key = KeyT(voxel_key(pts[g], G, v));
        keys[g] = key;
    }
    sk[t] = key;
    __syncthreads();
    if (!valid) return;
    bool head;
    if (i == 0) head = true;
    else if (t > 0) head = sk[t - 1] != key;
    else head = KeyT(voxel_key(pts[g - 1], G, v)) != key;
    run_head[g] = head ? 1u : 0u;
}

// run heads -> (run key, run start): rid = exclusive scan of the heads; rstart[nruns] = n
template <typename KeyT>
__global__ void __launch_bounds__(PT_THREADS)
voxel_runs(const KeyT *keys, const uint32_t *run_head, const uint32_t *rid, uint32_t n, KeyT *rkeys,
           uint32_t *rstart) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    if (run_head[g]) {
        const uint32_t r = rid[g];
        rkeys[r] = keys[g];
        rstart[r] = g;
    }
    if (g == 0) rstart[rid[n]] = n;
}

// One thread per sorted run; voxel heads sum their members in index order (the stable sort keeps
// a voxel's runs in index order) exactly like AccumulatedPoint::AddPoint.
template <typename KeyT>
__global__ void __launch_bounds__(PT_THREADS)
voxel_flags(const KeyT *skeys, uint32_t n, uint32_t *flag) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flag[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}

// vstart[vid[i]] = i for every voxel head i, and vstart[nvox] = n: voxel o's members are the
// sorted entries [vstart[o], vstart[o + 1])
__global__ void __launch_bounds__(PT_THREADS)
voxel_heads(const uint32_t *flag, const uint32_t *vid_excl, uint32_t n, uint32_t *vstart) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (flag[i]) vstart[vid_excl[i]] = i;
    if (i == 0) vstart[vid_excl[n]] = n;
}

// Adds pts[b .. e) to the sums in index order (a run of one voxel), its loads BATCH / 4 at a time
// (the run's length is known, so the loads need not wait for the run-end test).
template <int BATCH>
__device__ __forceinline__ void add_run(const float4 *pts, uint32_t b, uint32_t e, double &sx, double &sy,
                                        double &sz) {
    uint32_t j = b;
    for (; j + BATCH <= e; j += BATCH) {
        float4 p[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) p[u] = pts[j + u];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            sx = lsm_dadd(sx, (double)p[u].x);
            sy = lsm_dadd(sy, (double)p[u].y);
            sz = lsm_dadd(sz, (double)p[u].z);
        }
    }
    for (; j + 4 <= e; j += 4) {
        const float4 p0 = pts[j], p1 = pts[j + 1], p2 = pts[j + 2], p3 = pts[j + 3];
        sx = lsm_dadd(lsm_dadd(lsm_dadd(lsm_dadd(sx, (double)p0.x), (double)p1.x), (double)p2.x), (double)p3.x);
        sy = lsm_dadd(lsm_dadd(lsm_dadd(lsm_dadd(sy, (double)p0.y), (double)p1.y), (double)p2.y), (double)p3.y);
        sz = lsm_dadd(lsm_dadd(lsm_dadd(lsm_dadd(sz, (double)p0.z), (double)p1.z), (double)p2.z), (double)p3.z);
    }
    for (; j < e; ++j) {
        const float4 p = pts[j];
        sx = lsm_dadd(sx, (double)p.x);
        sy = lsm_dadd(sy, (double)p.y);
        sz = lsm_dadd(sz, (double)p.z);
    }
}

// run bounds loaded per batch (the next batch's loads are issued before this batch's points are
// summed, so a voxel of many runs does not wait on its run table run by run)
#ifndef LSM_VOX_RUN_BATCH
#define LSM_VOX_RUN_BATCH 8
#endif
constexpr uint32_t VOX_RUN_BATCH = LSM_VOX_RUN_BATCH;

// A wave of voxel_reduce takes as long as its voxel of most runs (one dependent chain each), and
// voxels of many runs are scattered among the small ones (near the sensor: at 0.4 m on an
// Ouster-128 scan 5 % of the voxels hold half the points, and nearly every wave of 64 consecutive
// voxels would hold one). voxel_order lists the voxels of more than VOX_RUN_BATCH runs first and
// the others after them (each class in voxel order: positions from a scan of the wide flags), so
// the long chains share their waves and the rest finish fast; the results do not depend on the
// order (each voxel's sums are its own thread's).
__global__ void __launch_bounds__(PT_THREADS)
voxel_wide(const uint32_t *vid_excl, const uint32_t *vstart, uint32_t nruns, uint32_t *wide) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nvox = vid_excl[nruns];
    if (o < nvox) wide[o] = vstart[o + 1] - vstart[o] > VOX_RUN_BATCH ? 1u : 0u;
    else if (o == nvox) wide[o] = 0u;
}

__global__ void __launch_bounds__(PT_THREADS)
voxel_order(const uint32_t *vid_excl, const uint32_t *wide, const uint32_t *wide_excl, uint32_t nruns,
            uint32_t *order) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nvox = vid_excl[nruns];
    if (o >= nvox) return;
    const uint32_t w = wide_excl[o];
    order[wide[o] ? w : wide_excl[nvox] + (o - w)] = o;
}

// One thread per voxel, in voxel_order's order (the grid covers the runs; threads past the voxel
// count exit): the voxel's runs in index order, each run's points in index order -- the left fold
// in f64 of AccumulatedPoint::AddPoint over the members.
template <typename KeyT>
__global__ void __launch_bounds__(PT_THREADS)
voxel_reduce(const KeyT *skeys, const uint32_t *srun, const uint32_t *rstart, const uint32_t *vid_excl,
             const uint32_t *vstart, const uint32_t *order, uint32_t nruns, const float4 *pts,
             const int32_t *pt_cloud, const VoxGeo *geo, double *cent, int32_t *vkeys, float4 *vpts,
             int32_t *vcloud) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= vid_excl[nruns]) return;
    const uint32_t o = order[t];
    const uint32_t q0 = vstart[o], q1 = vstart[o + 1];
    double sx = 0.0, sy = 0.0, sz = 0.0;
    uint32_t count = 0;
    uint32_t rb[VOX_RUN_BATCH], re[VOX_RUN_BATCH];
    auto load_batch = [&](uint32_t q) {
#pragma unroll
        for (uint32_t u = 0; u < VOX_RUN_BATCH; ++u) {
            rb[u] = re[u] = 0;
            if (q + u < q1) {
                const uint32_t r = srun[q + u];
                rb[u] = rstart[r];
                re[u] = rstart[r + 1];
            }
        }
    };
    load_batch(q0);
    const uint32_t first = rb[0];
    for (uint32_t q = q0; q < q1; q += VOX_RUN_BATCH) {
        uint32_t cb[VOX_RUN_BATCH], ce[VOX_RUN_BATCH];
#pragma unroll
        for (uint32_t u = 0; u < VOX_RUN_BATCH; ++u) {
            cb[u] = rb[u];
            ce[u] = re[u];
        }
        if (q + VOX_RUN_BATCH < q1) load_batch(q + VOX_RUN_BATCH);
#pragma unroll
        for (uint32_t u = 0; u < VOX_RUN_BATCH; ++u) {
            count += ce[u] - cb[u];
            add_run<8>(pts, cb[u], ce[u], sx, sy, sz);
        }
    }
    const uint64_t key = uint64_t(skeys[q0]);
    const double cnt = double(count);
    const double cx = lsm_ddiv(sx, cnt), cy = lsm_ddiv(sy, cnt), cz = lsm_ddiv(sz, cnt);
    cent[3 * o] = cx;
    cent[3 * o + 1] = cy;
    cent[3 * o + 2] = cz;
    const int c = pt_cloud[first];
    const VoxGeo G = geo[c];
    const uint64_t local = key - G.key_off;
    const int64_t kz = int64_t(local % uint64_t(G.dz));
    const int64_t ky = int64_t((local / uint64_t(G.dz)) % uint64_t(G.dy));
    const int64_t kx = int64_t(local / uint64_t(G.dz * G.dy));
    vkeys[3 * o] = int32_t(kx);
    vkeys[3 * o + 1] = int32_t(ky);
    vkeys[3 * o + 2] = int32_t(kz);
    vpts[o] = make_float4(float(cx), float(cy), float(cz), 0.f);
    vcloud[o] = c;
}

// vb[k] = vid[rid[pstart[k]]]: the first voxel id of cloud k (k = K: the voxel total); the sort
// keeps each cloud's runs together (key_off), so cloud k's sorted runs start at its first run id
__global__ void vox_cloud_bounds(const uint32_t *vid, const uint32_t *rid, const uint32_t *pstart, int n,
                                 uint32_t *vb) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) vb[k] = vid[rid[pstart[k]]];
}

// voxel o's f64 centroid and int32 key into its cloud's arrays (voff: the cloud's first voxel)
__global__ void vox_scatter(const double *cent, const int32_t *vkeys, const int32_t *vcloud,
                            uint32_t nvox, const uint32_t *voff, double *const *cp,
                            int32_t *const *kp) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nvox) return;
    const int c = vcloud[o];
    const uint32_t l = o - voff[c];
    double *dc = cp[c] + size_t(l) * 3;
    int32_t *dk = kp[c] + size_t(l) * 3;
    dc[0] = cent[3 * size_t(o)];
    dc[1] = cent[3 * size_t(o) + 1];
    dc[2] = cent[3 * size_t(o) + 2];
    dk[0] = vkeys[3 * size_t(o)];
    dk[1] = vkeys[3 * size_t(o) + 1];
    dk[2] = vkeys[3 * size_t(o) + 2];
}

__global__ void point_cloud_ids(const uint32_t *cloud_off, const uint32_t *cloud_n, int ncloud,
                                int32_t *pt_cloud) {
    int c = blockIdx.y;
    if (c >= ncloud) return;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cloud_n[c];
         i += gridDim.x * blockDim.x)
        pt_cloud[cloud_off[c] + i] = c;
}

// ------------------------------------------------------------------------------------------
// spatial index: global cell key per point, radix sort, gather, dense CSR cell table
// ------------------------------------------------------------------------------------------
struct GridGeo {
    float ox, oy, oz, cell, inv_cell;
    float cell_y, inv_cell_y;   // y cells: cell / LSM_YSUB
    int nx, ny, nz;
    int nbx, nby, nbz;
    uint32_t cell_off;     // offset of this cloud in its sort group's cell key space (31 bits)
    uint32_t pt_off;       // offset of this cloud in the batch point arrays
    uint32_t n;
    uint32_t ncells;       // nbx * nby * nbz * LSM_BLK_CELLS (blocked, padded)
};

__device__ __forceinline__ int cell_coord(float v, float o, float inv, int nmax) {
    return lsm_clampi((int)floorf((v - o) * inv), 0, nmax - 1);
}

// x as an order-preserving u32 (IEEE sign flip)
__device__ __forceinline__ uint32_t x_key(float x) {
    const uint32_t xb = __float_as_uint(x);
    return (xb & 0x80000000u) ? ~xb : (xb | 0x80000000u);
}

__global__ void __launch_bounds__(PT_THREADS)
grid_keys(const Seg *segs, const float4 *pts, const GridGeo *geo, uint64_t *keys,
          uint32_t *vals) {
    const Seg s = segs[blockIdx.x];
    const GridGeo G = geo[s.cloud];
    const int i = s.start + threadIdx.x;
    if (i >= int(G.n)) return;
    const uint32_t g = G.pt_off + i;
    float4 p = pts[g];
    int cx = cell_coord(p.x, G.ox, G.inv_cell, G.nx);
    int cy = cell_coord(p.y, G.oy, G.inv_cell_y, G.ny);
    int cz = cell_coord(p.z, G.oz, G.inv_cell, G.nz);
    // (cell, x) key: inside a cell points are ordered by x, which lets the correspondence search
    // walk a cell outwards from the query's x and stop once dx^2 exceeds the best distance
    keys[g] = (uint64_t(G.cell_off + uint32_t(lsm_cell_lin(G.nbx, G.nby, cx, cy, cz))) << 32) |
              x_key(p.x);
    vals[g] = g;
}

__global__ void __launch_bounds__(PT_THREADS)
grid_scatter(const Seg *segs, const GridGeo *geo, const CloudDev *cd, const uint32_t *svals,
             const float4 *pts, uint32_t *const *perm_out) {
    const Seg s = segs[blockIdx.x];
    const GridGeo G = geo[s.cloud];
    const int j = s.start + threadIdx.x;
    if (j < int(G.n)) {
        const uint32_t g = G.pt_off + j;
        const uint32_t v = svals[g];
        float4 *xyz = const_cast<float4 *>(cd[s.cloud].xyz);
        xyz[j] = pts[v];
        perm_out[s.cloud][j] = v - G.pt_off;   // reference (filter / voxel-key) order
    }
}

// cell_start[c] = first sorted position with key >= c (lower bound), for c in [0, ncells].
// One workgroup per tile of FILL_TILE cells: two binary searches bound the tile's points
// [p0, p1); every cell starts at p1, each cell's first point writes its own position, and a
// backward min-scan hands empty cells the start of the next occupied one. Keys are read once
// and the table is written once, coalesced.
constexpr int FILL_THREADS = 256;
constexpr int FILL_PER = 16;
constexpr int FILL_TILE = FILL_THREADS * FILL_PER;

__device__ __forceinline__ uint32_t lower_bound_cell(const uint64_t *k, uint32_t n, uint32_t target) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uint32_t(k[mid] >> 32) < target) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(FILL_THREADS)
grid_fill(const GridGeo *geo, int ncloud, const uint64_t *skeys, uint32_t *const *cell_out,
          uint32_t *const *bm_out, uint32_t *nonempty) {
    static_assert(FILL_THREADS == 256 && FILL_TILE % LSM_BLK_CELLS == 0, "virtual-block bits");
    __shared__ uint32_t tile[FILL_TILE];
    __shared__ uint32_t bounds[2];
    __shared__ uint32_t wmin[FILL_THREADS / LSM_WAVE];
    __shared__ uint32_t vbits[FILL_THREADS / LSM_WAVE];
    const int c = blockIdx.y;
    if (c >= ncloud) return;
    const GridGeo G = geo[c];
    const int64_t ncells1 = int64_t(G.ncells) + 1;
    uint32_t *out = cell_out[c];
    const uint64_t *k = skeys + G.pt_off;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t c0 = int64_t(blockIdx.x) * FILL_TILE; c0 < ncells1;
         c0 += int64_t(gridDim.x) * FILL_TILE) {
        const int64_t c1 = c0 + FILL_TILE < ncells1 ? c0 + FILL_TILE : ncells1;
        if (threadIdx.x < 2)
            bounds[threadIdx.x] = lower_bound_cell(k, G.n, G.cell_off + uint32_t(threadIdx.x ? c1 : c0));
        __syncthreads();
        const uint32_t p0 = bounds[0], p1 = bounds[1];
        for (int e = threadIdx.x; e < FILL_TILE; e += FILL_THREADS) tile[e] = p1;
        __syncthreads();
        uint32_t heads = 0;   // occupied cells of the tile (the cloud's count: bench bytes)
        for (uint32_t j = p0 + threadIdx.x; j < p1; j += FILL_THREADS) {
            const uint32_t cj = uint32_t(k[j] >> 32);
            if (j == 0 || uint32_t(k[j - 1] >> 32) != cj) {
                tile[cj - G.cell_off - uint32_t(c0)] = j;
                ++heads;
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) heads += __shfl_xor(heads, off, LSM_WAVE);
        if (lane == 0 && heads) atomicAdd(&nonempty[c], heads);
        __syncthreads();
        // backward min-scan: thread t owns cells [16 t, 16 t + 16)
        uint32_t v[FILL_PER];
        uint32_t m = 0xffffffffu;
#pragma unroll
        for (int i = FILL_PER - 1; i >= 0; --i) {
            v[i] = tile[threadIdx.x * FILL_PER + i];
            m = min(m, v[i]);
        }
        // minimum over the threads after this one (exclusive suffix), wave then workgroup
        uint32_t suf = m;
#pragma unroll
        for (int off = 1; off < LSM_WAVE; off <<= 1) {
            const uint32_t o = __shfl_down(suf, off, LSM_WAVE);
            if (lane + off < LSM_WAVE) suf = min(suf, o);
        }
        if (lane == 0) wmin[w] = suf;
        __syncthreads();
        uint32_t after = __shfl_down(suf, 1, LSM_WAVE);
        if (lane == LSM_WAVE - 1) after = 0xffffffffu;
        for (int q = w + 1; q < FILL_THREADS / LSM_WAVE; ++q) after = min(after, wmin[q]);
        after = min(after, p1);
        uint32_t run = after;
#pragma unroll
        for (int i = FILL_PER - 1; i >= 0; --i) {
            run = min(run, v[i]);
            v[i] = run;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FILL_PER; ++i) tile[threadIdx.x * FILL_PER + i] = v[i];
        __syncthreads();
        for (int e = threadIdx.x; e < FILL_TILE; e += FILL_THREADS)
            if (c0 + e < c1) out[c0 + e] = tile[e];
        // occupancy bits of the tile's FILL_VB virtual blocks (4 x LSM_BLKY x 4 cells; bit v =
        // layout block v >> VBS, x-chunk v & (LSM_BLKX / 4 - 1)): TPV threads per virtual block,
        // thread t tests 4 of its rows (row r = 4 (t % TPV) + i: z r / LSM_BLKY, y r % LSM_BLKY)
        {
            constexpr int VBS = LSM_BLKX_SHIFT - 2;
            constexpr int FILL_VB = FILL_TILE / LSM_VB_CELLS;   // 64 (cubic cells) or 32
            constexpr int TPV = FILL_THREADS / FILL_VB;          // 4 or 8
            constexpr int BPW = LSM_WAVE / TPV;                  // virtual blocks per wave
            static_assert(TPV * 4 == LSM_VB_ROWS && FILL_VB % 32 == 0, "virtual-block bits");
            const uint32_t vb = threadIdx.x / TPV, ti = threadIdx.x % TPV;
            const uint32_t v = uint32_t(c0 / LSM_VB_CELLS) + vb;
            const int64_t cell0 = int64_t(v >> VBS) * LSM_BLK_CELLS +
                                  ((v & ((1u << VBS) - 1u)) << 2) - c0;
            bool occ = false;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = int(ti) * 4 + i;
                const int64_t e0 = cell0 + (r / LSM_BLKY) * LSM_BLKY * LSM_BLKX +
                                   (r % LSM_BLKY) * LSM_BLKX, e1 = e0 + 4;
                const uint32_t a = tile[e0], b = e1 < FILL_TILE ? tile[e1] : p1;
                occ |= b > a;
            }
            uint64_t m = __ballot(occ);
#pragma unroll
            for (int sh = 1; sh < TPV; sh <<= 1) m |= m >> sh;   // bit TPV j: block j of the wave
            uint32_t bits = 0;
#pragma unroll
            for (int j = 0; j < BPW; ++j) bits |= uint32_t((m >> (TPV * j)) & 1u) << j;
            if (lane == 0) vbits[w] = bits;
            __syncthreads();
            constexpr int WPT = FILL_VB / 32;   // bit-mask words per tile
            if (threadIdx.x < WPT) {
                uint32_t word = 0;
#pragma unroll
                for (int q = 0; q < 32 / BPW; ++q)
                    word |= vbits[threadIdx.x * (32 / BPW) + q] << (q * BPW);
                bm_out[c][(c0 / FILL_TILE) * WPT + threadIdx.x] = word;
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// normals: KDTreeSearchParamHybrid(radius, max_nn) neighbourhoods on the cell grid
// ------------------------------------------------------------------------------------------
struct NormalParams {
    double r2;        // radius^2 in f64 (Open3D compares d^2 < radius*radius)
    float r;          // radius (search box half-width)
    float r2_lo;      // f32 d^2 below this: certainly inside (exact f64 test not needed)
    float r2_hi;      // f32 d^2 above this: certainly outside
    float hscale;     // f32 of the level-0 histogram scale NB8 / r^2 (see normals_kernel)
    int max_nn;
    float dense_k;    // own cell holds >= dense_k * cell^2 points: predicted > max_nn neighbours
                      // (0: off)
    int preclass;     // final pass: f32 pre-classification (0: every point takes the f64 test)
};

// Offsets of a candidate from the query in f64 (exact: both are f32 values) with their squares,
// and the exact nanoflann d^2 = ((dx^2 + dy^2) + dz^2) built from the same products
// (lsm_sqdist64 bit for bit: (p - q)^2 == (q - p)^2).
struct Off {
    double dx, dy, dz, xx, yy, zz, d2;
};

__device__ __forceinline__ Off make_off(float4 p, double qx, double qy, double qz) {
    Off o;
    o.dx = lsm_dsub((double)p.x, qx);
    o.dy = lsm_dsub((double)p.y, qy);
    o.dz = lsm_dsub((double)p.z, qz);
    o.xx = lsm_dmul(o.dx, o.dx);
    o.yy = lsm_dmul(o.dy, o.dy);
    o.zz = lsm_dmul(o.dz, o.dz);
    o.d2 = lsm_dadd(lsm_dadd(o.xx, o.yy), o.zz);
    return o;
}

__device__ __forceinline__ float f32_d2(float4 q, float4 p) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    return dx * dx + dy * dy + dz * dz;
}

// d^2 < r^2 decided exactly as the f64 reference does: the f32 estimate (relative error
// < 4e-7 for f32 inputs) settles every point farther than 4e-6 relative from the sphere; the
// rest take the exact f64 value. The f64 offsets are computed once and shared with the
// cumulants and the selection binning.
__device__ __forceinline__ bool in_ball(const NormalParams &np, float4 q, double qx, double qy,
                                        double qz, float4 p, Off &o) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    const float f = dx * dx + dy * dy + dz * dz;
    if (f > np.r2_hi) return false;
    o = make_off(p, qx, qy, qz);
    return f < np.r2_lo || o.d2 < np.r2;
}

// Covariance from centred cumulants (mathematically identical to Open3D's raw cumulants;
// centring on the query point avoids f64 cancellation at 35 m coordinates).
struct Cum {
    double sx, sy, sz, sxx, sxy, sxz, syy, syz, szz;
    int n;
};

// Cumulants from the exact f64 offsets of a point (f32 coordinates: the differences are exact).
// f32 sums were tried: they move some normals by ~1e-6, which is enough to shift chaotic
// (non-converging) registrations past the transform parity bar.
__device__ __forceinline__ void cum_add_pt(Cum &c, float4 p, double qx, double qy, double qz) {
    const double dx = double(p.x) - qx, dy = double(p.y) - qy, dz = double(p.z) - qz;
    c.sx += dx;
    c.sy += dy;
    c.sz += dz;
    c.sxx = fma(dx, dx, c.sxx);
    c.syy = fma(dy, dy, c.syy);
    c.szz = fma(dz, dz, c.szz);
    c.sxy = fma(dx, dy, c.sxy);
    c.sxz = fma(dx, dz, c.sxz);
    c.syz = fma(dy, dz, c.syz);
    c.n += 1;
}

// Neighbourhoods of at most NSMALL points take Open3D's own covariance arithmetic (small_normal,
// small_normal_from_list): normal_from_cum only marks them (w = 1) for that step.
// (8: headline parity 1999 / 1999 as with 16, the small-neighbourhood pass 2 ms per C3 step
// instead of 11: DESIGN.md §7)
#ifndef LSM_NSMALL
#define LSM_NSMALL 8
#endif
constexpr int NSMALL = LSM_NSMALL;
// the sparse half keeps the first members of each neighbourhood (LDS: 8 slots keep it at 8 waves
// per SIMD) and finishes every small neighbourhood from them without a second walk; there is no
// other pass for the sparse half's small ones, so NSMALL may not exceed what it keeps
constexpr int NSMALL_INLINE = NSMALL;
static_assert(NSMALL >= 3 && NSMALL <= 8,
              "the sparse half finishes neighbourhoods of 3..NSMALL points from the <= 8 members "
              "its scan 1 keeps in LDS");

// The normal of covariance A. prior (nullable): EstimateNormals on a cloud that already has
// normals -- a zero normal keeps the prior one, and the new normal is flipped when it points
// against the prior.
__device__ __forceinline__ float4 normal_from_cov(const sym3 &A, const float4 *prior, float w) {
    d3 v = fast_eigen3x3_min(A);
    if (sqrt(d3_dot(v, v)) == 0.0) {
        if (prior) return make_float4(prior->x, prior->y, prior->z, w);
        v = {0.0, 0.0, 1.0};
    }
    if (prior && v.x * double(prior->x) + v.y * double(prior->y) + v.z * double(prior->z) < 0.0)
        v = {-v.x, -v.y, -v.z};
    return make_float4(float(v.x), float(v.y), float(v.z), w);
}

__device__ __forceinline__ float4 normal_from_cum(const Cum &c, const float4 *prior = nullptr) {
    // a small neighbourhood only gets the mark: the kernel's small-normal step computes it
    if (c.n >= 3 && c.n <= NSMALL) return make_float4(0.f, 0.f, 0.f, 1.f);
    sym3 A;
    if (c.n >= 3) {
        const double inv = 1.0 / double(c.n);
        const double mx = c.sx * inv, my = c.sy * inv, mz = c.sz * inv;
        A.a00 = c.sxx * inv - mx * mx;
        A.a11 = c.syy * inv - my * my;
        A.a22 = c.szz * inv - mz * mz;
        A.a01 = c.sxy * inv - mx * my;
        A.a02 = c.sxz * inv - mx * mz;
        A.a12 = c.syz * inv - my * mz;
    } else {
        A = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    }
    return normal_from_cov(A, prior, 0.f);
}

// Cell range of [q - h, q + h] along one axis, widened by a small margin so every point within
// L-inf distance h is covered despite f32 rounding of the cell coordinate.
__device__ __forceinline__ void axis_range(float q, float o, float inv, float h, int nmax, int &lo,
                                           int &hi) {
    float a = (q - o) * inv;
    float hh = h * inv;
    lo = (int)floorf(a - hh - 1e-3f);
    hi = (int)floorf(a + hh + 1e-3f);
    lo = lo < 0 ? 0 : lo;
    hi = hi > nmax - 1 ? nmax - 1 : hi;
}

// squared distance from coordinate q to the cell slab [o + k*c, o + (k+1)*c) (0 inside)
__device__ __forceinline__ float slab_d2(float q, float o, float c, int k) {
    float lo = o + k * c, hi = lo + c;
    float d = q < lo ? lo - q : (q > hi ? q - hi : 0.f);
    return d * d;
}

// Visit the point ranges of the cells a radius-r ball around q can touch: rows of cells pruned by
// their slab distance, each row split at block boundaries into contiguous runs f(a, b, xl, xh).
// A run is sorted by x (cells of a row are x-ordered and each cell is x-sorted; the f32 cell
// index is monotone in x), and every ball point of the row has xl <= x <= xh (the chord of the
// row's nearest slab, widened for f32 rounding), so f may skip x < xl and stop at x > xh.
template <typename F>
__device__ __forceinline__ void ball_visit_runs(const CloudDev &C, float4 qf, float r, F &&f) {
    int xlo, xhi, ylo, yhi, zlo, zhi;
    axis_range(qf.x, C.ox, C.inv_cell, r, C.nx, xlo, xhi);
    axis_range(qf.y, C.oy, C.inv_cell_y, r, C.ny, ylo, yhi);
    axis_range(qf.z, C.oz, C.inv_cell, r, C.nz, zlo, zhi);
    const float prune = r * 1.0001f + 1e-6f;
    const float prune2 = prune * prune;
    for (int z = zlo; z <= zhi; ++z) {
        const float dz2 = slab_d2(qf.z, C.oz, C.cell, z);
        if (dz2 > prune2) continue;
        for (int y = ylo; y <= yhi; ++y) {
            const float dyz2 = dz2 + slab_d2(qf.y, C.oy, C.cell_y, y);
            if (dyz2 > prune2) continue;
            const float ch = sqrtf(prune2 - dyz2) * 1.0001f + 1e-6f * fabsf(qf.x) + 1e-5f;
            const float xl = qf.x - ch, xh = qf.x + ch;
            int x = xlo;
            while (x <= xhi) {
                const int xe = min(xhi, x | (LSM_BLKX - 1));   // end of this block's row part
                const int l0 = lsm_cell_lin(C.nbx, C.nby, x, y, z);
                const int l1 = lsm_cell_lin(C.nbx, C.nby, xe, y, z);
                const uint32_t a = lsm_ld(C.cell_start, l0), b = lsm_ld(C.cell_start, l1 + 1);
                if (b > a) f(a, b, xl, xh);
                x = xe + 1;
            }
        }
    }
}

// One x-sorted run [a, b) of a row with its window [xl, xh]: body(p, k) for every point in the
// window. Long runs find the window's first point by binary search on x (a run averages ~140
// points of which ~30 lie left of the window on HDL-64 scans); the walk stops past xh.
#ifndef LSM_SCAN_BSEARCH
#define LSM_SCAN_BSEARCH 16
#endif
#ifndef LSM_SCAN_SLACK
#define LSM_SCAN_SLACK 8
#endif
constexpr uint32_t SCAN_BSEARCH = LSM_SCAN_BSEARCH;
constexpr uint32_t SCAN_SLACK = LSM_SCAN_SLACK;   // scan_run_pred: entry search stops within this many points
// points per load group of the normals walks, and whether the next group's loads are issued
// before the current group is tested (measured per 65 keyframes: G4 6.65 ms, G2 + prefetch 6.43,
// G4 + prefetch 7.57 -- the extra registers cost occupancy)
#ifndef LSM_NORMALS_G_DEFAULT
#define LSM_NORMALS_G_DEFAULT 2
#endif
constexpr int NORMALS_G_DEFAULT = LSM_NORMALS_G_DEFAULT;
#ifndef LSM_NORMALS_GD_DEFAULT
#define LSM_NORMALS_GD_DEFAULT 4   // dense half, round 4 A/B: 2 / 3 / 4 -> 154.7 / 151.8 / 150.7 ms
#endif
constexpr int NORMALS_GD_DEFAULT = LSM_NORMALS_GD_DEFAULT;
#ifndef LSM_NORMALS_PF
#define LSM_NORMALS_PF 1
#endif
// the dense half of the split launch (LDS-bound occupancy: registers to spare) may pipeline
// over two register buffers (2)
#ifndef LSM_NORMALS_PFD
#define LSM_NORMALS_PFD LSM_NORMALS_PF
#endif

template <int G, typename Body>
__device__ __forceinline__ void scan_run(const float4 *xyz, uint32_t a, uint32_t b, float xl, float xh,
                                         Body &&body) {
    if (b - a > SCAN_BSEARCH) {
        uint32_t lo = a, hi = b;
        const float *xs = reinterpret_cast<const float *>(xyz);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (lsm_ld(xs, size_t(mid) * 4) < xl) lo = mid + 1;
            else hi = mid;
        }
        a = lo;
    }
    if (a >= b) return;
    if (G == 1) {
        float4 p = lsm_ld(xyz, a);
        for (uint32_t k = a; k < b; ++k) {
            const float4 pn = lsm_ld(xyz, min(k + 1, b - 1));   // next point in flight meanwhile
            if (p.x > xh) break;
            if (p.x >= xl) body(p, k);
            p = pn;
        }
        return;
    }
    // G points per memory round trip: the walk is a chain of L2 hits, one latency each
    for (uint32_t k = a; k < b; k += G) {
        float4 p[G];
#pragma unroll
        for (int g = 0; g < G; ++g) p[g] = lsm_ld(xyz, min(k + uint32_t(g), b - 1));
        bool stop = false;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (!stop) {
                if (k + uint32_t(g) >= b || p[g].x > xh) stop = true;
                else if (p[g].x >= xl) body(p[g], k + uint32_t(g));
            }
        }
        if (stop) break;
    }
}

// scan_run with the window test folded into a predicate: body(p, k, in) is called for every
// loaded point until the walk passes xh, `in` telling whether it lies in the window (fewer
// divergent branches per point than nested ifs).
// point readers of the walks (GlobalPts / BufPts): lsm_common.h
#ifndef LSM_NORMALS_BUF
#define LSM_NORMALS_BUF 1
#endif
#if LSM_NORMALS_BUF
typedef BufPts NormalsPts;
__device__ __forceinline__ BufPts normals_pts(const CloudDev &C) { return cloud_buf_pts(C); }
#else
typedef GlobalPts NormalsPts;
__device__ __forceinline__ GlobalPts normals_pts(const CloudDev &C) { return GlobalPts{C.xyz}; }
#endif

// body(p, k, in): `in` is the walk's liveness only -- the points a window search leaves before
// xl (at most SCAN_SLACK) lie outside the ball and fail the bodies' own exact tests, so the
// window's left edge needs no test of its own.
template <int G, int PF, typename Rd, typename Body>
__device__ __forceinline__ void scan_run_pred(const Rd &xyz, uint32_t a, uint32_t b, float xl,
                                              float xh, Body &&body) {
    if (b - a > SCAN_BSEARCH) {
        // 4-ary search (three probes per round trip) for a start at most SCAN_SLACK points
        // before the window's first point: the walk skips x < xl anyway
        uint32_t lo = a, hi = b;   // the first x >= xl lies in [lo, hi]
        while (hi - lo > SCAN_SLACK) {
            const uint32_t q = (hi - lo) >> 2;
            const uint32_t m1 = lo + q, m2 = lo + 2 * q, m3 = lo + 3 * q;
            const float x1 = xyz.x(m1), x2 = xyz.x(m2), x3 = xyz.x(m3);
            if (x3 < xl) lo = m3 + 1;
            else if (x2 < xl) { lo = m2 + 1; hi = m3; }
            else if (x1 < xl) { lo = m1 + 1; hi = m2; }
            else hi = m1;
        }
        a = lo;
    }
if constexpr (PF == 2) {
    // software-pipelined over two register buffers (the next group loads into the buffer not
    // being tested, so no copies rotate the pipeline); loads may run up to 2G - 1 points past
    // the run: within the cloud's LSM_XYZ_PAD spare points
    static_assert(2 * G - 1 <= LSM_XYZ_PAD, "prefetched group loads run past a run");
    if (a >= b) return;
    float4 pa[G], pb[G];
#pragma unroll
    for (int g = 0; g < G; ++g) pa[g] = xyz.pt(a + uint32_t(g));
    auto test = [&](const float4 (&p)[G], uint32_t k) {
        bool live = true;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            live = live && (k + uint32_t(g) < b) && !(p[g].x > xh);
            body(p[g], k + uint32_t(g), live);
        }
        return live;
    };
    for (uint32_t k = a;;) {
#pragma unroll
        for (int g = 0; g < G; ++g) pb[g] = xyz.pt(k + uint32_t(G + g));
        if (!test(pa, k)) break;
        k += G;
        if (k >= b) break;
#pragma unroll
        for (int g = 0; g < G; ++g) pa[g] = xyz.pt(k + uint32_t(G + g));
        if (!test(pb, k)) break;
        k += G;
        if (k >= b) break;
    }
    } else {
#if LSM_NORMALS_PF
    // software-pipelined: the next group's loads are in flight while this group is tested (the
    // loads may run up to 2G - 1 points past the run: within the cloud's LSM_XYZ_PAD spare points)
    static_assert(2 * G - 1 <= LSM_XYZ_PAD, "prefetched group loads run past a run");
    if (a >= b) return;
    float4 nx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) nx[g] = xyz.pt(a + uint32_t(g));
    for (uint32_t k = a; k < b; k += G) {
        float4 p[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            p[g] = nx[g];
            nx[g] = xyz.pt(k + uint32_t(G + g));
        }
#else
    static_assert(G <= LSM_XYZ_PAD, "group loads may run LSM_XYZ_PAD points past a run");
    for (uint32_t k = a; k < b; k += G) {
        float4 p[G];
#pragma unroll
        for (int g = 0; g < G; ++g) p[g] = xyz.pt(k + uint32_t(g));
#endif
        bool live = true;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            live = live && (k + uint32_t(g) < b) && !(p[g].x > xh);
            body(p[g], k + uint32_t(g), live);
        }
        if (!live) break;
    }
    }
}

// Exact kNN truncation (Open3D SearchHybrid keeps the max_nn nearest of the ball, ordered by
// (d2, traversal); here by (d2, sorted index)), one lane per point, no cross-lane traffic.
//
// The neighbours are ranked by the key (d2, k). A selection state splits the ball into
// "below" (certainly among the max_nn nearest), "members" (still undecided) and "above":
//   * an interval [dlo, dhi] x [klo, khi] of keys holding the members of the previous level
//     (exact: it is the min/max over them, and a monotone classification's member set is
//     exactly the keys between its extremes);
//   * a current level that bins the members, by d2 or -- once they all share one d2 -- by k:
//     bin(v) = clamp(floor((v - lo) * scale), 0, nb - 1), monotone in v (IEEE subtraction and
//     multiplication by a positive constant are monotone), and the chosen bin b.
// Every scan re-evaluates the same functions, so the classification is bit-for-bit consistent.
//   scan 1: count + centred cumulants of the ball and, when the ball's cells hold more than
//           max_nn points, the level-0 histogram (128 u8 bins of d2 over [0, r^2)) in the
//           lane's own LDS row. count <= max_nn (two thirds of the points): done.
//   else:   choose the bin holding the max_nn-th neighbour. A planar patch is uniform in d2, so
//           it holds ~5 points and usually fits SEL_CAP at once; otherwise rescan the ball of
//           radius sqrt(top) for the members' extremes and a 32-bin u32 histogram of them
//           (also the restart when a u8 bin saturates); exact d2 ties go on by index.
//   final:  rescan, accumulate every point below, collect the members (<= SEL_CAP) in the LDS
//           row and add the `need` smallest by (d2, k).
constexpr int NB8 = 128;          // level-0 bins (u8 counters)
constexpr int NB32 = 32;          // refinement bins (u32 counters)
#ifndef LSM_HSTRIDE
#define LSM_HSTRIDE 33
#endif
constexpr int HSTRIDE = LSM_HSTRIDE;   // LDS words per lane: 128 u8 / 32 u32 bins, padded to odd
// members collected by the final pass: 2 words per entry (the f32 rounding of the exact f64 d2,
// a monotone key, and the index; f32 ties are ordered by recomputing the exact f64 d2), so 16
// fit a lane's row. A chosen bin holding more needs a refine scan: 1.1 % of the dense points
// of a bench scan with 11 entries (3 words: f64 d2 + index), 0.02 % with 16 (numpy study)
constexpr int SEL_CAP = 16;
constexpr int MAX_REFINE = 32;    // d2 levels (~11 x 5 bits) then index levels (<= 7 x 5 bits)

// search radius covering every point with d2 < hi (slack for the f32 cell arithmetic)
__device__ __forceinline__ float sel_radius(double hi, float r) {
    return fminf(float(sqrt(hi)) * 1.0001f + 1e-5f, r);
}

struct Sel {
    double dlo, dhi;       // member interval in d2 (inclusive)
    uint32_t klo, khi;     // member interval in k (inclusive)
    double lo, scale;      // current level: bins of d2 (by_idx = 0) or of k (by_idx = 1)
    int nb, b, by_idx;
};

__device__ __forceinline__ int sel_level_bin(const Sel &S, double d2, uint32_t k) {
    const double v = S.by_idx ? double(k) : d2;
    const double t = (v - S.lo) * S.scale;
    return t < 0.0 ? 0 : (t >= double(S.nb) ? S.nb - 1 : int(t));
}

// -1: below (certainly among the max_nn nearest), 0: member, 1: above
__device__ __forceinline__ int sel_classify(const Sel &S, double d2, uint32_t k) {
    if (d2 < S.dlo) return -1;
    if (d2 > S.dhi) return 1;
    if (k < S.klo) return -1;
    if (k > S.khi) return 1;
    const int b = sel_level_bin(S, d2, k);
    return b < S.b ? -1 : (b > S.b ? 1 : 0);
}

// f32 thresholds of the classification: a point whose f32 d2 (within 4.2e-7 relative of the
// exact one; 2e-6 of margin) lies below `below32` is certainly "below" (and inside the ball), one
// above `above32` certainly "above". sel_classify: below iff d2 < dlo or (d2 <= dhi and bin < b),
// above iff d2 > dhi or (d2 >= dlo and bin > b); the bins of a d2 level are monotone in d2 with
// edges lo + j / scale. np.preclass = 0 disables both (every point takes the f64 test).
__device__ __forceinline__ void sel_thresholds(const Sel &S, const NormalParams &np,
                                               float &below32, float &above32) {
    double lo_t = S.dlo, hi_t = S.dhi;
    if (!S.by_idx && S.scale > 0.0) {   // (scale 0: one bin holding every point)
        lo_t = fmax(lo_t, fmin(S.dhi, S.lo + double(S.b) / S.scale));
        if (S.b < S.nb - 1) hi_t = fmin(hi_t, fmax(S.dlo, S.lo + double(S.b + 1) / S.scale));
    }
    lo_t = fmin(lo_t, np.r2);   // below also needs d2 < r2
    below32 = np.preclass && lo_t > 0.0 ? float(lo_t * (1.0 - 2e-6)) : -1.f;
    above32 = np.preclass && hi_t < 1e30 ? float(hi_t * (1.0 + 2e-6)) : INFINITY;
}

// A lane's LDS row. With HSTRIDE == 32 (no padding word: five 256-lane workgroups fit a CU's
// 160 KB) word w is stored at w ^ (lane & 31), so the loops in which every lane touches the same
// word of its own row (clearing, bin selection, member ranking) hit 32 distinct banks.
struct HRow {
    uint32_t *p;
    uint32_t sw;
    __device__ __forceinline__ uint32_t *at(uint32_t w) const { return p + (w ^ sw); }
    __device__ __forceinline__ uint32_t &operator[](uint32_t w) const { return p[w ^ sw]; }
    __device__ __forceinline__ uint32_t byte(uint32_t b) const {   // u8 bin b
        return reinterpret_cast<const uint8_t *>(p)[((b >> 2) ^ sw) * 4 + (b & 3)];
    }
};

// fire-and-forget LDS add (ds_add_u32: no read-back, so the walk does not wait on LDS)
__device__ __forceinline__ void lds_add(uint32_t *a, uint32_t v) {
    __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Accumulator policies of hybrid_lane: what is done with the neighbourhood of a point.
//   add(p, k): neighbour k (sorted index) at p; reset(): drop everything added; finish(): the
//   neighbourhood is complete.
// CumAcc: centred f64 cumulants -> the normal (oriented to a prior normal when the cloud has
// one: EstimateNormals on a cloud with normals, see normal_from_cum).
struct CumAcc {
    Cum c;
    double qx, qy, qz;
    float4 *out;
    const float4 *prior;
    __device__ void add(const float4 &p, uint32_t) { cum_add_pt(c, p, qx, qy, qz); }
    __device__ void reset() { c = Cum{}; }
    __device__ void finish() {
        if (out) *out = normal_from_cum(c, prior);   // (out null: a lane without a point)
    }
};

// ListAcc: the neighbour indices (sorted order) and exact f64 squared distances, unordered.
struct ListAcc {
    int32_t *idx;
    double *d2;
    int32_t *count;
    int cap, n;
    double qx, qy, qz;
    __device__ void add(const float4 &p, uint32_t k) {
        if (n < cap) {
            idx[n] = int32_t(k);
            d2[n] = lsm_sqdist64(qx, qy, qz, double(p.x), double(p.y), double(p.z));
        }
        ++n;
    }
    __device__ void reset() { n = 0; }
    __device__ void finish() { *count = n < cap ? n : cap; }
};

// KDTreeSearchParamHybrid(radius, max_nn) neighbourhood of point j of cloud C by one lane (H: the
// lane's HSTRIDE-word LDS row), handed to `acc`.
// Density prediction: a point whose own cell is crowded almost always has more than max_nn
// ball neighbours, and then scan 1's neighbourhood would be dropped again.
__device__ __forceinline__ bool predict_dense(const CloudDev &C, const NormalParams &np, float4 qf) {
    if (!(np.dense_k > 0.f)) return false;
    auto cc = [](float v, float o, float inv, int n) {
        const int c = (int)floorf((v - o) * inv);
        return c < 0 ? 0 : (c > n - 1 ? n - 1 : c);
    };
    const int l = lsm_cell_lin(C.nbx, C.nby, cc(qf.x, C.ox, C.inv_cell, C.nx),
                               cc(qf.y, C.oy, C.inv_cell_y, C.ny), cc(qf.z, C.oz, C.inv_cell, C.nz));
    return float(lsm_ld(C.cell_start, l + 1) - lsm_ld(C.cell_start, l)) >=
           np.dense_k * C.cell * C.cell_y;
}

// Phase statistics of hybrid_lane (diagnostics, normals_phase_kernel only): per lane, walk steps
// (loaded points inside the row windows) and members in scan 1, the refine scans and the final
// pass, and whether the lane needed the kNN truncation.
struct NPhase {
    uint32_t v[8];   // s1 steps, s1 members, refine steps, final steps, final added, dense, refines, predicted dense
};
#define NP_ST(ph, c, x)              \
    do {                             \
        if (PH) (ph)->v[c] += (x);   \
    } while (0)

// hybrid_lane modes. NL_AUTO: the whole procedure. The split launch (normals_sparse_kernel +
// normals_dense_kernel) runs it in two halves with the same decisions and the same summation
// order, so every normal is bit-identical to NL_AUTO's:
//   NL_SPARSE: a point predicted dense is deferred at once; otherwise scan 1 (cumulants and
//              count, no histogram: no LDS) finishes it when count <= max_nn, else defers it;
//   NL_DENSE:  a deferred point, as NL_AUTO runs a predicted-dense one (scan 1 builds the
//              histogram only; a point with count <= max_nn then takes the final pass whole,
//              which adds its ball in scan 1's order -- NL_AUTO's sums for either prediction).
// Returns false when the point was deferred.
//   NL_DENSE_NR: NL_DENSE without the refine scans: a point that needs one (a saturated u8 bin, or
//              a chosen bin holding more than SEL_CAP members: 0.002 % of the dense points) is
//              deferred (returns false) to normals_refine_kernel, which runs it as NL_DENSE. The
//              refine scans' live state sets the dense kernel's register count (101 VGPRs, 93
//              without them): leaving them out lets the dense half run 5 waves per SIMD.
constexpr int NL_AUTO = 0, NL_SPARSE = 1, NL_DENSE = 2, NL_DENSE_NR = 4;
#ifndef LSM_NDIAG
#define LSM_NDIAG 0   // diagnostics builds only (wrong normals): 1 / 3 stop the dense half after
                      // scan 1 (3: without its histogram adds), 2 before its final pass
#endif

template <int G, typename Acc, bool PH = false, int MODE = NL_AUTO, int PF = LSM_NORMALS_PF>
__device__ bool hybrid_lane(const CloudDev &C, int j, const NormalParams &np,
                            unsigned long long *stats, uint32_t *H, Acc &acc,
                            NPhase *ph = nullptr, uint32_t *SK = nullptr) {
    const HRow R{H, HSTRIDE == 32 ? (__lane_id() & 31u) : 0u};
    const float4 qf = lsm_ld(C.xyz, j);
    const double qx = qf.x, qy = qf.y, qz = qf.z;
    const NormalsPts pts = normals_pts(C);
    // Dense-predicted points skip acc.add in scan 1 (histogram only); a wrong guess costs one
    // plain rescan below, which visits the ball in scan 1's order (identical sums).
    const bool dense = (MODE == NL_DENSE || MODE == NL_DENSE_NR) ? true : predict_dense(C, np, qf);
    if (MODE == NL_SPARSE && dense) return false;
    NP_ST(ph, 7, dense ? 1u : 0u);
    if (MODE != NL_SPARSE) {
#pragma unroll 1   // (unrolled, the 32 swizzled word addresses stay live across the scans)
        for (int b = 0; b < NB8 / 4; ++b) R[b] = 0;
    }
    Sel S = {-INFINITY, INFINITY, 0u, 0xffffffffu, 0.0, double(NB8) / np.r2, NB8, 0, 0};
    bool sat = false;
    int count = 0;
    // Scan 1 with f32 decisions: a point is certainly inside when f < r2_lo, and certainly in level-0 bin
    // floor(t) when t = f * hscale is more than 2e-4 from a bin edge (|t - t_exact| < 6e-5:
    // f32 d^2 and the scale are within 4.2e-7 relative, t < 128). The rest (the sphere's
    // rounding band, bin edges) take the exact f64 distance, so the histogram is the one the
    // f64 binning of the later scans implies.
    auto scan1 = [&](const float4 &p, uint32_t k, bool in) {
            NP_ST(ph, 0, in ? 1u : 0u);
            const float dx = p.x - qf.x, dy = p.y - qf.y, dz = p.z - qf.z;
            const float f = dx * dx + dy * dy + dz * dz;
            if (MODE == NL_SPARSE) {   // the same ball membership as the binned test below
                if (in && (f < np.r2_lo ||
                           (f <= np.r2_hi && make_off(p, qx, qy, qz).d2 < np.r2))) {
                    acc.add(p, k);
                    // the first NSMALL_INLINE members (a small neighbourhood: all of them)
                    if (SK && count < NSMALL_INLINE) SK[count * PT_THREADS] = k;
                    ++count;
                }
                return;
            }
            const float t = f * np.hscale;
            const float fr = __builtin_amdgcn_fractf(t);   // t - floor(t) (v_fract)
            const bool fast = in && f < np.r2_lo && fr > 2e-4f && fr < 1.f - 2e-4f;
            int bb = fast ? int(t) : -1;
            if (in && !fast && f <= np.r2_hi) {   // the sphere's rounding band, bin edges
                const Off o = make_off(p, qx, qy, qz);
                if (o.d2 < np.r2) bb = sel_level_bin(S, o.d2, k);
            }
            if (bb >= 0) {
                NP_ST(ph, 1, 1u);
                if (!dense) acc.add(p, k);
                ++count;
#if LSM_NDIAG == 3   // diagnostics build: no histogram adds (the walk's own cost)
                count += bb & 1;
#else
                lds_add(R.at(bb >> 2), 1u << ((bb & 3) << 3));   // u8 bin, carries detected below
#endif
            }
    };
    ball_visit_runs(C, qf, np.r, [&](uint32_t a, uint32_t b, float xl, float xh) {
        scan_run_pred<G, PF>(pts, a, b, xl, xh, scan1);
    });
    if (MODE == NL_SPARSE) {
        if (count > np.max_nn) return false;
        acc.finish();
        return true;
    }
#if LSM_NDIAG == 1 || LSM_NDIAG == 3
    if constexpr (MODE == NL_DENSE) {   // diagnostics build: the dense half stops after scan 1
        acc.c.n = count;
        acc.finish();
        return true;
    }
#endif
    double top = np.r2;   // every point below or member has d2 <= top (up to rounding)
    uint32_t need = uint32_t(np.max_nn);   // still to take from the members
    if (count <= np.max_nn) {
        if (!dense) {
            acc.finish();
            return true;
        }
        S.dlo = INFINITY;   // mispredicted: every ball point is below, the final pass adds them
        need = 0;
    } else {
        if (!dense) acc.reset();
        NP_ST(ph, 5, 1u);
        if (stats) atomicAdd(stats, 1ull);   // points that needed the kNN truncation
        // A u8 bin that passed 255 carried into its neighbour byte (or out of its word): each
        // such carry lowers the bin total by 255 or 256, so the total tells.
        if (count > 255) {
            uint32_t tot = 0;
#pragma unroll 1
            for (int b = 0; b < NB8 / 4; ++b) {
                const uint32_t w = R[b];
                tot += (w & 0xffu) + ((w >> 8) & 0xffu) + ((w >> 16) & 0xffu) + (w >> 24);
            }
            sat = tot != uint32_t(count);
        }
    }
    // rescan the members of the current state: their key extremes and a histogram by `next`
    auto refine = [&](const Sel &next, double &dmin, double &dmax, uint32_t &kmin, uint32_t &kmax) {
        NP_ST(ph, 6, 1u);
#pragma unroll 1
        for (int b = 0; b < NB32; ++b) R[b] = 0;
        dmin = INFINITY;
        dmax = -INFINITY;
        kmin = 0xffffffffu;
        kmax = 0u;
        ball_visit_runs(C, qf, sel_radius(top, np.r), [&](uint32_t a, uint32_t b, float xl, float xh) {
            scan_run_pred<G, PF>(pts, a, b, xl, xh, [&](const float4 &p, uint32_t k, bool in) {
                NP_ST(ph, 2, in ? 1u : 0u);
                Off o;
                if (in && in_ball(np, qf, qx, qy, qz, p, o) && sel_classify(S, o.d2, k) == 0) {
                    lds_add(R.at(sel_level_bin(next, o.d2, k)), 1u);
                    dmin = fmin(dmin, o.d2);
                    dmax = fmax(dmax, o.d2);
                    kmin = min(kmin, k);
                    kmax = max(kmax, k);
                }
            });
        });
    };
    bool u8 = true;
    if (MODE == NL_DENSE_NR && count > np.max_nn && sat) return false;   // refine: deferred
    if (count > np.max_nn && sat) {                             // a u8 bin saturated: level 0 as 32 x u32 bins
        Sel next = S;
        next.scale = double(NB32) / np.r2;
        next.nb = NB32;
        S.b = 0;
        S.scale = 0.0;                     // every ball point is a member (one bin)
        S.nb = 1;
        double dmin, dmax;
        uint32_t kmin, kmax;
        refine(next, dmin, dmax, kmin, kmax);
        S = next;
        u8 = false;
    }
    for (int it = 0; it < MAX_REFINE && count > np.max_nn; ++it) {
        uint32_t acc = 0;
        int bstar = S.nb - 1;
        for (int b = 0; b < S.nb; ++b) {
            const uint32_t hb = u8 ? R.byte(b) : R[b];
            if (acc + hb >= need) {
                bstar = b;
                break;
            }
            acc += hb;
        }
        const uint32_t bin_count = u8 ? R.byte(bstar) : R[bstar];
        need -= acc;
        S.b = bstar;
        if (!S.by_idx) top = fmin(top, S.lo + double(bstar + 1) / S.scale);
        if (bin_count <= SEL_CAP) break;
        if (MODE == NL_DENSE_NR) return false;   // refine: deferred
        // next level over the chosen bin's range, clipped to the exact member extremes known
        // so far (so no member falls below lo: a clamped lowest bin could never split); the
        // extremes found by the same scan then replace the whole classification chain
        Sel next = S;
        {
            const double vlo = S.by_idx ? double(S.klo) : S.dlo;
            const double vhi = S.by_idx ? double(S.khi) + 1.0 : S.dhi;
            const double elo = fmax(S.lo + double(bstar) / S.scale, vlo);
            const double ehi = fmin(S.lo + double(bstar + 1) / S.scale, vhi);
            next.lo = elo;
            next.scale = ehi > elo ? double(NB32) / (ehi - elo) : S.scale * double(NB32);
            next.nb = NB32;
        }
        double dmin, dmax;
        uint32_t kmin, kmax;
        refine(next, dmin, dmax, kmin, kmax);
        u8 = false;
        if (!S.by_idx && dmin == dmax) {
            // every member has the same d2: order them by index instead
            next.by_idx = 1;
            next.lo = double(kmin);
            next.scale = double(NB32) / (double(kmax - kmin) + 1.0);
            refine(next, dmin, dmax, kmin, kmax);
        }
        next.dlo = dmin;
        next.dhi = dmax;
        next.klo = next.by_idx ? kmin : 0u;
        next.khi = next.by_idx ? kmax : 0xffffffffu;
        top = fmin(top, dmax);
        S = next;
    }
    // final pass: everything below, plus the `need` smallest members. f32 pre-classification:
    // d2 below min(r2, dlo, the chosen d2 bin's lower edge) is certainly "below", d2 above
    // max(dhi-side bounds) certainly "above"; only the band between takes the exact f64 test
    // (the f32 d2 is within 4.2e-7 relative; 2e-6 of margin).
#if LSM_NDIAG == 2
    if constexpr (MODE == NL_DENSE) {   // diagnostics build: the dense half stops before the final pass
        acc.c.n = count + int(need) + int(top * 1e6);
        acc.finish();
        return true;
    }
#endif
    float below32, above32;
    sel_thresholds(S, np, below32, above32);
    uint32_t m = 0;
    // final-pass classification of one point: true = add it now (below); members are collected
    auto fin = [&](const float4 &p, uint32_t k, bool in) -> bool {
        NP_ST(ph, 3, in ? 1u : 0u);
        const float fd = f32_d2(qf, p);
        if (!in || fd > np.r2_hi || fd > above32) return false;
        if (fd < below32) {
            NP_ST(ph, 4, 1u);
            return true;
        }
        const Off o = make_off(p, qx, qy, qz);
        if (fd >= np.r2_lo && !(o.d2 < np.r2)) return false;
        const int cl = sel_classify(S, o.d2, k);
        if (cl < 0) {
            NP_ST(ph, 4, 1u);
            return true;
        }
        if (cl == 0) {
            if (m < SEL_CAP) {
                R[2 * m] = __float_as_uint(float(o.d2));
                R[2 * m + 1] = k;
            }
            ++m;
        }
        return false;
    };
    ball_visit_runs(C, qf, sel_radius(top, np.r), [&](uint32_t a, uint32_t b, float xl, float xh) {
        scan_run_pred<G, PF>(pts, a, b, xl, xh, [&](const float4 &p, uint32_t k, bool in) {
            if (fin(p, k, in)) acc.add(p, k);
        });
    });
    const uint32_t mm = m < SEL_CAP ? m : SEL_CAP;
    for (uint32_t e = 0; e < mm; ++e) {
        const uint32_t fe = R[2 * e];   // non-negative floats order like their bit patterns
        const uint32_t ke = R[2 * e + 1];
        uint32_t rank = 0;
        double de = -1.0;   // exact d2 of e, computed at its first f32 tie
        for (uint32_t g = 0; g < mm; ++g) {
            const uint32_t fg = R[2 * g];
            if (fg < fe) {
                ++rank;
            } else if (fg == fe && g != e) {
                // f32 keys tie: the exact (d2, index) order (the f32 rounding is monotone, so
                // distinct keys already order like the exact distances)
                const uint32_t kg = R[2 * g + 1];
                if (de < 0.0) de = make_off(lsm_ld(C.xyz, ke), qx, qy, qz).d2;
                const double dg = make_off(lsm_ld(C.xyz, kg), qx, qy, qz).d2;
                rank += (dg < de || (dg == de && kg < ke)) ? 1u : 0u;
            }
        }
        if (rank < need) acc.add(lsm_ld(C.xyz, ke), ke);
    }
    acc.finish();
    return true;
}

// Small neighbourhoods in Open3D's arithmetic (keyframe.py:160-162 -> [O3D]
// EstimatePerPointCovariances -> ComputeCovariance). A neighbourhood of a few points -- near-
// collinear points of one distant ring -- has a rank-deficient covariance whose smallest
// eigenvector the rounding of the cumulants decides, so the centred cumulants of the main path
// (better numerics, different rounding) would pick a different normal there. A neighbourhood
// of 3 .. NSMALL points (normal_from_cum leaves only a mark, w = 1) is redone exactly as Open3D
// does it: the ball's members in the search's order (ascending d2, ties by reference index), the
// nine raw f64 cumulants summed in that order with every product rounded on its own, each divided
// by n, cov = E[pp^T] - mu mu^T, FastEigen3x3 (and w = 0). Every kernel that computes normals does
// this for its own small neighbourhoods right after the main path: the sparse half from the
// members its scan 1 kept (small_normal_from_list, no second walk), the others by a second walk
// (small_normal; rare there).

// The normal of point j from its neighbourhood Kk[0 .. m) (LDS, stride STRIDE words) in
// the search's order, in Open3D's arithmetic (ComputeCovariance: raw f64 cumulants in that
// order, each divided by n; FastEigen3x3).
// The f64 coordinates of sorted point k as Open3D's cloud holds them: a voxelised cloud's f64
// centroid (C.xyz64, reference order), else the f32 point. The small neighbourhoods' covariance
// is decided by rounding (rank-deficient), so it must see the same coordinates: at C5's 0.4 m
// scale nearly every neighbourhood is small, and the f32 rounding of the centroids alone moved
// 12 of 512 coarse-stage registrations past the bar (tools/bench_parity.py).
__device__ __forceinline__ void pt_f64(const CloudDev &C, uint32_t k, double &x, double &y,
                                       double &z) {
    if (C.xyz64) {
        const size_t r = size_t(lsm_ld(C.perm, k)) * 3;
        x = lsm_ld(C.xyz64, r);
        y = lsm_ld(C.xyz64, r + 1);
        z = lsm_ld(C.xyz64, r + 2);
    } else {
        const float4 p = lsm_ld(C.xyz, k);
        x = p.x;
        y = p.y;
        z = p.z;
    }
}

// the exact squared distance that orders a small neighbourhood: nanoflann's ((dx^2 + dy^2) +
// dz^2) of the f64 coordinates for a voxelised cloud, else the walks' exact d2 of the f32 points
__device__ __forceinline__ double small_d2(const CloudDev &C, double qx, double qy, double qz,
                                           uint32_t k) {
    if (C.xyz64) {
        double x, y, z;
        pt_f64(C, k, x, y, z);
        return lsm_sqdist64(qx, qy, qz, x, y, z);
    }
    return make_off(lsm_ld(C.xyz, k), qx, qy, qz).d2;
}

template <int STRIDE>
__device__ __forceinline__ void small_cov_normal(const CloudDev &C, int j, const uint32_t *Kk,
                                                 int m) {
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0, c4 = 0.0, c5 = 0.0, c6 = 0.0, c7 = 0.0, c8 = 0.0;
    for (int q = 0; q < m; ++q) {
        double x, y, z;
        pt_f64(C, Kk[q * STRIDE], x, y, z);
        c0 = lsm_dadd(c0, x);
        c1 = lsm_dadd(c1, y);
        c2 = lsm_dadd(c2, z);
        c3 = lsm_dadd(c3, lsm_dmul(x, x));
        c4 = lsm_dadd(c4, lsm_dmul(x, y));
        c5 = lsm_dadd(c5, lsm_dmul(x, z));
        c6 = lsm_dadd(c6, lsm_dmul(y, y));
        c7 = lsm_dadd(c7, lsm_dmul(y, z));
        c8 = lsm_dadd(c8, lsm_dmul(z, z));
    }
    sym3 A = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    if (m >= 3) {
        const double dn = double(m);
        c0 = lsm_ddiv(c0, dn);
        c1 = lsm_ddiv(c1, dn);
        c2 = lsm_ddiv(c2, dn);
        c3 = lsm_ddiv(c3, dn);
        c4 = lsm_ddiv(c4, dn);
        c5 = lsm_ddiv(c5, dn);
        c6 = lsm_ddiv(c6, dn);
        c7 = lsm_ddiv(c7, dn);
        c8 = lsm_ddiv(c8, dn);
        A.a00 = lsm_dsub(c3, lsm_dmul(c0, c0));
        A.a01 = lsm_dsub(c4, lsm_dmul(c0, c1));
        A.a02 = lsm_dsub(c5, lsm_dmul(c0, c2));
        A.a11 = lsm_dsub(c6, lsm_dmul(c1, c1));
        A.a12 = lsm_dsub(c7, lsm_dmul(c1, c2));
        A.a22 = lsm_dsub(c8, lsm_dmul(c2, c2));
    }
    const_cast<float4 *>(C.nrm)[j] =
        normal_from_cov(A, C.prior_ref ? C.prior_ref + C.perm[j] : nullptr, 0.f);
}

// The ordering key of a neighbour: the f32 rounding of its exact d2 (monotone: it orders like d2
// wherever the keys differ; equal keys fall back to the exact (d2, reference index) order).
__device__ __forceinline__ bool small_before(const CloudDev &C, double qx, double qy, double qz,
                                             uint32_t fk, double dk, uint32_t k, uint32_t fq,
                                             uint32_t kq) {
    if (fk != fq) return fk < fq;
    const double dq = small_d2(C, qx, qy, qz, kq);
    return dk < dq || (dk == dq && lsm_ld(C.perm, k) < lsm_ld(C.perm, kq));
}

// Open3D's arithmetic for the small neighbourhood of point j, at most CAP points: the ball walked
// again, its members kept in the search's order in the lane's LDS F / Kk (stride STRIDE words,
// CAP slots; C workgroup-uniform).
template <int CAP, int STRIDE>
__device__ __forceinline__ void small_normal(const CloudDev &C, int j, const NormalParams &np,
                                             uint32_t *F, uint32_t *Kk) {
    const int cap = np.max_nn < CAP ? np.max_nn : CAP;
    const float4 qf = lsm_ld(C.xyz, j);
    const double qx = qf.x, qy = qf.y, qz = qf.z;
    double ox, oy, oz;   // the query as the ordering sees it (pt_f64)
    pt_f64(C, uint32_t(j), ox, oy, oz);
    int m = 0;
    const NormalsPts pts = normals_pts(C);
    ball_visit_runs(C, qf, np.r, [&](uint32_t a, uint32_t b, float xl, float xh) {
        scan_run_pred<2, 1>(pts, a, b, xl, xh, [&](const float4 &p, uint32_t k, bool in) {
            Off o;
            if (!in || !in_ball(np, qf, qx, qy, qz, p, o)) return;
            const double dk = C.xyz64 ? small_d2(C, ox, oy, oz, k) : o.d2;
            const uint32_t fk = __float_as_uint(float(dk));   // non-negative: orders as u32
            auto before = [&](int q) {
                return small_before(C, ox, oy, oz, fk, dk, k, F[q * STRIDE], Kk[q * STRIDE]);
            };
            int pos;
            if (m < cap) pos = m++;
            else if (cap > 0 && before(cap - 1)) pos = cap - 1;
            else return;
            for (; pos > 0 && before(pos - 1); --pos) {
                F[pos * STRIDE] = F[(pos - 1) * STRIDE];
                Kk[pos * STRIDE] = Kk[(pos - 1) * STRIDE];
            }
            F[pos * STRIDE] = fk;
            Kk[pos * STRIDE] = k;
        });
    });
    small_cov_normal<STRIDE>(C, j, Kk, m);
}

// The same from the whole neighbourhood already collected in walk order (Kk[0 .. m), the
// sparse half's scan 1): sorted into the search's order in place, then the normal.
template <int STRIDE>
__device__ __forceinline__ void small_normal_from_list(const CloudDev &C, int j, uint32_t *F,
                                                       uint32_t *Kk, int m) {
    double qx, qy, qz;   // the query as the ordering sees it (pt_f64)
    pt_f64(C, uint32_t(j), qx, qy, qz);
    for (int a = 0; a < m; ++a) {
        const uint32_t k = Kk[a * STRIDE];
        const double dk = small_d2(C, qx, qy, qz, k);
        const uint32_t fk = __float_as_uint(float(dk));
        int pos = a;
        for (; pos > 0 && small_before(C, qx, qy, qz, fk, dk, k, F[(pos - 1) * STRIDE],
                                       Kk[(pos - 1) * STRIDE]);
             --pos) {
            F[pos * STRIDE] = F[(pos - 1) * STRIDE];
            Kk[pos * STRIDE] = Kk[(pos - 1) * STRIDE];
        }
        F[pos * STRIDE] = fk;
        Kk[pos * STRIDE] = k;
    }
    small_cov_normal<STRIDE>(C, j, Kk, m);
}

// After a kernel's hybrid_lane: a neighbourhood of 3 .. NSMALL points (normal_from_cum left only
// a mark) gets Open3D's arithmetic, its member lists in the lane's LDS row (H: HSTRIDE words).
__device__ __forceinline__ void small_after(const CloudDev &C, int j, const NormalParams &np,
                                            const CumAcc &acc, uint32_t *H) {
    static_assert(2 * NSMALL <= HSTRIDE, "small_normal's lists fit a lane's LDS row");
    if (acc.out && acc.c.n >= 3 && acc.c.n <= NSMALL) small_normal<NSMALL, 1>(C, j, np, H, H + NSMALL);
}

// Own-cell population from which a point is predicted to have more than max_nn neighbours in
// its ball (a performance guess only: both outcomes are exact): frac * max_nn * (cell / r)^2,
// a surface's share of the ball in one cell. On HDL-64 scans with cell = r = 0.3 m and
// max_nn = 300, frac = 0.27 mispredicts ~4 % of the ball work either way.
// (a bench sweep of frac over 0.20-0.45: 0.27 best)
constexpr double NORMALS_DENSE_FRAC = 0.27;
float dense_k(int max_nn, double r2) {
    if (r2 <= 0.0) return 0.f;
    return float(NORMALS_DENSE_FRAC * double(max_nn) / r2);
}

// LSM_NORMALS_EXACT=1 (a test knob, read per call): no f32 pre-classification in the final pass
// -- the tests' proof that it leaves every neighbourhood, and so every normal, bit-identical
int normals_preclass() { return lsm_knob("LSM_NORMALS_EXACT", 0.0) != 0.0 ? 0 : 1; }

NormalParams normal_params(double radius, int max_nn) {
    NormalParams np;
    np.r2 = radius * radius;
    np.r = float(radius);
    np.r2_lo = float(np.r2 * (1.0 - 4e-6));
    np.r2_hi = float(np.r2 * (1.0 + 4e-6));
    np.hscale = float(double(NB8) / np.r2);
    np.max_nn = max_nn;
    np.dense_k = dense_k(max_nn, np.r2);
    np.preclass = normals_preclass();
    return np;
}

#ifdef LSM_NORMALS_WPE
#define LSM_NORMALS_ATTR __attribute__((amdgpu_waves_per_eu(LSM_NORMALS_WPE)))
#else
#define LSM_NORMALS_ATTR
#endif
template <int G>
__global__ void __launch_bounds__(PT_THREADS) LSM_NORMALS_ATTR
normals_kernel(const Seg *segs, const CloudDev *cd, NormalParams np,
               unsigned long long *stats) {
    __shared__ uint32_t lds[PT_THREADS * HSTRIDE];
    const Seg s = segs[blockIdx.x];
    const CloudDev C = cd[s.cloud];
    const int j = s.start + threadIdx.x;
    if (j >= C.n) return;
    const float4 q = lsm_ld(C.xyz, j);
    CumAcc acc{Cum{}, double(q.x), double(q.y), double(q.z), const_cast<float4 *>(C.nrm) + j,
               C.prior_ref ? C.prior_ref + C.perm[j] : nullptr};
    hybrid_lane<G>(C, j, np, stats, lds + threadIdx.x * HSTRIDE, acc);
    small_after(C, j, np, acc, lds + threadIdx.x * HSTRIDE);
    // statistics run only (LSM_NORMALS_STATS): neighbourhood sizes |kNN(max_nn) & ball(r)| -- the
    // algorithmic work of the normals (9 cumulant FMAs per neighbour), summed
    // over 64 counters to spread the atomics
    if (stats) atomicAdd(stats + 8 + (blockIdx.x & 63), (unsigned long long)acc.c.n);
}


// Split launch, first half: the points predicted sparse (NL_SPARSE, no LDS). Deferred points are
// appended to their cloud's dense list dlist[geo.pt_off + ...] (wave-aggregated; the order of
// the list does not matter: every point's computation is independent of the others).
// registers of the sparse half capped for 8 waves per SIMD (64 VGPRs; 14 spilled outside the
// walks): normals 148.2 -> 143.8 ms per step (7 waves: 144.1; uncapped, 80 VGPRs: 6 waves)
// Append point j (when `take`) to a cloud's list, one atomic per workgroup: the workgroup's
// entries stay one run in lane order. Every thread of the workgroup must call it.
__device__ __forceinline__ void wg_append(bool take, uint32_t j, uint32_t *list, uint32_t *cnt) {
    __shared__ uint32_t s_cnt[PT_THREADS / LSM_WAVE + 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t bm = __ballot(take);
    if (lane == 0) s_cnt[w] = uint32_t(__popcll(bm));
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int q = 0; q < PT_THREADS / LSM_WAVE; ++q) tot += s_cnt[q];
        s_cnt[PT_THREADS / LSM_WAVE] = tot ? atomicAdd(cnt, tot) : 0u;
    }
    __syncthreads();
    if (take) {
        uint32_t base = s_cnt[PT_THREADS / LSM_WAVE];
        for (int q = 0; q < w; ++q) base += s_cnt[q];
        list[base + __popcll(bm & ((uint64_t(1) << lane) - 1))] = j;
    }
    __syncthreads();   // s_cnt is reused by the next call
}

#ifndef LSM_NSPARSE_WPE
#define LSM_NSPARSE_WPE 8
#endif
#if LSM_NSPARSE_WPE > 0
#define LSM_NSPARSE_ATTR __attribute__((amdgpu_waves_per_eu(LSM_NSPARSE_WPE)))
#else
#define LSM_NSPARSE_ATTR
#endif
template <int G>
__global__ void __launch_bounds__(PT_THREADS) LSM_NSPARSE_ATTR
normals_sparse_kernel(const Seg *segs, const CloudDev *cd, const GridGeo *geo, NormalParams np,
                      uint32_t *dlist, uint32_t *dcnt, unsigned long long *stats) {
    __shared__ uint32_t s_f[NSMALL_INLINE * PT_THREADS];   // small_normal's member lists
    __shared__ uint32_t s_k[NSMALL_INLINE * PT_THREADS];
    const Seg s = segs[blockIdx.x];
    const CloudDev C = cd[s.cloud];
    const int j = s.start + threadIdx.x;
    const bool valid = j < C.n;
    bool defer = false, small = false;
    int small_n = 0;
    if (valid) {
        const float4 q = lsm_ld(C.xyz, j);
        CumAcc acc{Cum{}, double(q.x), double(q.y), double(q.z), const_cast<float4 *>(C.nrm) + j,
                   C.prior_ref ? C.prior_ref + C.perm[j] : nullptr};
        defer = !hybrid_lane<G, CumAcc, false, NL_SPARSE>(C, j, np, nullptr, nullptr, acc,
                                                           nullptr, s_k + threadIdx.x);
        if (stats && !defer) atomicAdd(stats + 8 + (blockIdx.x & 63), (unsigned long long)acc.c.n);
        small = !defer && acc.c.n >= 3 && acc.c.n <= NSMALL_INLINE;
        small_n = acc.c.n;
    }
    // a neighbourhood of 3..NSMALL points gets Open3D's arithmetic at once from the members scan 1
    // kept (the dense, refine and one-kernel paths walk their rare small ones again themselves)
    if (small) small_normal_from_list<PT_THREADS>(C, j, s_f + threadIdx.x, s_k + threadIdx.x, small_n);
    // one append per workgroup: its deferred points stay one run in cell order (the dense
    // half's waves then hold neighbouring points)
    wg_append(defer, uint32_t(j), dlist + geo[s.cloud].pt_off, dcnt + s.cloud);
}

// Split launch, second half: one lane per entry of the clouds' dense lists (NL_DENSE), so the
// truncated neighbourhoods run in full waves. The grid is the first half's (a cloud's list never
// holds more entries than the cloud has points); workgroups past the list return at once.
// LSM_NDENSE_WPE: waves per SIMD requested for the dense half (0: no request)
#ifndef LSM_NDENSE_WPE
#define LSM_NDENSE_WPE 0
#endif
#if LSM_NDENSE_WPE > 0
#define LSM_NDENSE_ATTR __attribute__((amdgpu_waves_per_eu(LSM_NDENSE_WPE)))
#else
#define LSM_NDENSE_ATTR LSM_NORMALS_ATTR
#endif
template <int G>
__global__ void __launch_bounds__(PT_THREADS) LSM_NDENSE_ATTR
normals_dense_kernel(const Seg *segs, const CloudDev *cd, const GridGeo *geo, NormalParams np,
                     const uint32_t *dlist, const uint32_t *dcnt, unsigned long long *stats,
                     uint32_t *rlist, uint32_t *rcnt) {
    __shared__ uint32_t lds[PT_THREADS * HSTRIDE];
    const Seg s = segs[blockIdx.x];
    const uint32_t slot = uint32_t(s.start) + threadIdx.x;
    if (slot >= dcnt[s.cloud]) return;
    const CloudDev C = cd[s.cloud];
    const uint32_t off = geo[s.cloud].pt_off;
    const int j = int(dlist[off + slot]);
    const float4 q = lsm_ld(C.xyz, j);
    CumAcc acc{Cum{}, double(q.x), double(q.y), double(q.z), const_cast<float4 *>(C.nrm) + j,
               C.prior_ref ? C.prior_ref + C.perm[j] : nullptr};
    // the rare points that need a refine scan go to the cloud's refine list
    const bool done = hybrid_lane<G, CumAcc, false, NL_DENSE_NR, LSM_NORMALS_PFD>(
        C, j, np, stats, lds + threadIdx.x * HSTRIDE, acc);
    if (done) small_after(C, j, np, acc, lds + threadIdx.x * HSTRIDE);
    const uint64_t bm = __ballot(!done);
    if (bm) {
        const int lane = threadIdx.x & 63, leader = __ffsll((unsigned long long)bm) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(rcnt + s.cloud, uint32_t(__popcll(bm)));
        base = uint32_t(__shfl(int(base), leader, LSM_WAVE));
        if (!done) rlist[off + base + __popcll(bm & ((uint64_t(1) << lane) - 1))] = uint32_t(j);
    }
    if (stats && done) atomicAdd(stats + 8 + (blockIdx.x & 63), (unsigned long long)acc.c.n);
}

// The dense half's deferred points (NL_DENSE with its refine scans): blockIdx.x = cloud, the
// workgroups of a cloud stride over its refine list (most clouds have none).
constexpr int REFINE_BLOCKS = 4;
template <int G>
__global__ void __launch_bounds__(PT_THREADS)
normals_refine_kernel(const CloudDev *cd, const GridGeo *geo, NormalParams np,
                      const uint32_t *rlist, const uint32_t *rcnt, unsigned long long *stats) {
    __shared__ uint32_t lds[PT_THREADS * HSTRIDE];
    const int c = blockIdx.x;
    const uint32_t n = rcnt[c];
    const CloudDev C = cd[c];
    const uint32_t off = geo[c].pt_off;
    for (uint32_t slot = blockIdx.y * PT_THREADS + threadIdx.x; slot < n;
         slot += gridDim.y * PT_THREADS) {
        const int j = int(rlist[off + slot]);
        const float4 q = lsm_ld(C.xyz, j);
        CumAcc acc{Cum{}, double(q.x), double(q.y), double(q.z), const_cast<float4 *>(C.nrm) + j,
                   C.prior_ref ? C.prior_ref + C.perm[j] : nullptr};
        hybrid_lane<G, CumAcc, false, NL_DENSE, LSM_NORMALS_PFD>(C, j, np, stats,
                                                                 lds + threadIdx.x * HSTRIDE, acc);
        small_after(C, j, np, acc, lds + threadIdx.x * HSTRIDE);
        if (stats) atomicAdd(stats + 8 + (blockIdx.x & 63), (unsigned long long)acc.c.n);
    }
}

// The dense half of the split launch: the dense lists' points, then the few the dense kernel
// deferred to a refine scan. rlist / rcnt: scratch of the dense lists' size / K words.
template <int G>
void launch_dense_half(hipStream_t st, hipStream_t rst, const Seg *d_segs, int nseg,
                       const CloudDev *d_cd, const GridGeo *d_geo, int K, const NormalParams &np,
                       const uint32_t *dlist, const uint32_t *dcnt, unsigned long long *d_ns,
                       uint32_t *rlist, uint32_t *rcnt, lsm_ctx *ctx, const char *stat) {
    normals_dense_kernel<G><<<nseg, PT_THREADS, 0, st>>>(d_segs, d_cd, d_geo, np, dlist, dcnt,
                                                         d_ns, rlist, rcnt);
    // the refine scans (a few long single-lane chains) on rst: the side stream when it may
    // overlap what follows (lsm_ctx::side)
    // Timed under its own name ("normals_refine"): on the side stream its window overlaps the
    // ICP kernels it shares the chip with, so it is reported beside the normals' time, not in it.
    (void)stat;
    if (rst != st) {
        (void)hipEventRecord(ctx->side_ev, st);
        (void)hipStreamWaitEvent(rst, ctx->side_ev, 0);
    }
    hipEvent_t ev;
    ctx->tic("normals_refine", &ev, rst);
    normals_refine_kernel<G><<<dim3(K, REFINE_BLOCKS), PT_THREADS, 0, rst>>>(d_cd, d_geo, np, rlist,
                                                                            rcnt, d_ns);
    ctx->toc("normals_refine", ev, rst);
    if (rst != st) {
        (void)hipEventRecord(ctx->side_ev, rst);
        ctx->side_pending = true;
    }
}

#ifdef LSM_DIAG
// normals_kernel with phase statistics (LSM_NORMALS_PHASES=1, diagnostics builds): per counter the
// lane sum (out[c]) and the per-wave maximum summed over waves (out[8 + c]: the wave's cost
// under divergence)
__global__ void __launch_bounds__(PT_THREADS)
normals_phase_kernel(const Seg *segs, const CloudDev *cd, NormalParams np,
                     unsigned long long *out) {
    __shared__ uint32_t lds[PT_THREADS * HSTRIDE];
    const Seg s = segs[blockIdx.x];
    const CloudDev C = cd[s.cloud];
    const int j = s.start + threadIdx.x;
    NPhase ph{};
    if (j < C.n) {
        const float4 q = lsm_ld(C.xyz, j);
        CumAcc acc{Cum{}, double(q.x), double(q.y), double(q.z), const_cast<float4 *>(C.nrm) + j,
                   C.prior_ref ? C.prior_ref + C.perm[j] : nullptr};
        hybrid_lane<NORMALS_G_DEFAULT, CumAcc, true>(C, j, np, nullptr, lds + threadIdx.x * HSTRIDE,
                                                     acc, &ph);
    }
    for (int c = 0; c < 8; ++c) {
        uint32_t sum = ph.v[c], mx = ph.v[c];
        for (int off = 32; off > 0; off >>= 1) {
            sum += __shfl_xor(sum, off, LSM_WAVE);
            mx = max(mx, __shfl_xor(mx, off, LSM_WAVE));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(out + c, (unsigned long long)sum);
            atomicAdd(out + 8 + c, (unsigned long long)mx);
        }
    }
}
#endif

// Neighbour lists of FPFH (ComputeFPFHFeature's KDTreeSearchParamHybrid): at most `cap` per
// point, row j of idx / d2 (sorted order), count[j].
__global__ void __launch_bounds__(PT_THREADS)
nbr_lists_kernel(const Seg *segs, const CloudDev *cd, NormalParams np, int32_t *idx, double *d2,
                 int32_t *count, int cap) {
    __shared__ uint32_t lds[PT_THREADS * HSTRIDE];
    const Seg s = segs[blockIdx.x];
    const CloudDev C = cd[s.cloud];
    const int j = s.start + threadIdx.x;
    if (j >= C.n) return;
    const float4 q = lsm_ld(C.xyz, j);
    ListAcc acc{idx + size_t(j) * cap, d2 + size_t(j) * cap, count + j, cap, 0,
                double(q.x), double(q.y), double(q.z)};
    hybrid_lane<NORMALS_G_DEFAULT>(C, j, np, nullptr, lds + threadIdx.x * HSTRIDE, acc);
}

// ------------------------------------------------------------------------------------------
// download in reference order
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
download_kernel(const float4 *xyz, const float4 *nrm, const uint32_t *perm, int n, double *oxyz,
                double *onrm) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t r = perm[j];
    if (oxyz) {
        float4 p = xyz[j];
        oxyz[3 * r] = p.x;
        oxyz[3 * r + 1] = p.y;
        oxyz[3 * r + 2] = p.z;
    }
    if (onrm) {
        float4 q = nrm[j];
        onrm[3 * r] = q.x;
        onrm[3 * r + 1] = q.y;
        onrm[3 * r + 2] = q.z;
    }
}

// helpers ----------------------------------------------------------------------------------
// A launch's workgroup table: (cloud, first point) per per_block points of every cloud, in the
// context's grow-only host storage (a fresh vector per call cost page faults)
struct SegTable {
    const Seg *p = nullptr;
    size_t n = 0;
    const Seg *data() const { return p; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
};
static_assert(sizeof(Seg) == sizeof(uint64_t), "Seg tables live in u64 storage");

// Every table upload of the pre-processing and normals paths first orders the main stream after
// a refine kernel still running on the side stream (lsm_ctx::side): the refine reads the launch's
// CloudDev / GridGeo tables (g_cd / g_geo, lz_cd / lz_gg), and the next upload may overwrite them
// before run_normals' own join (lsm_normals_complete's (radius, max_nn) groups did). The join is a
// device-side wait, only recorded while a refine is pending.
template <typename T>
int upload_vec(lsm_ctx *ctx, const char *name, const std::vector<T> &v, T **out) {
    ctx->join_side_device();
    T *d = static_cast<T *>(ctx->buf(name, v.size() * sizeof(T)));
    if (!d) {
        ctx->set_error(std::string("scratch allocation failed: ") + name);
        return LSM_ENOMEM;
    }
    if (!v.empty())
        LSM_HIP_TRY(ctx, hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice,
                                        ctx->stream));
    *out = d;
    return LSM_OK;
}

int upload_vec(lsm_ctx *ctx, const char *name, const SegTable &v, Seg **out) {
    ctx->join_side_device();
    Seg *d = static_cast<Seg *>(ctx->buf(name, v.size() * sizeof(Seg)));
    if (!d) {
        ctx->set_error(std::string("scratch allocation failed: ") + name);
        return LSM_ENOMEM;
    }
    if (!v.empty())
        LSM_HIP_TRY(ctx, hipMemcpyAsync(d, v.data(), v.size() * sizeof(Seg), hipMemcpyHostToDevice,
                                        ctx->stream));
    *out = d;
    return LSM_OK;
}

int ensure_cloud_buffers(lsm_ctx *ctx, Cloud *c, int64_t n, bool normals) {
    if (c->cap < n || !c->d_xyz) {
        (void)hipFree(c->d_xyz);
        (void)hipFree(c->d_nrm);
        (void)hipFree(c->d_perm);
        c->d_xyz = nullptr;
        c->d_nrm = nullptr;
        c->d_perm = nullptr;
        int64_t cap = std::max<int64_t>(n, 1);
        // LSM_XYZ_PAD spare points past the end: the normals walks load whole groups without
        // clamping the index (the spare lanes' values are never used)
        if (hipMalloc(&c->d_xyz, (cap + LSM_XYZ_PAD) * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->d_perm, cap * sizeof(uint32_t)) != hipSuccess) {
            ctx->set_error("hipMalloc failed for processed cloud");
            return LSM_ENOMEM;
        }
        c->cap = cap;
    }
    if (normals && !c->d_nrm) {
        if (hipMalloc(&c->d_nrm, c->cap * sizeof(float4)) != hipSuccess) {
            ctx->set_error("hipMalloc failed for normals");
            return LSM_ENOMEM;
        }
    }
    return LSM_OK;
}

inline int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (uint64_t(1) << b) <= v) ++b;
    return b;
}

// Radix sorts (grid (cell, x) keys, voxel run keys). rocPRIM's gfx950 defaults sort 8 bits per
// onesweep pass. 64-bit keys sort 9 bits per pass (the grid's ~63-bit keys: 7 passes, not 8;
// measured 13.9 -> 13.3 ms of grid per C3 step); 11 bits would need 192 KB of histogram LDS for
// 64-bit keys, and 11-bit passes over 32-bit keys measured slower than four 8-bit ones.
// LSM_RADIX_BITS_K32 / LSM_RADIX_BITS_K64 build A/B variants.
#ifndef LSM_RADIX_BITS_K64
#define LSM_RADIX_BITS_K64 9
#endif
template <int BITS, int BS, int IPT>
using OnesweepConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 16>, rocprim::kernel_config<BS, IPT>, BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
template <typename Key> struct SortConfigFor { using type = rocprim::default_config; };
#ifdef LSM_RADIX_BITS_K32
template <> struct SortConfigFor<uint32_t> { using type = OnesweepConfig<LSM_RADIX_BITS_K32, 512, 16>; };
#endif
#ifdef LSM_RADIX_BITS_K64
template <> struct SortConfigFor<uint64_t> { using type = OnesweepConfig<LSM_RADIX_BITS_K64, 512, 16>; };
#endif
template <typename Key> using SortConfig = typename SortConfigFor<Key>::type;

}  // namespace

// ==========================================================================================
// host orchestration
// ==========================================================================================
namespace {

SegTable point_segments(lsm_ctx *ctx, const char *name, const std::vector<uint32_t> &n,
                        int per_block) {
    size_t tot = 0;
    for (uint32_t v : n) tot += (size_t(v) + per_block - 1) / size_t(per_block);
    std::vector<uint64_t> &h = ctx->host_tables[name];
    if (h.size() < tot) h.resize(tot + tot / 4);
    Seg *segs = reinterpret_cast<Seg *>(h.data());
    size_t j = 0;
    for (size_t k = 0; k < n.size(); ++k)
        for (uint32_t s = 0; s < n[k]; s += uint32_t(per_block)) segs[j++] = {int32_t(k), int32_t(s)};
    return SegTable{segs, tot};
}

// filter_radius_height over the batch: writes the kept points of cloud k, in reference order, to
// out[off[k] .. off[k] + cnt[k]).
// Also the boxes of the filtered clouds (bb: 6 per cloud), read back with the counts in one
// synchronisation (the voxel grid or the spatial grid needs them next).
int run_filter(lsm_ctx *ctx, std::vector<Cloud *> &clouds, const lsm_prep_params &p,
               float4 **out, std::vector<uint32_t> &off, std::vector<uint32_t> &cnt,
               std::vector<double> &bb) {
    hipStream_t st = ctx->stream;
    const int K = int(clouds.size());
    std::vector<const float *> raw(K);
    std::vector<int32_t> nraw(K), first_block(K), nblocks(K);
    std::vector<uint32_t> nr(K);
    int64_t total_raw = 0;
    int32_t nb_acc = 0;
    for (int k = 0; k < K; ++k) {
        raw[k] = clouds[k]->d_raw;
        nraw[k] = int32_t(clouds[k]->n_raw);
        first_block[k] = nb_acc;
        nblocks[k] = int32_t((clouds[k]->n_raw + FILTER_CHUNK - 1) / FILTER_CHUNK);
        nb_acc += nblocks[k];
        total_raw += clouds[k]->n_raw;
    }
    if (total_raw >= (int64_t(1) << 32)) {
        ctx->set_error("batch too large (>= 2^32 raw points); split the batch");
        return LSM_EINVAL;
    }
    for (int k = 0; k < K; ++k) nr[k] = uint32_t(clouds[k]->n_raw);
    const SegTable fsegs = point_segments(ctx, "h_fsegs", nr, FILTER_CHUNK);
    const int nfb = int(fsegs.size());
    int rc;
    const float **d_raw;
    int32_t *d_nraw;
    Seg *d_fsegs;
    if ((rc = upload_vec(ctx, "f_raw", raw, const_cast<const float ***>(&d_raw)))) return rc;
    if ((rc = upload_vec(ctx, "f_nraw", nraw, &d_nraw))) return rc;
    if ((rc = upload_vec(ctx, "f_segs", fsegs, &d_fsegs))) return rc;
    uint32_t *d_bcount = (uint32_t *)ctx->buf("f_bcount", size_t(nfb + 1) * 4);
    uint32_t *d_boff = (uint32_t *)ctx->buf("f_boff", size_t(nfb + 1) * 4);
    float4 *d_fpts = (float4 *)ctx->buf("f_pts", size_t(std::max<int64_t>(total_raw, 1)) * 16);
    uint32_t *d_fidx = (uint32_t *)ctx->buf("f_idx", size_t(std::max<int64_t>(total_raw, 1)) * 4);
    if (!d_bcount || !d_boff || !d_fpts || !d_fidx) {
        ctx->set_error("scratch allocation failed (filter)");
        return LSM_ENOMEM;
    }
    // min_radius = -inf switches the lower radius bound off (keep-all passes over derived clouds:
    // a point on the sensor axis, x = y = 0, still passes); any other value is squared, as the
    // reference's r2 > min_radius ** 2 (keyframe.py:92)
    const double minr2 = (std::isinf(p.min_radius) && p.min_radius < 0) ? -INFINITY
                                                                         : p.min_radius * p.min_radius;
    FilterParams fp{p.max_radius * p.max_radius, minr2, p.min_height, p.max_height};
    std::vector<uint32_t> boff_h(size_t(nfb) + 1, 0);
    if (nfb > 0) {
        hipEvent_t ev;
        ctx->tic("filter", &ev);
        filter_count<<<nfb, FILTER_THREADS, 0, st>>>(d_fsegs, d_raw, d_nraw, fp, d_bcount);
        size_t tmpb = 0;
        LSM_HIP_TRY(ctx, rocprim::exclusive_scan(nullptr, tmpb, d_bcount, d_boff, 0u, size_t(nfb) + 1,
                                rocprim::plus<uint32_t>(), st));
        void *tmp = ctx->buf("scan_tmp", tmpb);
        // the extra element (bcount[nfb] = 0) turns boff[nfb] into the total
        LSM_HIP_TRY(ctx, hipMemsetAsync(d_bcount + nfb, 0, 4, st));
        LSM_HIP_TRY(ctx, rocprim::exclusive_scan(tmp, tmpb, d_bcount, d_boff, 0u, size_t(nfb) + 1,
                                rocprim::plus<uint32_t>(), st));
        filter_write<<<nfb, FILTER_THREADS, 0, st>>>(d_fsegs, d_raw, d_nraw, fp, d_boff, d_fpts,
                                                     d_fidx);
        ctx->toc("filter", ev);
        int32_t *d_fb, *d_nb;
        uint32_t *d_off = (uint32_t *)ctx->buf("f_coff", size_t(K) * 4);
        uint32_t *d_cnt = (uint32_t *)ctx->buf("f_ccnt", size_t(K) * 4);
        double *d_bb = (double *)ctx->buf("f_bb", size_t(K) * 48);
        if (!d_off || !d_cnt || !d_bb) return LSM_ENOMEM;
        if ((rc = upload_vec(ctx, "f_fb", first_block, &d_fb))) return rc;
        if ((rc = upload_vec(ctx, "f_nb", nblocks, &d_nb))) return rc;
        filter_cloud_ranges<<<(K + 255) / 256, 256, 0, st>>>(d_boff, d_fb, d_nb, K, d_off, d_cnt);
        if ((rc = run_bbox(ctx, d_fpts, d_off, d_cnt, K, d_bb, "f_bbk"))) return rc;
        bb.resize(size_t(K) * 6);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(boff_h.data(), d_boff, boff_h.size() * 4,
                                        hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipMemcpyAsync(bb.data(), d_bb, bb.size() * 8, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    } else {
        bb.assign(size_t(K) * 6, 0.0);
        for (int k = 0; k < K; ++k)
            for (int a = 0; a < 3; ++a) {   // empty clouds: (+inf, -inf), as bbox_final leaves them
                bb[6 * k + a] = INFINITY;
                bb[6 * k + 3 + a] = -INFINITY;
            }
    }
    off.assign(K, 0);
    cnt.assign(K, 0);
    uint32_t run = 0;
    for (int k = 0; k < K; ++k) {
        if (nblocks[k] == 0) {
            off[k] = run;
            continue;
        }
        off[k] = boff_h[first_block[k]];
        cnt[k] = boff_h[first_block[k] + nblocks[k]] - off[k];
        run = off[k] + cnt[k];
    }
    *out = d_fpts;
    return LSM_OK;
}

// voxel_down_sample over the batch; replaces (pts, off, cnt) by the voxel centroids (f32 working
// copy) and stores the f64 centroids / int32 keys on each cloud.
// bb: the filtered clouds' boxes in, the voxelised clouds' boxes out (read back with the voxel
// counts in one synchronisation)
int run_voxel(lsm_ctx *ctx, std::vector<Cloud *> &clouds, double v, float4 **pts,
              std::vector<uint32_t> &off, std::vector<uint32_t> &cnt, std::vector<double> &bb) {
    hipStream_t st = ctx->stream;
    const int K = int(clouds.size());
    int rc;
    uint32_t ntot = 0;
    for (int k = 0; k < K; ++k) ntot = std::max(ntot, off[k] + cnt[k]);
    uint32_t *d_off, *d_cnt;
    if ((rc = upload_vec(ctx, "v_off", off, &d_off))) return rc;
    if ((rc = upload_vec(ctx, "v_cnt", cnt, &d_cnt))) return rc;
    std::vector<VoxGeo> geo(K);
    uint64_t key_off = 0;
    for (int k = 0; k < K; ++k) {
        VoxGeo &G = geo[k];
        G = {0.0, 0.0, 0.0, 1, 1, 1, key_off};
        if (cnt[k] == 0) continue;
        // Open3D: voxel_min_bound = min_bound - v3 * 0.5; voxel_max_bound = max_bound + v3 * 0.5
        const double half = v * 0.5;
        double vmin[3], vmax[3];
        for (int a = 0; a < 3; ++a) {
            vmin[a] = bb[6 * k + a] - half;
            vmax[a] = bb[6 * k + 3 + a] + half;
        }
        const double ext =
            std::max(vmax[0] - vmin[0], std::max(vmax[1] - vmin[1], vmax[2] - vmin[2]));
        if (v * double(std::numeric_limits<int>::max()) < ext) {
            ctx->set_error("voxel_size is too small.");
            return LSM_EINVAL;
        }
        int64_t d[3];
        for (int a = 0; a < 3; ++a)
            d[a] = (int64_t)std::floor((bb[6 * k + 3 + a] - vmin[a]) / v) + 2;
        const uint64_t cells = uint64_t(d[0]) * uint64_t(d[1]) * uint64_t(d[2]);
        if (cells > (uint64_t(1) << 44)) {
            ctx->set_error("voxel grid too large for the 64-bit key space");
            return LSM_EINVAL;
        }
        G = {vmin[0], vmin[1], vmin[2], d[0], d[1], d[2], key_off};
        key_off += cells;
    }
    VoxGeo *d_geo;
    if ((rc = upload_vec(ctx, "v_geo", geo, &d_geo))) return rc;
    const SegTable segs = point_segments(ctx, "h_vsegs", cnt, PT_THREADS);
    Seg *d_segs;
    if ((rc = upload_vec(ctx, "v_segs", segs, &d_segs))) return rc;
    const size_t N = std::max<uint32_t>(ntot, 1);
    uint64_t *k_in = (uint64_t *)ctx->buf("v_kin", N * 8);
    uint64_t *k_out = (uint64_t *)ctx->buf("v_kout", N * 8);
    uint32_t *v_out = (uint32_t *)ctx->buf("v_vout", N * 4);
    uint32_t *flag = (uint32_t *)ctx->buf("v_flag", N * 4 + 4);
    uint32_t *vid = (uint32_t *)ctx->buf("v_vid", N * 4 + 4);
    uint32_t *vstart = (uint32_t *)ctx->buf("v_vstart", N * 4 + 4);
    uint32_t *rid = (uint32_t *)ctx->buf("v_rid", N * 4 + 4);
    uint32_t *rstart = (uint32_t *)ctx->buf("v_rstart", N * 4 + 4);
    uint32_t *vorder = (uint32_t *)ctx->buf("v_order", N * 4);
    uint32_t *vwex = (uint32_t *)ctx->buf("v_wex", N * 4 + 4);
    int32_t *ptc = (int32_t *)ctx->buf("v_ptc", N * 4);
    double *cent = (double *)ctx->buf("v_cent", N * 24);
    int32_t *vkeys = (int32_t *)ctx->buf("v_keys", N * 12);
    float4 *vpts = (float4 *)ctx->buf("v_pts", N * 16);
    int32_t *vcloud = (int32_t *)ctx->buf("v_vcloud", N * 4);
    if (!k_in || !k_out || !v_out || !flag || !vid || !vstart || !rid || !rstart || !vorder || !vwex || !ptc ||
        !cent ||
        !vkeys || !vpts || !vcloud) {
        ctx->set_error("scratch allocation failed (voxel)");
        return LSM_ENOMEM;
    }
    uint32_t nvox = 0;
    std::vector<uint32_t> vcount(K, 0);
    if (!segs.empty()) {
        hipEvent_t ev;
        ctx->tic("voxel", &ev);
        point_cloud_ids<<<dim3(64, K), 256, 0, st>>>(d_off, d_cnt, K, ptc);
        const int endbit = bits_for(key_off);
        const int nb = int((ntot + PT_THREADS - 1) / PT_THREADS);
        // exclusive scan of n + 1 flags (flag[n] = 0): out[n] = the flag total
        auto scan_flags = [&](const uint32_t *in, uint32_t *out, uint32_t n) -> int {
            size_t tb = 0;
            LSM_HIP_TRY(ctx, rocprim::exclusive_scan(nullptr, tb, in, out, 0u, size_t(n) + 1,
                                                     rocprim::plus<uint32_t>(), st));
            void *tp = ctx->buf("scan_tmp", tb);
            if (!tp) return LSM_ENOMEM;
            LSM_HIP_TRY(ctx, rocprim::exclusive_scan(tp, tb, in, out, 0u, size_t(n) + 1,
                                                     rocprim::plus<uint32_t>(), st));
            return LSM_OK;
        };
        // keys and run heads, run ids (scan), run (key, start), stable radix sort of the runs,
        // voxel heads over the sorted runs and their scan (voxel ids), per-voxel sums
        auto chain = [&](auto *kin, auto *kout) -> int {
            using KeyT = std::remove_pointer_t<decltype(kin)>;
            voxel_keys<KeyT><<<int(segs.size()), PT_THREADS, 0, st>>>(d_segs, *pts, d_off, d_cnt,
                                                                      d_geo, v, kout, flag);
            LSM_HIP_TRY(ctx, hipMemsetAsync(flag + ntot, 0, 4, st));
            int r;
            if ((r = scan_flags(flag, rid, ntot))) return r;
            voxel_runs<KeyT><<<nb, PT_THREADS, 0, st>>>(kout, flag, rid, ntot, kin, rstart);
            uint32_t nruns = 0;   // the sort's length (one read-back)
            LSM_HIP_TRY(ctx, hipMemcpyAsync(&nruns, rid + ntot, 4, hipMemcpyDeviceToHost, st));
            LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
            const rocprim::counting_iterator<uint32_t> run_ids(0u);
            size_t tb = 0;
            LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs<SortConfig<KeyT>>(nullptr, tb, kin, kout, run_ids, v_out,
                                                                         size_t(nruns), 0, endbit, st));
            void *tp = ctx->buf("sort_tmp", tb);
            if (!tp) return LSM_ENOMEM;
            LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs<SortConfig<KeyT>>(tp, tb, kin, kout, run_ids, v_out,
                                                                         size_t(nruns), 0, endbit, st));
            const int rb = int((nruns + PT_THREADS - 1) / PT_THREADS);
            voxel_flags<KeyT><<<rb, PT_THREADS, 0, st>>>(kout, nruns, flag);
            LSM_HIP_TRY(ctx, hipMemsetAsync(flag + nruns, 0, 4, st));
            if ((r = scan_flags(flag, vid, nruns))) return r;
            voxel_heads<<<rb, PT_THREADS, 0, st>>>(flag, vid, nruns, vstart);
            // voxels <= runs: the flags and their scan cover nruns + 1 entries (past nvox: 0)
            voxel_wide<<<int((nruns + 1 + PT_THREADS - 1) / PT_THREADS), PT_THREADS, 0, st>>>(vid, vstart, nruns,
                                                                                               flag);
            if ((r = scan_flags(flag, vwex, nruns))) return r;
            voxel_order<<<rb, PT_THREADS, 0, st>>>(vid, flag, vwex, nruns, vorder);
            voxel_reduce<KeyT><<<rb, PT_THREADS, 0, st>>>(kout, v_out, rstart, vid, vstart, vorder, nruns,
                                                          *pts, ptc, d_geo, cent, vkeys, vpts, vcloud);
            return LSM_OK;
        };
        rc = endbit <= 32 ? chain(reinterpret_cast<uint32_t *>(k_in), reinterpret_cast<uint32_t *>(k_out))
                          : chain(k_in, k_out);
        if (rc) return rc;
        // voxels per cloud: the sort keeps each cloud's runs together (key_off), so cloud k's
        // voxel ids run from vid[rid[P_k]] to vid[rid[P_k+1]], P_k = the points of the clouds
        // before it
        std::vector<uint32_t> pstart(size_t(K) + 1, 0);
        for (int k = 0; k < K; ++k) pstart[k + 1] = pstart[k] + cnt[k];
        uint32_t *d_pstart, *d_vb = (uint32_t *)ctx->buf("v_vb", (size_t(K) + 1) * 4);
        if (!d_vb) return LSM_ENOMEM;
        if ((rc = upload_vec(ctx, "v_pstart", pstart, &d_pstart))) return rc;
        vox_cloud_bounds<<<(K + 1 + 255) / 256, 256, 0, st>>>(vid, rid, d_pstart, K + 1, d_vb);
        // the centroids' boxes for the spatial grid, before the one read-back
        uint32_t *d_voff = (uint32_t *)ctx->buf("v_coff", size_t(K) * 4);
        uint32_t *d_vcnt = (uint32_t *)ctx->buf("v_ccnt", size_t(K) * 4);
        double *d_vbb = (double *)ctx->buf("v_bb", size_t(K) * 48);
        if (!d_voff || !d_vcnt || !d_vbb) return LSM_ENOMEM;
        vox_cloud_ranges<<<(K + 255) / 256, 256, 0, st>>>(d_vb, K, d_voff, d_vcnt);
        if ((rc = run_bbox(ctx, vpts, d_voff, d_vcnt, K, d_vbb, "v_bbk"))) return rc;
        ctx->toc("voxel", ev);
        std::vector<uint32_t> vb(size_t(K) + 1);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(vb.data(), d_vb, vb.size() * 4, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipMemcpyAsync(bb.data(), d_vbb, bb.size() * 8, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
        nvox = vb[K];
        for (int k = 0; k < K; ++k) vcount[k] = vb[k + 1] - vb[k];
    }
    uint32_t run = 0;
    for (int k = 0; k < K; ++k) {
        off[k] = run;
        cnt[k] = vcount[k];
        run += vcount[k];
    }
    for (int k = 0; k < K; ++k) {
        Cloud *c = clouds[k];
        if (c->vox_cap < int64_t(cnt[k]) || !c->d_vox) {
            (void)hipFree(c->d_vox);
            (void)hipFree(c->d_vkeys);
            c->d_vox = nullptr;
            c->d_vkeys = nullptr;
            c->vox_cap = std::max<int64_t>(cnt[k], 1);
            if (hipMalloc(&c->d_vox, c->vox_cap * 24) != hipSuccess ||
                hipMalloc(&c->d_vkeys, c->vox_cap * 12) != hipSuccess) {
                ctx->set_error("hipMalloc failed (voxel outputs)");
                return LSM_ENOMEM;
            }
        }
    }
    if (nvox) {   // every cloud's f64 centroids and keys in one launch (not 2 K copies)
        std::vector<double *> cp(K);
        std::vector<int32_t *> kp(K);
        for (int k = 0; k < K; ++k) {
            cp[k] = clouds[k]->d_vox;
            kp[k] = clouds[k]->d_vkeys;
        }
        double **d_cp;
        int32_t **d_kp;
        uint32_t *d_voff;
        if ((rc = upload_vec(ctx, "v_cp", cp, &d_cp))) return rc;
        if ((rc = upload_vec(ctx, "v_kp", kp, &d_kp))) return rc;
        if ((rc = upload_vec(ctx, "v_voff", off, &d_voff))) return rc;
        vox_scatter<<<(nvox + 255) / 256, 256, 0, st>>>(cent, vkeys, vcloud, nvox, d_voff, d_cp, d_kp);
    }
    *pts = vpts;
    return LSM_OK;
}

}  // namespace

#ifdef LSM_DIAG
// diagnostics builds: phase statistics of the one-kernel form to stderr (LSM_NORMALS_PHASES)
int normals_phases(lsm_ctx *ctx, const Seg *d_segs, int nseg, const CloudDev *d_cd,
                   const NormalParams &np, int64_t npts) {
    hipStream_t st = ctx->stream;
    unsigned long long *d_ph = (unsigned long long *)ctx->buf("n_phase", 16 * 8);
    if (!d_ph) return LSM_ENOMEM;
    LSM_HIP_TRY(ctx, hipMemsetAsync(d_ph, 0, 16 * 8, st));
    normals_phase_kernel<<<nseg, PT_THREADS, 0, st>>>(d_segs, d_cd, np, d_ph);
    unsigned long long h[16];
    LSM_HIP_TRY(ctx, hipMemcpyAsync(h, d_ph, sizeof(h), hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    const char *nm[8] = {"s1_steps", "s1_members", "refine_steps", "final_steps",
                         "final_added", "dense", "refines", "pred_dense"};
    fprintf(stderr, "normals phases over %lld points (lane sum / point, wave max sum / point):\n",
            (long long)npts);
    for (int c = 0; c < 8; ++c)
        fprintf(stderr, "  %-13s %10.3f %10.3f\n", nm[c], double(h[c]) / double(npts),
                double(h[8 + c]) * 64.0 / double(npts));
    return LSM_OK;
}
#endif

// Every normal of the clouds of `d_segs` (one workgroup per 256-point segment; K clouds, N >= the
// batch's points, d_geo: each cloud's pt_off into the batch lists, npts: the points):
//   * the split launch -- the sparse half (the points predicted sparse: scan 1 with cumulants and
//     count, finished when the ball holds <= max_nn), the deferred points in full waves of the
//     clouds' dense lists, and the few the dense half leaves to a refine scan -- or, with
//     LSM_NORMALS_SPLIT=0 (a test knob: bit-identical), the one-kernel form;
//   * every kernel finishes its small neighbourhoods in Open3D's covariance arithmetic.
// In statistics mode (lsm_set_timing(ctx, 2)) it also counts the neighbours of every normal
// (SURVEY.md §8d's algorithmic work) and the points that needed the kNN truncation.
int run_normals(lsm_ctx *ctx, const Seg *d_segs, int nseg, const CloudDev *d_cd,
                const GridGeo *d_geo, int K, size_t N, const NormalParams &np, int64_t npts,
                const char *stat) {
    if (nseg <= 0) return LSM_OK;
    hipStream_t st = ctx->stream;
    ctx->join_side_device();   // an earlier refine may still read the list buffers below
    unsigned long long *d_ns = nullptr;
    if (ctx->statistics) {
        d_ns = (unsigned long long *)ctx->buf("n_stats", 72 * 8);
        if (!d_ns) return LSM_ENOMEM;
        LSM_HIP_TRY(ctx, hipMemsetAsync(d_ns, 0, 72 * 8, st));
    }
#ifdef LSM_DIAG
    if (getenv("LSM_NORMALS_PHASES")) {
        const int rc = normals_phases(ctx, d_segs, nseg, d_cd, np, npts);
        if (rc) return rc;
    }
#endif
    if (lsm_knob("LSM_NORMALS_SPLIT", 1.0) != 0.0) {
        uint32_t *dlist = (uint32_t *)ctx->buf("n_dlist", N * 4);
        uint32_t *dcnt = (uint32_t *)ctx->buf("n_dcnt", size_t(K) * 8);
        uint32_t *rlist = (uint32_t *)ctx->buf("n_rlist", N * 4);
        if (!dlist || !dcnt || !rlist) return LSM_ENOMEM;
        LSM_HIP_TRY(ctx, hipMemsetAsync(dcnt, 0, size_t(K) * 8, st));
        normals_sparse_kernel<NORMALS_G_DEFAULT><<<nseg, PT_THREADS, 0, st>>>(d_segs, d_cd, d_geo,
                                                                             np, dlist, dcnt, d_ns);
        // LSM_NORMALS_SIDE (default 1): the refine kernel on the side stream (not with the
        // statistics, which read its counters right away)
        hipStream_t rst = st;
        if (!d_ns && lsm_knob("LSM_NORMALS_SIDE", 1.0) != 0.0) {
            if (!ctx->side) {
                if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess ||
                    hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming) != hipSuccess) {
                    ctx->set_error("side stream creation failed");
                    return LSM_EHIP;
                }
            }
            rst = ctx->side;
        }
        launch_dense_half<NORMALS_GD_DEFAULT>(st, rst, d_segs, nseg, d_cd, d_geo, K, np, dlist,
                                              dcnt, d_ns, rlist, dcnt + K, ctx, stat);
    } else {
        normals_kernel<NORMALS_G_DEFAULT><<<nseg, PT_THREADS, 0, st>>>(d_segs, d_cd, np, d_ns);
    }
    if (d_ns) {
        unsigned long long h[72] = {};
        LSM_HIP_TRY(ctx, hipMemcpyAsync(h, d_ns, sizeof(h), hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
        ctx->stats["normals_truncated"].launches += int64_t(h[0]);
        unsigned long long nb = 0;
        for (int k = 8; k < 72; ++k) nb += h[k];
        ctx->stats["normals_neighbours"].launches += int64_t(nb);
        ctx->stats["normals_points"].launches += npts;
    }
    return LSM_OK;
}

int lsm_prep_batch(lsm_ctx *ctx, std::vector<Cloud *> &clouds, const lsm_prep_params &p,
                   int64_t *n_out) {
    hipStream_t st = ctx->stream;
    const int K = int(clouds.size());
    int rc;
    hipEvent_t ev;

    // ---------------- filter / voxel ----------------
    float4 *wpts = nullptr;
    std::vector<uint32_t> woff, wn;
    std::vector<double> bb;   // boxes of the clouds the grid indexes (filtered, or voxelised)
    if ((rc = run_filter(ctx, clouds, p, &wpts, woff, wn, bb))) return rc;
    const bool vox = p.voxel_size > 0.0;
    if (vox && (rc = run_voxel(ctx, clouds, p.voxel_size, &wpts, woff, wn, bb))) return rc;

    // ---------------- spatial grid ----------------

    std::vector<GridGeo> geo(K);
    // The (cell, x) sort runs per group of consecutive clouds whose cells fit 31 bits: keys of
    // at most 63 bits, 7 onesweep passes of 9 bits (a 2000-keyframe batch's cells need 32 bits
    // with the finer y cells: one sort over all of it would take 8 passes)
    constexpr uint64_t GROUP_CELLS = (uint64_t(1) << 31) - 2;
    std::vector<int> gfirst{0};      // first cloud of every sort group
    std::vector<uint64_t> gcells{0};  // cells of every group
    uint64_t cell_total = 0;
    // the library's cell: 0.375 m for raw scans; for voxelised clouds (sparser: one point per
    // voxel) max(0.75, 2.5 voxel) -- C5's 0.4 / 0.2 / 0.1 m scales measured 9243 pairs/s at 0.375
    // m cells, 9611 at (1.0, 0.75, 0.75), 9625-9890 at 1.0-1.5 m for the coarsest
    // (profiles/r06/c5_gridcells_ysub.txt); the grid only indexes the points
    const float cell_req = p.grid_cell > 0 ? float(p.grid_cell)
                           : vox ? std::max(LSM_VOXEL_GRID_CELL_MIN, float(2.5 * p.voxel_size))
                                 : LSM_DEFAULT_GRID_CELL;
    for (int k = 0; k < K; ++k) {
        GridGeo &G = geo[k];
        G.pt_off = woff[k];
        G.n = wn[k];
        G.ox = G.oy = G.oz = 0.f;
        G.nx = G.ny = G.nz = 1;
        float c = cell_req;
        if (wn[k] > 0) {
            float ext[3];
            for (int a = 0; a < 3; ++a) ext[a] = float(bb[6 * k + 3 + a] - bb[6 * k + a]);
            for (;;) {
                const int64_t nx = int64_t(std::floor(ext[0] / c)) + 1;
                const int64_t ny = int64_t(std::floor(ext[1] / (c / float(LSM_YSUB)))) + 1;
                const int64_t nz = int64_t(std::floor(ext[2] / c)) + 1;
                const int64_t padded = ((nx + LSM_BLKX - 1) / LSM_BLKX) *
                                       ((ny + LSM_BLKY - 1) / LSM_BLKY) * ((nz + 3) / 4) *
                                       LSM_BLK_CELLS;
                if (padded <= MAX_CELLS_PER_CLOUD) {
                    G.nx = int(nx);
                    G.ny = int(ny);
                    G.nz = int(nz);
                    break;
                }
                c *= 1.25f;
            }
            G.ox = float(bb[6 * k]);
            G.oy = float(bb[6 * k + 1]);
            G.oz = float(bb[6 * k + 2]);
        }
        G.cell = c;
        G.inv_cell = 1.f / c;
        G.cell_y = c / float(LSM_YSUB);      // exact: a power-of-two division
        G.inv_cell_y = 1.f / G.cell_y;
        G.nbx = (G.nx + LSM_BLKX - 1) / LSM_BLKX;
        G.nby = (G.ny + LSM_BLKY - 1) / LSM_BLKY;
        G.nbz = (G.nz + LSM_BLK - 1) / LSM_BLK;
        G.ncells = uint32_t(G.nbx) * G.nby * G.nbz * LSM_BLK_CELLS;
        if (cell_total + uint64_t(G.ncells) + 1 > GROUP_CELLS) {   // a new sort group
            gfirst.push_back(k);
            gcells.push_back(0);
            cell_total = 0;
        }
        G.cell_off = uint32_t(cell_total);   // offset in the group's cell key space
        cell_total += uint64_t(G.ncells);
        gcells.back() = cell_total;
    }
    std::vector<CloudDev> cdev(K);
    std::vector<uint32_t *> perm_ptrs(K), cell_ptrs(K), bm_ptrs(K);
    for (int k = 0; k < K; ++k) {
        Cloud *c = clouds[k];
        if ((rc = ensure_cloud_buffers(ctx, c, wn[k], p.want_normals != 0))) return rc;
        const int64_t ncells = int64_t(geo[k].ncells);
        if (c->cell_cap < ncells + 1 || !c->d_cell) {
            (void)hipFree(c->d_cell);
            c->d_cell = nullptr;
            c->cell_cap = ncells + 1;
            if (hipMalloc(&c->d_cell, size_t(c->cell_cap) * 4) != hipSuccess) {
                ctx->set_error("hipMalloc failed (cell table)");
                return LSM_ENOMEM;
            }
        }
        const int64_t bmw = ncells / (32 * LSM_VB_CELLS) + 2;   // a bit per virtual block
        if (c->bmask_cap < bmw || !c->d_bmask) {
            (void)hipFree(c->d_bmask);
            c->d_bmask = nullptr;
            c->bmask_cap = bmw;
            if (hipMalloc(&c->d_bmask, size_t(bmw) * 4) != hipSuccess) {
                ctx->set_error("hipMalloc failed (block mask)");
                return LSM_ENOMEM;
            }
        }
        CloudDev &D = cdev[k];
        D.xyz = c->d_xyz;
        D.bmask = c->d_bmask;
        D.nrm = p.want_normals ? c->d_nrm : nullptr;
        D.cell_start = c->d_cell;
        D.ox = geo[k].ox;
        D.oy = geo[k].oy;
        D.oz = geo[k].oz;
        D.cell = geo[k].cell;
        D.inv_cell = geo[k].inv_cell;
        D.cell_y = geo[k].cell_y;
        D.inv_cell_y = geo[k].inv_cell_y;
        D.nx = geo[k].nx;
        D.ny = geo[k].ny;
        D.nz = geo[k].nz;
        D.nbx = geo[k].nbx;
        D.nby = geo[k].nby;
        D.nbz = geo[k].nbz;
        D.n = int(wn[k]);
        D.perm = c->d_perm;
        D.xyz64 = (vox && c->d_vox) ? c->d_vox : nullptr;   // the f64 centroids (reference order)
        D.prior_ref = (p.want_normals && c->d_prior_ref && c->prior_n == int64_t(wn[k]))
                          ? c->d_prior_ref : nullptr;
        perm_ptrs[k] = c->d_perm;
        cell_ptrs[k] = c->d_cell;
        bm_ptrs[k] = c->d_bmask;
    }
    GridGeo *d_geo;
    CloudDev *d_cd;
    uint32_t **d_perm_ptrs, **d_cell_ptrs, **d_bm_ptrs;
    if ((rc = upload_vec(ctx, "g_bmp", bm_ptrs, &d_bm_ptrs))) return rc;
    if ((rc = upload_vec(ctx, "g_geo", geo, &d_geo))) return rc;
    if ((rc = upload_vec(ctx, "g_cd", cdev, &d_cd))) return rc;
    if ((rc = upload_vec(ctx, "g_perm", perm_ptrs, &d_perm_ptrs))) return rc;
    if ((rc = upload_vec(ctx, "g_cellp", cell_ptrs, &d_cell_ptrs))) return rc;
    const SegTable psegs = point_segments(ctx, "h_gsegs", wn, PT_THREADS);
    Seg *d_psegs;
    if ((rc = upload_vec(ctx, "g_segs", psegs, &d_psegs))) return rc;
    uint32_t ntot = 0;
    for (int k = 0; k < K; ++k) ntot = std::max(ntot, woff[k] + wn[k]);
    const size_t N = std::max<uint32_t>(ntot, 1);
    uint64_t *k_in = (uint64_t *)ctx->buf("g_kin", N * 8);
    uint64_t *k_out = (uint64_t *)ctx->buf("g_kout", N * 8);
    uint32_t *v_in = (uint32_t *)ctx->buf("g_vin", N * 4);
    uint32_t *v_out = (uint32_t *)ctx->buf("g_vout", N * 4);
    uint32_t *nonempty = (uint32_t *)ctx->buf("g_nonempty", size_t(K) * 4);
    if (!k_in || !k_out || !v_in || !v_out || !nonempty) {
        ctx->set_error("scratch allocation failed (grid)");
        return LSM_ENOMEM;
    }
    ctx->tic("grid", &ev);
    LSM_HIP_TRY(ctx, hipMemsetAsync(nonempty, 0, size_t(K) * 4, st));
    int64_t maxcells1 = 0;
    for (int k = 0; k < K; ++k) maxcells1 = std::max<int64_t>(maxcells1, int64_t(geo[k].ncells) + 1);
    if (!psegs.empty()) {
        grid_keys<<<int(psegs.size()), PT_THREADS, 0, st>>>(d_psegs, wpts, d_geo, k_in, v_in);
        // one sort per group over its clouds' (contiguous) points
        const int ng = int(gfirst.size());
        auto grange = [&](int g, uint32_t &a, uint32_t &n) {
            const int k0 = gfirst[size_t(g)], k1 = g + 1 < ng ? gfirst[size_t(g) + 1] : K;
            a = woff[size_t(k0)];
            n = woff[size_t(k1) - 1] + wn[size_t(k1) - 1] - a;
        };
        size_t tmpb = 0;
        for (int g = 0; g < ng; ++g) {
            uint32_t a, n;
            grange(g, a, n);
            size_t b = 0;
            LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs<SortConfig<uint64_t>>(
                                 nullptr, b, k_in + a, k_out + a, v_in + a, v_out + a, size_t(n), 0,
                                 32 + bits_for(gcells[size_t(g)]), st));
            tmpb = std::max(tmpb, b);
        }
        void *tmp = ctx->buf("sort_tmp", tmpb);
        for (int g = 0; g < ng; ++g) {
            uint32_t a, n;
            grange(g, a, n);
            if (n == 0) continue;
            size_t b = tmpb;
            LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs<SortConfig<uint64_t>>(
                                 tmp, b, k_in + a, k_out + a, v_in + a, v_out + a, size_t(n), 0,
                                 32 + bits_for(gcells[size_t(g)]), st));
        }
        grid_scatter<<<int(psegs.size()), PT_THREADS, 0, st>>>(d_psegs, d_geo, d_cd, v_out, wpts,
                                                              d_perm_ptrs);
    }
    {
        const int gx = int(std::min<int64_t>((maxcells1 + FILL_TILE - 1) / FILL_TILE, 4096));
        grid_fill<<<dim3(gx, K), FILL_THREADS, 0, st>>>(d_geo, K, k_out, d_cell_ptrs, d_bm_ptrs,
                                                        nonempty);
    }
    ctx->toc("grid", ev);

    // ---------------- normals ----------------
    const bool lazy = p.want_normals == LSM_NORMALS_LAZY;
    if (p.want_normals && !lazy && !psegs.empty()) {
        const NormalParams np = normal_params(p.normal_radius, p.max_nn);
        int64_t npts = 0;
        for (int k = 0; k < K; ++k) npts += wn[k];
        ctx->tic("normals", &ev);
        if ((rc = run_normals(ctx, d_psegs, int(psegs.size()), d_cd, d_geo, K, N, np, npts,
                              "normals")))
            return rc;
        ctx->toc("normals", ev);
    }

    std::vector<uint32_t> hne(K);
    LSM_HIP_TRY(ctx, hipMemcpyAsync(hne.data(), nonempty, size_t(K) * 4, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    LSM_HIP_TRY(ctx, hipGetLastError());
    ctx->collect_timings();
    for (int k = 0; k < K; ++k) {
        Cloud *c = clouds[k];
        c->n = wn[k];
        c->processed = true;
        c->has_normals = p.want_normals != 0;
        c->lazy = p.want_normals == LSM_NORMALS_LAZY && wn[k] > 0;
        c->lazy_radius = p.normal_radius;
        c->lazy_max_nn = p.max_nn;
        c->voxelized = vox;
        c->dev = cdev[k];
        c->nonempty_cells = hne[k];
        if (n_out) n_out[k] = wn[k];
    }
    return LSM_OK;
}

int lsm_normals_complete(lsm_ctx *ctx, std::vector<Cloud *> &clouds) {
    hipStream_t st = ctx->stream;
    int rc;
    // one pass per (radius, max_nn) of the pending clouds
    std::vector<Cloud *> todo;
    for (Cloud *c : clouds)
        if (c && c->lazy && c->n > 0 && c->d_nrm) todo.push_back(c);
    while (!todo.empty()) {
        const double r = todo[0]->lazy_radius;
        const int mnn = todo[0]->lazy_max_nn;
        std::vector<Cloud *> grp, rest;
        for (Cloud *c : todo) (c->lazy_radius == r && c->lazy_max_nn == mnn ? grp : rest).push_back(c);
        std::vector<CloudDev> cd(grp.size());
        std::vector<uint32_t> n(grp.size());
        std::vector<GridGeo> gg(grp.size());
        uint32_t tot = 0;
        for (size_t k = 0; k < grp.size(); ++k) {
            cd[k] = grp[k]->dev;
            cd[k].nrm = grp[k]->d_nrm;
            n[k] = uint32_t(grp[k]->n);
            gg[k] = GridGeo{};
            gg[k].pt_off = tot;
            gg[k].n = n[k];
            tot += n[k];
        }
        const SegTable segs = point_segments(ctx, "h_lzsegs", n, PT_THREADS);
        CloudDev *d_cd;
        Seg *d_segs;
        GridGeo *d_gg;
        if ((rc = upload_vec(ctx, "lz_cd", cd, &d_cd))) return rc;
        if ((rc = upload_vec(ctx, "lz_segs", segs, &d_segs))) return rc;
        if ((rc = upload_vec(ctx, "lz_gg", gg, &d_gg))) return rc;
        hipEvent_t ev;
        ctx->tic("normals_lazy", &ev);
        if ((rc = run_normals(ctx, d_segs, int(segs.size()), d_cd, d_gg, int(grp.size()),
                              std::max<size_t>(tot, 1), normal_params(r, mnn), int64_t(tot),
                              "normals_lazy")))
            return rc;
        ctx->toc("normals_lazy", ev);
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
        LSM_HIP_TRY(ctx, hipGetLastError());
        for (Cloud *c : grp) c->lazy = false;
        todo.swap(rest);
    }
    ctx->collect_timings();
    return LSM_OK;
}

int lsm_download_run(lsm_ctx *ctx, Cloud *c, double *xyz, double *nrm, int64_t cap) {
    (void)cap;
    hipStream_t st = ctx->stream;
    const int n = int(c->n);
    if (n == 0) return LSM_OK;
    double *dx = (double *)ctx->buf("dl_xyz", size_t(n) * 24);
    double *dn = (double *)ctx->buf("dl_nrm", size_t(n) * 24);
    if (!dx || !dn) return LSM_ENOMEM;
    const bool xyz_from_vox = c->voxelized;
    download_kernel<<<(n + 255) / 256, 256, 0, st>>>(c->d_xyz, c->d_nrm, c->d_perm, n,
                                                     (xyz && !xyz_from_vox) ? dx : nullptr,
                                                     nrm ? dn : nullptr);
    if (xyz) {
        if (xyz_from_vox)
            LSM_HIP_TRY(ctx, hipMemcpyAsync(xyz, c->d_vox, size_t(n) * 24, hipMemcpyDeviceToHost, st));
        else
            LSM_HIP_TRY(ctx, hipMemcpyAsync(xyz, dx, size_t(n) * 24, hipMemcpyDeviceToHost, st));
    }
    if (nrm) LSM_HIP_TRY(ctx, hipMemcpyAsync(nrm, dn, size_t(n) * 24, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    return LSM_OK;
}

// ==========================================================================================
// FPFH: [O3D] ComputeFPFHFeature(cloud, KDTreeSearchParamHybrid(r, max_nn))
// ==========================================================================================
namespace {

// ComputePairFeatures (Rusu's Darboux frame), f64: (theta, alpha, phi); false when the points
// coincide or the frame degenerates (Open3D returns zeros then).
__device__ bool pair_features(const double *p1, const double *n1, const double *p2,
                              const double *n2, double f[3]) {
    double dp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    const double d = sqrt((dp[0] * dp[0] + dp[1] * dp[1]) + dp[2] * dp[2]);
    f[0] = f[1] = f[2] = 0.0;
    if (d == 0.0) return false;
    const double a1 = ((n1[0] * dp[0] + n1[1] * dp[1]) + n1[2] * dp[2]) / d;
    const double a2 = ((n2[0] * dp[0] + n2[1] * dp[1]) + n2[2] * dp[2]) / d;
    const double *m1 = n1, *m2 = n2;
    double phi = a1;
    if (acos(fabs(a1)) > acos(fabs(a2))) {
        m1 = n2;
        m2 = n1;
        dp[0] = -dp[0];
        dp[1] = -dp[1];
        dp[2] = -dp[2];
        phi = -a2;
    }
    double v[3] = {dp[1] * m1[2] - dp[2] * m1[1], dp[2] * m1[0] - dp[0] * m1[2],
                   dp[0] * m1[1] - dp[1] * m1[0]};
    const double vn = sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    if (vn == 0.0) return false;
    v[0] /= vn;
    v[1] /= vn;
    v[2] /= vn;
    const double w[3] = {m1[1] * v[2] - m1[2] * v[1], m1[2] * v[0] - m1[0] * v[2],
                         m1[0] * v[1] - m1[1] * v[0]};
    f[1] = (v[0] * m2[0] + v[1] * m2[1]) + v[2] * m2[2];
    f[0] = atan2((w[0] * m2[0] + w[1] * m2[1]) + w[2] * m2[2],
                 (m1[0] * m2[0] + m1[1] * m2[1]) + m1[2] * m2[2]);
    f[2] = phi;
    return true;
}

__device__ __forceinline__ int fbin(double v) {
    const int h = int(floor(v));
    return h < 0 ? 0 : (h >= 11 ? 10 : h);
}

// SPFH of every point: the pairs (point, neighbour) over its list without the point itself,
// 11 bins each of theta, alpha, phi, increment 100 / (k - 1) (k counts the point itself)
__global__ void __launch_bounds__(PT_THREADS)
spfh_kernel(const CloudDev *cd, const int32_t *__restrict__ idx, const int32_t *__restrict__ cnt,
            int cap, double *__restrict__ spfh) {
    const CloudDev C = cd[0];
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= C.n) return;
    double h[33];
#pragma unroll
    for (int b = 0; b < 33; ++b) h[b] = 0.0;
    const int k = cnt[j];
    if (k > 1) {
        const double incr = 100.0 / double(k - 1);
        const float4 pj = C.xyz[j], nj = C.nrm[j];
        const double p1[3] = {pj.x, pj.y, pj.z}, n1[3] = {nj.x, nj.y, nj.z};
        for (int e = 0; e < k; ++e) {
            const int q = idx[size_t(j) * cap + e];
            if (q == j) continue;
            const float4 pq = C.xyz[q], nq = C.nrm[q];
            const double p2[3] = {pq.x, pq.y, pq.z}, n2[3] = {nq.x, nq.y, nq.z};
            double f[3];
            pair_features(p1, n1, p2, n2, f);
            const double twopi = 2.0 * 3.14159265358979323846;
            const int b0 = fbin(11.0 * (f[0] + 3.14159265358979323846) / twopi);
            const int b1 = fbin(11.0 * (f[1] + 1.0) * 0.5);
            const int b2 = fbin(11.0 * (f[2] + 1.0) * 0.5);
#pragma unroll
            for (int b = 0; b < 11; ++b) {
                h[b] += b == b0 ? incr : 0.0;
                h[11 + b] += b == b1 ? incr : 0.0;
                h[22 + b] += b == b2 ? incr : 0.0;
            }
        }
    }
    for (int b = 0; b < 33; ++b) spfh[size_t(j) * 33 + b] = h[b];
}

// FPFH = SPFH(j) + the neighbours' SPFH weighted by 1 / d^2 and normalised to 100 per group of
// 11 bins; written in reference order (row perm[j]).
__global__ void __launch_bounds__(PT_THREADS)
fpfh_kernel(const CloudDev *cd, const int32_t *__restrict__ idx, const double *__restrict__ d2,
            const int32_t *__restrict__ cnt, int cap, const double *__restrict__ spfh,
            double *__restrict__ out) {
    const CloudDev C = cd[0];
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= C.n) return;
    double acc[33];
#pragma unroll
    for (int b = 0; b < 33; ++b) acc[b] = 0.0;
    const int k = cnt[j];
    double *o = out + size_t(C.perm[j]) * 33;
    if (k <= 1) {
        for (int b = 0; b < 33; ++b) o[b] = 0.0;
        return;
    }
    for (int e = 0; e < k; ++e) {
        const int q = idx[size_t(j) * cap + e];
        const double dd = d2[size_t(j) * cap + e];
        if (q == j || dd == 0.0) continue;
        const double *sq = spfh + size_t(q) * 33;
#pragma unroll
        for (int b = 0; b < 33; ++b) acc[b] += sq[b] / dd;
    }
    double s[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int b = 0; b < 33; ++b) s[b / 11] += acc[b];
#pragma unroll
    for (int g = 0; g < 3; ++g) s[g] = s[g] != 0.0 ? 100.0 / s[g] : 0.0;
    const double *sj = spfh + size_t(j) * 33;
#pragma unroll
    for (int b = 0; b < 33; ++b) o[b] = acc[b] * s[b / 11] + sj[b];
}

// Exact nearest feature (33-D, squared L2 summed in dimension order; ties -> lower index): one
// thread per query row, target rows staged through LDS in tiles.
constexpr int FT = 64;
__global__ void __launch_bounds__(PT_THREADS)
feature_nn_kernel(const double *__restrict__ a, int na, const double *__restrict__ b, int nb,
                  int32_t *__restrict__ nn) {
    __shared__ double tile[FT * 33];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double q[33];
    if (i < na)
        for (int d = 0; d < 33; ++d) q[d] = a[size_t(i) * 33 + d];
    double best = INFINITY;
    int bi = -1;
    for (int t0 = 0; t0 < nb; t0 += FT) {
        const int m = min(FT, nb - t0);
        __syncthreads();
        for (int e = threadIdx.x; e < m * 33; e += blockDim.x) tile[e] = b[size_t(t0) * 33 + e];
        __syncthreads();
        if (i < na) {
            for (int r = 0; r < m; ++r) {
                double s = 0.0;
#pragma unroll
                for (int d = 0; d < 33; ++d) {
                    const double e = q[d] - tile[r * 33 + d];
                    s += e * e;
                }
                if (s < best) {
                    best = s;
                    bi = t0 + r;
                }
            }
        }
    }
    if (i < na) nn[i] = bi;
}

// mutual filter: keep (i, ij[i]) when ji[ij[i]] == i, in increasing i (one workgroup)
__global__ void __launch_bounds__(1024)
mutual_kernel(const int32_t *__restrict__ ij, int na, const int32_t *__restrict__ ji,
              int32_t *__restrict__ out, uint32_t *__restrict__ nout) {
    __shared__ uint32_t wcnt[1024 / LSM_WAVE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < na; base += 1024) {
        const int i = base + int(threadIdx.x);
        const bool on = i < na && ij[i] >= 0 && ji[ij[i]] == i;
        const uint64_t m = __ballot(on);
        if (lane == 0) wcnt[w] = __popcll(m);
        __syncthreads();
        uint32_t before = carry, tot = 0;
        for (int q = 0; q < 1024 / LSM_WAVE; ++q) {
            before += q < w ? wcnt[q] : 0u;
            tot += wcnt[q];
        }
        if (on) {
            const uint32_t slot = before + __popcll(m & ((uint64_t(1) << lane) - 1));
            out[2 * slot] = i;
            out[2 * slot + 1] = ij[i];
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *nout = carry;
}

}  // namespace

int lsm_fpfh_run(lsm_ctx *ctx, Cloud *c, double radius, int max_nn) {
    hipStream_t st = ctx->stream;
    const int n = int(c->n);
    if (!c->d_fpfh || c->fpfh_cap < n) {
        (void)hipFree(c->d_fpfh);
        c->d_fpfh = nullptr;
        if (hipMalloc(&c->d_fpfh, size_t(std::max(n, 1)) * 33 * 8) != hipSuccess) {
            ctx->set_error("hipMalloc failed for FPFH features");
            return LSM_ENOMEM;
        }
        c->fpfh_cap = std::max(n, 1);
    }
    c->fpfh_n = n;
    if (n == 0) return LSM_OK;
    const int cap = std::max(max_nn, 1);
    int32_t *d_idx = (int32_t *)ctx->buf("fp_idx", size_t(n) * cap * 4);
    double *d_d2 = (double *)ctx->buf("fp_d2", size_t(n) * cap * 8);
    int32_t *d_cnt = (int32_t *)ctx->buf("fp_cnt", size_t(n) * 4);
    double *d_spfh = (double *)ctx->buf("fp_spfh", size_t(n) * 33 * 8);
    if (!d_idx || !d_d2 || !d_cnt || !d_spfh) return LSM_ENOMEM;
    std::vector<CloudDev> cdv(1, c->dev);
    cdv[0].nrm = c->d_nrm;
    CloudDev *d_cd;
    int rc;
    if ((rc = upload_vec(ctx, "fp_cd", cdv, &d_cd))) return rc;
    const SegTable segs =
        point_segments(ctx, "h_fpsegs", std::vector<uint32_t>(1, uint32_t(n)), PT_THREADS);
    Seg *d_segs;
    if ((rc = upload_vec(ctx, "fp_segs", segs, &d_segs))) return rc;
    NormalParams np;
    np.r2 = radius * radius;
    np.r = float(radius);
    np.r2_lo = float(np.r2 * (1.0 - 4e-6));
    np.r2_hi = float(np.r2 * (1.0 + 4e-6));
    np.hscale = float(double(NB8) / np.r2);
    np.max_nn = max_nn;
    np.dense_k = dense_k(max_nn, np.r2);
    np.preclass = normals_preclass();
    hipEvent_t ev;
    ctx->tic("fpfh", &ev);
    nbr_lists_kernel<<<int(segs.size()), PT_THREADS, 0, st>>>(d_segs, d_cd, np, d_idx, d_d2, d_cnt,
                                                              cap);
    const int g = (n + PT_THREADS - 1) / PT_THREADS;
    spfh_kernel<<<g, PT_THREADS, 0, st>>>(d_cd, d_idx, d_cnt, cap, d_spfh);
    fpfh_kernel<<<g, PT_THREADS, 0, st>>>(d_cd, d_idx, d_d2, d_cnt, cap, d_spfh, c->d_fpfh);
    ctx->toc("fpfh", ev);
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    LSM_HIP_TRY(ctx, hipGetLastError());
    ctx->collect_timings();
    return LSM_OK;
}

int lsm_feature_corr_run(lsm_ctx *ctx, Cloud *s, Cloud *t, int mutual, int ransac_n,
                         int32_t *out, int64_t cap, int64_t *n_out) {
    hipStream_t st = ctx->stream;
    const int na = int(s->fpfh_n), nb = int(t->fpfh_n);
    int32_t *d_ij = (int32_t *)ctx->buf("fc_ij", size_t(std::max(na, 1)) * 4);
    int32_t *d_ji = (int32_t *)ctx->buf("fc_ji", size_t(std::max(nb, 1)) * 4);
    int32_t *d_out = (int32_t *)ctx->buf("fc_out", size_t(std::max(na, 1)) * 8);
    uint32_t *d_n = (uint32_t *)ctx->buf("fc_n", 4);
    if (!d_ij || !d_ji || !d_out || !d_n) return LSM_ENOMEM;
    *n_out = 0;
    if (na == 0 || nb == 0) return LSM_OK;
    hipEvent_t ev;
    ctx->tic("feature_nn", &ev);
    feature_nn_kernel<<<(na + PT_THREADS - 1) / PT_THREADS, PT_THREADS, 0, st>>>(s->d_fpfh, na,
                                                                               t->d_fpfh, nb, d_ij);
    std::vector<int32_t> h;
    uint32_t nm = 0;
    if (mutual) {
        feature_nn_kernel<<<(nb + PT_THREADS - 1) / PT_THREADS, PT_THREADS, 0, st>>>(
            t->d_fpfh, nb, s->d_fpfh, na, d_ji);
        mutual_kernel<<<1, 1024, 0, st>>>(d_ij, na, d_ji, d_out, d_n);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(&nm, d_n, 4, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    }
    ctx->toc("feature_nn", ev);
    if (mutual && int64_t(nm) >= int64_t(3) * ransac_n) {
        h.resize(size_t(nm) * 2);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(h.data(), d_out, h.size() * 4, hipMemcpyDeviceToHost, st));
    } else {   // too few mutual pairs (or no filter): every source feature's nearest
        std::vector<int32_t> ij(na);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(ij.data(), d_ij, size_t(na) * 4, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
        h.resize(size_t(na) * 2);
        for (int i = 0; i < na; ++i) {
            h[2 * i] = i;
            h[2 * i + 1] = ij[i];
        }
    }
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    ctx->collect_timings();
    const int64_t m = int64_t(h.size() / 2);
    *n_out = m;
    if (out) std::memcpy(out, h.data(), size_t(std::min(m, cap)) * 8);
    return LSM_OK;
}

// ------------------------------------------------------------------------------------------
// voxel_down_sample of a cloud with normals: the second voxelisation of preprocess_fpfh
// (keyframe.py:202-203). [O3D] VoxelDownSample on a cloud with normals: the same keys and
// per-voxel point means as the first pass (voxel_keys / voxel_reduce), and per voxel the sum of
// the members' non-NaN normals divided by the member count (AccumulatedPoint::GetAverageNormal:
// not re-normalised). Input points are the cloud's reference-order f64 points (the first pass's
// centroids for a voxelised cloud).
// ------------------------------------------------------------------------------------------
namespace {

__global__ void __launch_bounds__(256)
vn_ref_kernel(const float4 *xyz, const float4 *nrm, const uint32_t *perm, int n, double *P,
              double *N) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t r = perm[j];
    if (P) {
        const float4 p = xyz[j];
        P[3 * r] = p.x;
        P[3 * r + 1] = p.y;
        P[3 * r + 2] = p.z;
    }
    const float4 v = nrm[j];
    N[3 * r] = v.x;
    N[3 * r + 1] = v.y;
    N[3 * r + 2] = v.z;
}

__global__ void __launch_bounds__(256)
vn_bbox_kernel(const double *P, int n, double *bb) {
    __shared__ double red[6][256];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = threadIdx.x; i < n; i += 256)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], P[3 * i + a]);
            hi[a] = fmax(hi[a], P[3 * i + a]);
        }
    for (int a = 0; a < 3; ++a) {
        red[a][threadIdx.x] = lo[a];
        red[3 + a][threadIdx.x] = hi[a];
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s)
            for (int a = 0; a < 3; ++a) {
                red[a][threadIdx.x] = fmin(red[a][threadIdx.x], red[a][threadIdx.x + s]);
                red[3 + a][threadIdx.x] = fmax(red[3 + a][threadIdx.x], red[3 + a][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) bb[threadIdx.x] = red[threadIdx.x][0];
}

__global__ void __launch_bounds__(256)
vn_keys_kernel(const double *P, int n, VoxGeo G, double v, uint64_t *keys, uint32_t *vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t kx = (int64_t)(int)floor(lsm_ddiv(lsm_dsub(P[3 * i], G.ox), v));
    const int64_t ky = (int64_t)(int)floor(lsm_ddiv(lsm_dsub(P[3 * i + 1], G.oy), v));
    const int64_t kz = (int64_t)(int)floor(lsm_ddiv(lsm_dsub(P[3 * i + 2], G.oz), v));
    keys[i] = uint64_t((kx * G.dy + ky) * G.dz + kz);
    vals[i] = uint32_t(i);
}

__global__ void __launch_bounds__(256)
vn_reduce_kernel(const uint64_t *skeys, const uint32_t *svals, const uint32_t *vid,
                 const uint32_t *flag, uint32_t n, const double *P, const double *N, VoxGeo G,
                 double *cent, int32_t *vkeys, float *raw, float4 *avgn) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint64_t key = skeys[i];
    double s[3] = {0.0, 0.0, 0.0}, t[3] = {0.0, 0.0, 0.0};
    uint32_t j = i;
    for (; j < n && skeys[j] == key; ++j) {   // members in index order (stable sort)
        const uint32_t m = svals[j];
        for (int a = 0; a < 3; ++a) s[a] = lsm_dadd(s[a], P[3 * m + a]);
        const double nx = N[3 * m], ny = N[3 * m + 1], nz = N[3 * m + 2];
        if (!isnan(nx) && !isnan(ny) && !isnan(nz)) {
            t[0] = lsm_dadd(t[0], nx);
            t[1] = lsm_dadd(t[1], ny);
            t[2] = lsm_dadd(t[2], nz);
        }
    }
    const double cnt = double(j - i);
    const uint32_t o = vid[i];
    double c[3], a3[3];
    for (int a = 0; a < 3; ++a) {
        c[a] = lsm_ddiv(s[a], cnt);
        a3[a] = lsm_ddiv(t[a], cnt);
        cent[3 * o + a] = c[a];
        raw[3 * o + a] = float(c[a]);
    }
    vkeys[3 * o] = int32_t(int64_t(key / uint64_t(G.dz * G.dy)));
    vkeys[3 * o + 1] = int32_t(int64_t((key / uint64_t(G.dz)) % uint64_t(G.dy)));
    vkeys[3 * o + 2] = int32_t(int64_t(key % uint64_t(G.dz)));
    avgn[o] = make_float4(float(a3[0]), float(a3[1]), float(a3[2]), 0.f);
}

// normals of a processed cloud from reference-order values: nrm[j] = src[perm[j]]
__global__ void __launch_bounds__(256)
vn_adopt_kernel(const float4 *src, const uint32_t *perm, int n, float4 *nrm) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) nrm[j] = src[perm[j]];
}

}  // namespace

int lsm_voxel_normals_run(lsm_ctx *ctx, Cloud *c, double v, Cloud *o) {
    hipStream_t st = ctx->stream;
    if (!(v > 0.0)) {
        ctx->set_error("voxel_size <= 0.");
        return LSM_EINVAL;
    }
    const int n = int(c->n);
    double *P = c->voxelized ? c->d_vox : (double *)ctx->buf("vn_P", size_t(std::max(n, 1)) * 24);
    double *N = (double *)ctx->buf("vn_N", size_t(std::max(n, 1)) * 24);
    double *d_bb = (double *)ctx->buf("vn_bb", 48);
    if (!P || !N || !d_bb) return LSM_ENOMEM;
    VoxGeo G = {0.0, 0.0, 0.0, 1, 1, 1, 0};
    uint32_t nvox = 0;
    double *cent = nullptr;
    int32_t *vkeys = nullptr;
    float *raw = nullptr;
    float4 *avgn = nullptr;
    if (n > 0) {
        const int nb = (n + 255) / 256;
        vn_ref_kernel<<<nb, 256, 0, st>>>(c->d_xyz, c->d_nrm, c->d_perm, n,
                                          c->voxelized ? nullptr : P, N);
        vn_bbox_kernel<<<1, 256, 0, st>>>(P, n, d_bb);
        double bb[6];
        LSM_HIP_TRY(ctx, hipMemcpyAsync(bb, d_bb, 48, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
        // the same geometry as run_voxel (Open3D's min_bound - v/2 origin and its range check)
        const double half = v * 0.5;
        double vmin[3], vmax[3];
        for (int a = 0; a < 3; ++a) {
            vmin[a] = bb[a] - half;
            vmax[a] = bb[3 + a] + half;
        }
        const double ext = std::max(vmax[0] - vmin[0], std::max(vmax[1] - vmin[1], vmax[2] - vmin[2]));
        if (v * double(std::numeric_limits<int>::max()) < ext) {
            ctx->set_error("voxel_size is too small.");
            return LSM_EINVAL;
        }
        int64_t d[3];
        for (int a = 0; a < 3; ++a) d[a] = (int64_t)std::floor((bb[3 + a] - vmin[a]) / v) + 2;
        const uint64_t cells = uint64_t(d[0]) * uint64_t(d[1]) * uint64_t(d[2]);
        if (cells > (uint64_t(1) << 44)) {
            ctx->set_error("voxel grid too large for the 64-bit key space");
            return LSM_EINVAL;
        }
        G = {vmin[0], vmin[1], vmin[2], d[0], d[1], d[2], 0};
        uint64_t *k_in = (uint64_t *)ctx->buf("v_kin", size_t(n) * 8);
        uint64_t *k_out = (uint64_t *)ctx->buf("v_kout", size_t(n) * 8);
        uint32_t *v_in = (uint32_t *)ctx->buf("v_vin", size_t(n) * 4);
        uint32_t *v_out = (uint32_t *)ctx->buf("v_vout", size_t(n) * 4);
        uint32_t *flag = (uint32_t *)ctx->buf("v_flag", size_t(n) * 4 + 4);
        uint32_t *vid = (uint32_t *)ctx->buf("v_vid", size_t(n) * 4 + 4);
        cent = (double *)ctx->buf("vn_cent", size_t(n) * 24);
        vkeys = (int32_t *)ctx->buf("vn_keys", size_t(n) * 12);
        raw = (float *)ctx->buf("vn_raw", size_t(n) * 12);
        avgn = (float4 *)ctx->buf("vn_avgn", size_t(n) * 16);
        if (!k_in || !k_out || !v_in || !v_out || !flag || !vid || !cent || !vkeys || !raw || !avgn) {
            ctx->set_error("scratch allocation failed (voxel normals)");
            return LSM_ENOMEM;
        }
        vn_keys_kernel<<<nb, 256, 0, st>>>(P, n, G, v, k_in, v_in);
        size_t tmpb = 0;
        const int endbit = bits_for(cells);
        LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs(nullptr, tmpb, k_in, k_out, v_in, v_out, size_t(n), 0,
                                                   endbit, st));
        void *tmp = ctx->buf("sort_tmp", tmpb);
        if (!tmp) return LSM_ENOMEM;
        LSM_HIP_TRY(ctx, rocprim::radix_sort_pairs(tmp, tmpb, k_in, k_out, v_in, v_out, size_t(n), 0,
                                                   endbit, st));
        voxel_flags<<<nb, 256, 0, st>>>(k_out, uint32_t(n), flag);
        LSM_HIP_TRY(ctx, hipMemsetAsync(flag + n, 0, 4, st));
        tmpb = 0;
        LSM_HIP_TRY(ctx, rocprim::exclusive_scan(nullptr, tmpb, flag, vid, 0u, size_t(n) + 1,
                                                 rocprim::plus<uint32_t>(), st));
        tmp = ctx->buf("scan_tmp", tmpb);
        if (!tmp) return LSM_ENOMEM;
        LSM_HIP_TRY(ctx, rocprim::exclusive_scan(tmp, tmpb, flag, vid, 0u, size_t(n) + 1,
                                                 rocprim::plus<uint32_t>(), st));
        vn_reduce_kernel<<<nb, 256, 0, st>>>(k_out, v_out, vid, flag, uint32_t(n), P, N, G, cent,
                                             vkeys, raw, avgn);
        LSM_HIP_TRY(ctx, hipMemcpyAsync(&nvox, vid + n, 4, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    }
    // the output: a raw cloud of the f32 centroids carrying the averaged normals, pre-processed
    // with a keep-all filter (grid only), then given those normals and the f64 centroids / keys
    const int64_t m = std::max<int64_t>(nvox, 1);
    if (hipMalloc(&o->d_raw, size_t(m) * 12) != hipSuccess ||
        hipMalloc(&o->d_prior_ref, size_t(m) * 16) != hipSuccess ||
        hipMalloc(&o->d_vox, size_t(m) * 24) != hipSuccess ||
        hipMalloc(&o->d_vkeys, size_t(m) * 12) != hipSuccess) {
        ctx->set_error("hipMalloc failed (voxel normals)");
        return LSM_ENOMEM;
    }
    o->vox_cap = m;
    o->n_raw = nvox;
    o->prior_n = nvox;
    if (nvox) {
        LSM_HIP_TRY(ctx, hipMemcpyAsync(o->d_raw, raw, size_t(nvox) * 12, hipMemcpyDeviceToDevice, st));
        LSM_HIP_TRY(ctx, hipMemcpyAsync(o->d_prior_ref, avgn, size_t(nvox) * 16, hipMemcpyDeviceToDevice, st));
        LSM_HIP_TRY(ctx, hipMemcpyAsync(o->d_vox, cent, size_t(nvox) * 24, hipMemcpyDeviceToDevice, st));
        LSM_HIP_TRY(ctx, hipMemcpyAsync(o->d_vkeys, vkeys, size_t(nvox) * 12, hipMemcpyDeviceToDevice, st));
    }
    lsm_prep_params kp;
    lsm_default_prep_params(&kp);
    kp.min_radius = -INFINITY;   // keep-all: no lower radius bound (a centroid may sit at x = y = 0)
    kp.max_radius = 1e15;
    kp.min_height = -1e15;
    kp.max_height = 1e15;
    kp.voxel_size = 0.0;
    kp.want_normals = 0;
    kp.grid_cell = 0.0;
    std::vector<Cloud *> one{o};
    int rc = lsm_prep_batch(ctx, one, kp, nullptr);
    if (rc) return rc;
    if (o->n != int64_t(nvox)) {   // cannot happen with the keep-all bounds above
        ctx->set_error("internal: voxel_down_sample with normals lost centroids");
        return LSM_EHIP;
    }
    if ((rc = ensure_cloud_buffers(ctx, o, o->n, true))) return rc;
    if (nvox)
        vn_adopt_kernel<<<(int(nvox) + 255) / 256, 256, 0, st>>>(o->d_prior_ref, o->d_perm, int(nvox),
                                                                 o->d_nrm);
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    LSM_HIP_TRY(ctx, hipGetLastError());
    o->dev.nrm = o->d_nrm;
    o->dev.xyz64 = o->d_vox;   // normals estimated on it later see the f64 centroids
    o->has_normals = true;
    o->voxelized = true;
    return LSM_OK;
}
