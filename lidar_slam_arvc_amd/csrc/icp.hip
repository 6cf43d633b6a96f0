// icp.hip -- registration_icp on the device (keyframe.py:231-260 -> [O3D] RegistrationICP),
// batched over independent keyframe pairs.
//
// One correspondence pass (GetRegistrationResultAndCorrespondences) + one update
// (TransformationEstimationPointToPlane / PointToPoint::ComputeTransformation) per launch group:
//
//   nn_kernel          one lane per source point: transform by the pair's T (f64), exact 1-NN in
//                      the target's cell grid (own cell, then the 26 neighbours pruned by their
//                      lower-bound distance). A query whose nearest point is provably inside the
//                      3x3x3 block is resolved; the rest (a few %) go to a queue.
//   nn_fallback_g      32 lanes (or a wave) per queued query: expanding boxes, the group strides over each
//                      cell row, (d2, index) wave-min -> exact nearest within max_corr.
//   accumulate         one lane per source point: f64 residual / Jacobian of the correspondence,
//                      fixed-tree wave + LDS reduction into per-block partials (deterministic).
//   solve              one wave per pair: ordered sum of the pair's partials, fitness / rmse,
//                      Open3D's convergence rule, Eigen-style LDLT (P2Plane) or Horn/Umeyama
//                      (P2P), T <- dT * T.
//
// Correspondences use d^2 < max_corr^2 (SearchHybrid + lower_bound); fitness = |C| / N_src,
// inlier_rmse = sqrt(sum d^2 / |C|) (0, 0 when C is empty); empty C -> identity update.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <type_traits>
#include <vector>

#include "lsm_ctx.h"
#include "lsm_umeyama.h"

namespace {

constexpr int NN_THREADS = 256;
constexpr int NXCD = 8;

struct NNParams {
    float maxc2;       // max_correspondence_distance^2 (f32, correspondence test)
    float maxc;        // max_correspondence_distance
    int method;
    int max_iter;
    double rel_fit, rel_rmse;
    int split_max;     // most lanes one uncertified query's box search is split over
    int split_place;   // where the split groups sit in the workgroup (LSM_NN_SPLIT_PLACE)
    float m0;          // rho margin of the searches without a previous pass (see prune2)
    uint32_t lin;      // runs of at most this many points are scanned whole (no entry search)
    double m_mul, m_add;   // rho margin of a search after a pass that moved the query by dq
    float direct_rc;   // warm-start distance (cells) from which a query skips the box search
    int direct_iter;   // ... once its pair has made this many updates
    int kcold, kmax;   // box half-widths (cells): cold start, largest warm box
    int cold_seed;     // seed cold searches with a point of the query's own cell
    int hmax;          // transform-history slots per pair (max_iteration + 2)
};

// Correspondence state of one source point, carried from pass to pass (SoA arrays):
//   corr[i]  nearest target point (sorted index), -1 = none within max_corr
//   rec[i]   8 bytes: the search's second-nearest point alt (sorted index, or none), the pass s
//            of the search that left the record, and rho: a lower bound on the distance from
//            q_s to every target point other than corr[i] and alt (to every point when corr[i]
//            = -1), metres. q_s, the f32 query point of that search, is not stored: it is
//            recomputed from the pair's transform at pass s (the transform history), the same
//            f64 transform of the same source point, so bit for bit the point the search used.
// Stability certificate: if the query now sits at q with D = |q - q_s|, the nearer w of corr[i]
// and alt[i] (exact f32 (d2, index) order) is the nearest neighbour whenever |q - w| + D < rho:
// every other point is at least rho - D away. The pair only swaps places when alt[i] wins. Later
// ICP passes move the source by micrometres to millimetres, so nearly every query of a
// converging pair is certified with a few loads; the second point keeps queries whose nearest
// neighbour flips between two close target points certified.
struct FallbackItem {
    int32_t pair;
    int32_t i;        // source point (sorted order)
    int32_t best;     // best target index found by the box search (-1 none)
    float best_d2;
    float second_d2;  // second-smallest distance examined (a point other than best)
    float margin;     // rho margin of this query (see prune2)
};

// rec[i] = (alt | s << 24, rho bits); alt 0xFFFFFF = none (target clouds hold < 2^24 - 1 points,
// passes < 256: the host checks both, else every pass searches every query)
constexpr uint32_t REC_NONE = 0xFFFFFFu;
constexpr int REC_SHIFT = 24;
__device__ __forceinline__ int2 rec_pack(int alt, int pass, float rho) {
    return make_int2(int((alt < 0 ? REC_NONE : uint32_t(alt)) | (uint32_t(pass) << REC_SHIFT)),
                     __float_as_int(rho));
}
// transforms of a pair per pass (12 doubles: the top 3 rows), hist[(pair * hmax + pass) * 12]
constexpr int HIST_STRIDE = 12;

__device__ __forceinline__ bool better(float d2, int idx, float bd2, int bidx) {
    return d2 < bd2 || (d2 == bd2 && idx < bidx);
}

// T . p in f64 with ONE fixed rounding sequence (explicit fmas, no compiler contraction): the
// certificate check recomputes a search's query point from the transform history and relies on
// getting the search's point bit for bit, whichever call site (and inlining) computed it.
__device__ __forceinline__ void transform_point(const double *T, float4 p, double &x, double &y,
                                                double &z) {
#pragma clang fp contract(off)
    const double px = p.x, py = p.y, pz = p.z;
    x = __builtin_fma(T[2], pz, __builtin_fma(T[1], py, __builtin_fma(T[0], px, T[3])));
    y = __builtin_fma(T[6], pz, __builtin_fma(T[5], py, __builtin_fma(T[4], px, T[7])));
    z = __builtin_fma(T[10], pz, __builtin_fma(T[9], py, __builtin_fma(T[8], px, T[11])));
}

// Running (nearest, second-nearest) over examined target points (the fallback's search state).
// A point is examined at most once as the current best (k == bidx is skipped: the warm-start
// point is revisited by the box scan), so the second distance always belongs to a different point.
// `lim` caches prune2(): the squared pruning radius, refreshed whenever bd2 or sd2 changes.
struct Top2 {
    float bd2;
    int bidx;
    float sd2;
    float lim;
    float m;   // margin of prune2
};

// Squared pruning radius of a search: the second-best distance, capped at (best + m)^2 and
// never below the best (ties with the best are always examined, so the (d2, index) minimum is
// exact). Every point the search skips is at least this far, so it is a valid rho (the radius
// only shrinks during a search). m = 0 gives a plain nearest-neighbour search (rho = best
// distance: certifies nothing); m = (this pass's displacement) + 1 mm leaves room for the
// next passes' motion.
__device__ __forceinline__ float prune2(float bd2, float sd2, float m) {
    const float c = __builtin_amdgcn_sqrtf(bd2) + m;
    return fmaxf(bd2, fminf(sd2, c * c));
}

__device__ __forceinline__ Top2 top2_init(int bidx, float bd2, float sd2, float m) {
    return Top2{bd2, bidx, sd2, prune2(bd2, sd2, m), m};
}

__device__ __forceinline__ void top2_add(float d2, int k, Top2 &b) {
    if (k == b.bidx || !(d2 < b.sd2 || (d2 == b.bd2 && k < b.bidx))) return;
    if (better(d2, k, b.bd2, b.bidx)) {
        b.sd2 = b.bd2;
        b.bd2 = d2;
        b.bidx = k;
    } else {
        b.sd2 = d2;
    }
    b.lim = prune2(b.bd2, b.sd2, b.m);
}

// The box search's state: nearest and second-nearest points (both with indices, in (d2, index)
// order) and the third-smallest distance examined. Pruning at the third distance (capped at
// (best + m)^2, as prune2) makes the search's rho a bound on every point other than the two, so
// the certificate can follow the nearest neighbour when it flips to the second point.
struct Top3 {
    float bd2;
    int bidx;
    float sd2;
    int sidx;
    float td2;
    float lim;   // prune2(bd2, td2, m)
    float m;
};

__device__ __forceinline__ Top3 top3_init(int bidx, float bd2, float m) {
    return Top3{bd2, bidx, INFINITY, -1, INFINITY, prune2(bd2, INFINITY, m), m};
}

__device__ __forceinline__ void top_add(float d2, int k, Top3 &b) {
    if (k == b.bidx || k == b.sidx || !(d2 <= b.td2)) return;
    if (better(d2, k, b.bd2, b.bidx)) {
        b.td2 = b.sd2;
        b.sd2 = b.bd2;
        b.sidx = b.bidx;
        b.bd2 = d2;
        b.bidx = k;
    } else if (better(d2, k, b.sd2, b.sidx)) {
        b.td2 = b.sd2;
        b.sd2 = d2;
        b.sidx = k;
    } else {
        b.td2 = d2;
    }
    b.lim = prune2(b.bd2, b.td2, b.m);
}

// The f32 squared distance that ranks candidates: ONE fixed rounding sequence (explicit fmas,
// no compiler contraction), so every search path -- box search, walks in either direction,
// fallback, warm start, certificate -- computes bit-identical values and exact (d2, index) ties
// resolve the same way everywhere (hipcc contracts a * b + c per call site otherwise).
__device__ __forceinline__ float sqd(const float4 t, float qx, float qy, float qz) {
#pragma clang fp contract(off)
    const float dx = qx - t.x, dy = qy - t.y, dz = qz - t.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// One x-sorted run [a, b) of a cell row whose slab is at least dyz2 (squared, underestimated)
// from the query: enter at the query's x (binary search on long runs) and walk outwards while
// dx^2 + dyz2 <= the pruning radius (strict '>' stops: equal distances are still examined, so
// (d2, index) ties resolve exactly as a full scan would).

// Search statistics (LSM_NN_STATS=1, diagnostics only): per lane, reduced per wave at the end.
struct NNStat {
    uint32_t v[8];   // searched, rows, runs, bsearch steps, points, sum K, cold, pending
};
constexpr int NN_NSTAT = 8;
#define NN_ST(ns, c, x) \
    do {                \
        if (ns) (ns)->v[c] += (x); \
    } while (0)

// Loads are issued NN_G at a time (independent addresses: one memory round trip per group rather
// than per point); a group may read up to NN_G - 1 points past the walk's stop, never past the
// run. Short runs (<= lin points) are scanned whole.
#ifndef LSM_NN_G
#define LSM_NN_G 2
#endif
constexpr int NN_G = LSM_NN_G;
// LSM_NN_PF: software-pipelined walks (scan_run). Measured per 1999-pair step: G 4 104.8 ms,
// G 2 108.8, G 2 + prefetch 94.3, G 1 / 3 / 4 + prefetch 103.4 / 108.2 / 128.3 (registers)
#ifndef LSM_NN_PF
#define LSM_NN_PF 1
#endif
// LSM_NN_BUF: the box walks read the target through a buffer descriptor (32-bit offsets)
#ifndef LSM_NN_BUF
#define LSM_NN_BUF 1
#endif

template <typename Rd>
__device__ __forceinline__ void scan_run(const Rd &xyz, uint32_t a, uint32_t b, float qx,
                                         float qy, float qz, float dyz2, Top3 &t2, uint32_t lin,
                                         NNStat *ns = nullptr) {
    NN_ST(ns, 2, 1);
    if (b - a <= lin) {
        NN_ST(ns, 4, b - a);
        for (uint32_t k = a; k < b; k += NN_G) {
            float4 t[NN_G];
#pragma unroll
            for (int g = 0; g < NN_G; ++g) t[g] = xyz.pt(min(k + uint32_t(g), b - 1));
#pragma unroll
            for (int g = 0; g < NN_G; ++g)
                if (k + uint32_t(g) < b) top_add(sqd(t[g], qx, qy, qz), int(k + uint32_t(g)), t2);
        }
        return;
    }
    uint32_t lo = a, hi = b;
    while (lo < hi) {
        NN_ST(ns, 3, 1);
        const uint32_t mid = (lo + hi) >> 1;
        if (xyz.x(mid) < qx) lo = mid + 1;
        else hi = mid;
    }
    // rightwards from lo (x >= qx), then leftwards from lo - 1 (x < qx). LSM_NN_PF: the first
    // groups of both walks are loaded together, and each walk loads its next group before
    // testing the current one (loads clamped to the run).
#if LSM_NN_PF == 2
    // the same walks over two register buffers each (the next group loads into the buffer not
    // being tested: no copies rotate the pipeline)
    float4 ra[NN_G], rb[NN_G], la[NN_G], lb[NN_G];
#pragma unroll
    for (int g = 0; g < NN_G; ++g) {
        ra[g] = xyz.pt(min(lo + uint32_t(g), b - 1));
        la[g] = xyz.pt(uint32_t(max(int(lo) - 1 - g, int(a))));
    }
    auto right = [&](const float4 (&t)[NN_G], uint32_t k) {
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            const float dx = t[g].x - qx;
            if (k + uint32_t(g) >= b || dx * dx + dyz2 > t2.lim) return false;
            NN_ST(ns, 4, 1);
            top_add(sqd(t[g], qx, qy, qz), int(k + uint32_t(g)), t2);
        }
        return true;
    };
    auto left = [&](const float4 (&t)[NN_G], int k) {
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            const float dx = qx - t[g].x;
            if (k - g < int(a) || dx * dx + dyz2 > t2.lim) return false;
            NN_ST(ns, 4, 1);
            top_add(sqd(t[g], qx, qy, qz), k - g, t2);
        }
        return true;
    };
    for (uint32_t k = lo; k < b;) {
#pragma unroll
        for (int g = 0; g < NN_G; ++g) rb[g] = xyz.pt(min(k + uint32_t(NN_G + g), b - 1));
        if (!right(ra, k)) break;
        k += NN_G;
        if (k >= b) break;
#pragma unroll
        for (int g = 0; g < NN_G; ++g) ra[g] = xyz.pt(min(k + uint32_t(NN_G + g), b - 1));
        if (!right(rb, k)) break;
        k += NN_G;
    }
    for (int k = int(lo) - 1; k >= int(a);) {
#pragma unroll
        for (int g = 0; g < NN_G; ++g) lb[g] = xyz.pt(uint32_t(max(k - NN_G - g, int(a))));
        if (!left(la, k)) break;
        k -= NN_G;
        if (k < int(a)) break;
#pragma unroll
        for (int g = 0; g < NN_G; ++g) la[g] = xyz.pt(uint32_t(max(k - NN_G - g, int(a))));
        if (!left(lb, k)) break;
        k -= NN_G;
    }
    return;
#endif
#if LSM_NN_PF
    float4 r[NN_G], l[NN_G];
#pragma unroll
    for (int g = 0; g < NN_G; ++g) {
        r[g] = xyz.pt(min(lo + uint32_t(g), b - 1));
        l[g] = xyz.pt(uint32_t(max(int(lo) - 1 - g, int(a))));
    }
#endif
    for (uint32_t k = lo; k < b; k += NN_G) {
        float4 t[NN_G];
#if LSM_NN_PF
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            t[g] = r[g];
            r[g] = xyz.pt(min(k + uint32_t(NN_G + g), b - 1));
        }
#else
#pragma unroll
        for (int g = 0; g < NN_G; ++g) t[g] = xyz.pt(min(k + uint32_t(g), b - 1));
#endif
        bool stop = false;
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            if (!stop) {
                const float dx = t[g].x - qx;
                if (k + uint32_t(g) >= b || dx * dx + dyz2 > t2.lim) {
                    stop = true;
                } else {
                    NN_ST(ns, 4, 1);
                    top_add(sqd(t[g], qx, qy, qz), int(k + uint32_t(g)), t2);
                }
            }
        }
        if (stop) break;
    }
    for (int k = int(lo) - 1; k >= int(a); k -= NN_G) {
        float4 t[NN_G];
#if LSM_NN_PF
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            t[g] = l[g];
            l[g] = xyz.pt(uint32_t(max(k - NN_G - g, int(a))));
        }
#else
#pragma unroll
        for (int g = 0; g < NN_G; ++g) t[g] = xyz.pt(uint32_t(max(k - g, int(a))));
#endif
        bool stop = false;
#pragma unroll
        for (int g = 0; g < NN_G; ++g) {
            if (!stop) {
                const float dx = qx - t[g].x;
                if (k - g < int(a) || dx * dx + dyz2 > t2.lim) {
                    stop = true;
                } else {
                    NN_ST(ns, 4, 1);
                    top_add(sqd(t[g], qx, qy, qz), k - g, t2);
                }
            }
        }
        if (stop) break;
    }
}

// Conservative lower-bound radius from a squared f32 distance / an f32 box bound (metres):
// covers the f32 rounding of distances and of the grid's cell coordinates.
__device__ __forceinline__ float rho_from(float d2, float bound) {
    const float r = fminf(sqrtf(d2), bound);
    return r == INFINITY ? INFINITY : fmaxf(r * (1.f - 1e-5f) - 2e-5f, 0.f);
}

// squared distance (in cells^2) from fractional coordinate f to cell k's slab [k, k+1)
__device__ __forceinline__ float slab_cells2(float f, int k) {
    const float d = f < float(k) ? float(k) - f : (f > float(k + 1) ? f - float(k + 1) : 0.f);
    return d * d;
}


// ------------------------------------------------------------------------------------------
// device-side work plan: the blocks of the pairs still iterating, balanced over the XCDs
// ------------------------------------------------------------------------------------------
// Logical block g (pair order, active pairs only) lives in XCD lane l = g / per at position
// m = g % per; grid slot t = 8 m + l, so consecutive workgroups (round-robin over the 8 XCDs)
// take one lane each: a pair stays on one or two XCDs (its target stays in those L2s) and a
// lone straggler pair still spreads over the whole chip. Rebuilt on the device after every
// solve, so the host never waits between passes.
struct TaskPlan {
    const int32_t *plan;   // [0] active blocks, [1] per-lane blocks
    const int32_t *pref;   // [npairs + 1] prefix of the active pairs' block counts
    const int4 *coarse;    // [c] (pair, pref[pair], pref[pair + 1], blk0) of the pair holding
                           // active block c * PLAN_COARSE
    int npairs;
    int32_t *err;          // set by a one-task-per-workgroup kernel launched on too small a grid
};

constexpr int PLAN_THREADS = 1024;
// block -> pair lookup: the pair of every PLAN_COARSE-th block is tabled, the rest is a short
// forward walk over the prefix (replaces an 11-step binary search over 2000 pairs, a chain of
// dependent loads at the start of every workgroup of the per-pass kernels)
constexpr int PLAN_COARSE = 64;

__global__ void __launch_bounds__(PLAN_THREADS)
plan_kernel(const PairState *__restrict__ st, int npairs, int32_t *__restrict__ pref,
            int4 *__restrict__ coarse, int32_t *__restrict__ plan,
            const uint32_t *__restrict__ active = nullptr, int32_t *poll = nullptr) {
    __shared__ int32_t wsum[PLAN_THREADS / LSM_WAVE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int32_t carry = 0;
    for (int base = 0; base < npairs; base += PLAN_THREADS) {
        const int k = base + threadIdx.x;
        const int32_t v = (k < npairs && st[k].active) ? st[k].nblk : 0;
        int32_t x = v;   // inclusive wave scan
#pragma unroll
        for (int off = 1; off < LSM_WAVE; off <<= 1) {
            const int32_t y = __shfl_up(x, off, LSM_WAVE);
            if (lane >= off) x += y;
        }
        if (lane == LSM_WAVE - 1) wsum[w] = x;
        __syncthreads();
        int32_t before = carry, tot = 0;
        for (int q = 0; q < PLAN_THREADS / LSM_WAVE; ++q) {
            before += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        if (k < npairs) {
            pref[k + 1] = before + x;
            // coarse entries c with pref[k] <= c * PLAN_COARSE < pref[k + 1]
            for (int32_t c = (before + x - v + PLAN_COARSE - 1) / PLAN_COARSE;
                 c * PLAN_COARSE < before + x; ++c)
                coarse[c] = make_int4(k, before + x - v, before + x, st[k].blk0);
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pref[0] = 0;
        plan[0] = carry;
        plan[1] = (carry + NXCD - 1) / NXCD;
        if (poll) {   // host-mapped pinned words the host polls (no copy dispatches per pass)
            __hip_atomic_store(poll, int32_t(*active), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(poll + 1, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
        }
    }
}

// grid slot t -> block task: 1 = work, 0 = padding, -1 = past the end of the plan
__device__ __forceinline__ int plan_task(const TaskPlan &tp, const PairState *st, int t,
                                         BlockTask &task) {
    const int32_t total = tp.plan[0], per = tp.plan[1];
    const int l = t & (NXCD - 1), m = t / NXCD;
    if (m >= per) return -1;
    const int32_t g = l * per + m;
    if (g >= total) return 0;
    // the pair lo with pref[lo] <= g < pref[lo + 1] (it has at least one block): usually the
    // tabled pair itself, else a few steps further
    const int4 c = lsm_ld(tp.coarse, g / PLAN_COARSE);
    int lo = c.x;
    int32_t p0 = c.y, p1 = c.z, b0 = c.w;
    if (p1 <= g) {
        do {
            ++lo;
            p0 = p1;
            p1 = lsm_ld(tp.pref, lo + 1);
        } while (p1 <= g);
        b0 = st[lo].blk0;
    }
    const int32_t blk = g - p0;
    task.pair = lo;
    task.start = blk * NN_THREADS;
    task.slot = b0 + blk;
    task.pad = 0;
    return 1;
}

// ------------------------------------------------------------------------------------------
// correspondence search (the hot kernel)
// ------------------------------------------------------------------------------------------
// One workgroup per block of 256 source points of an active pair (XCD-balanced work plan).
// Passes >= 1 first run the stability check on every point (two loads per query: the source
// point and its previous neighbour); the queries it cannot certify are compacted in LDS and
// box-searched by the leading lanes, so whole waves of certified queries retire at once. Pass 0
// (and every pass with LSM_NN_NOCERT=1) box-searches every point. Queries the box search cannot
// resolve go to nn_fallback. Every path computes the same (d2, index) minimum with the same f32
// arithmetic, so the result does not depend on which path resolved a query.
//
// Box search: the cells within the warm-start radius R = sqrt(previous neighbour's distance)
// (at most NN_KMAX cells each way), or the 9x9x9 cells around the query's cell on a cold start.
// Rows of cells are visited centre-out and pruned by their slab distance against the pruning
// radius (prune2: it yields rho); inside a row the x-sorted runs are walked from the query's x.
// A query is resolved when its best distance is provably below every unsearched point (the box
// faces not clipped by the grid), else queued for the fallback.
constexpr int NN_KMAX = 4;
// cold start (no previous neighbour: pass 0): 9x9x9 cells. nn + fallback ms per step, C3 / C4
// (LSM_NN_KCOLD): 1: 102.9 / 106.1; 2: 92.8 / 64.8; 3: 93.1 / 52.1; 4: 93.2 / 47.2; 5 (with
// NN_KMAX 5): 95.3 / 47.4 -- a wider first box settles the revisit pairs' far queries (large
// initial errors) without the fallback
constexpr int NN_KCOLD = 4;
// In pairs with >= NN_DIRECT_ITER updates, warm starts at least NN_DIRECT_RC cells away skip the
// box search (nn_query). nn + fallback ms per step, C3 (1999 sequence pairs) / C4 (512 revisit
// pairs): off 100.4 / 64.7; 3 cells from update 0: 92.5 / 93.6; from 4: 92.9 / 71.5; from 12:
// 93.5 / 66.8; from 20: 94.8 / 66.1; 4 cells from 12: 97.2 / 64.4
constexpr double NN_DIRECT_RC = 3.0;
constexpr int NN_DIRECT_ITER = 12;

// Returns true when resolved (result / rho set), false when the fallback must finish it (t2
// holds what the box search found).
// (nearest, second) reduction over the L lanes of a query group (L a power of two, the group
// aligned inside the wave); lanes holding the same point merge their second distances.
// `lim` becomes a valid pruning bound of the whole group: every point some lane skipped is at
// least that lane's lim away, every examined non-best point at least the merged second.
// (The only point two lanes can both hold is the warm start; a duplicate third distance only
// lowers rho, which stays a valid bound.)
__device__ __forceinline__ void group_top3(Top3 &t, int L) {
    float lim = t.lim;
    for (int off = L >> 1; off > 0; off >>= 1) {
        const float od = __shfl_xor(t.bd2, off, LSM_WAVE);
        const int oi = __shfl_xor(t.bidx, off, LSM_WAVE);
        const float os = __shfl_xor(t.sd2, off, LSM_WAVE);
        const int osi = __shfl_xor(t.sidx, off, LSM_WAVE);
        const float ot = __shfl_xor(t.td2, off, LSM_WAVE);
        lim = fminf(lim, __shfl_xor(lim, off, LSM_WAVE));
        if (oi >= 0) top_add(od, oi, t);
        if (osi >= 0) top_add(os, osi, t);
        t.td2 = fminf(t.td2, ot);
    }
    t.lim = fminf(prune2(t.bd2, t.td2, t.m), lim);
}

// Box search of one query by a group of L lanes (sub = this lane's index in the group): the
// rows of the box are dealt round-robin over the group in centre-out order, each lane keeps
// its own (nearest, second) and pruning radius, and the group merges them at the end. L = 1
// is the plain per-lane search; a workgroup with few uncertified queries splits each over
// several lanes, so a long search chain (a far or ambiguous query of a pair that keeps
// iterating) is not left to one lane. Every lane of the group returns the same values.
// GBUF: read the target through a buffer descriptor (G must then be wave-uniform), else through
// 64-bit global addresses (the box-queue kernel, whose waves may hold queries of several pairs)
template <bool GBUF = bool(LSM_NN_BUF)>
__device__ __forceinline__ bool nn_query(const double *T, const CloudDev &S, const CloudDev &G,
                                         int i, int prev, float m, const NNParams &prm,
                                         int &result, int &alt, float &rho, Top3 &t2, float4 &qp,
                                         int sub = 0, int L = 1, NNStat *ns = nullptr,
                                         bool direct_ok = false) {
    NN_ST(ns, 0, 1);
    double qx64, qy64, qz64;
    transform_point(T, lsm_ld(S.xyz, i), qx64, qy64, qz64);
    const float qx = float(qx64), qy = float(qy64), qz = float(qz64);
    qp = make_float4(qx, qy, qz, 0.f);
    t2 = top3_init(-1, INFINITY, m);
    result = -1;
    alt = -1;
    rho = INFINITY;
    if (G.n <= 0) return true;
    // warm start: the previous pass's nearest neighbour bounds this pass's search. The search
    // stays exact -- the (d2, index) minimum over all points does not depend on the start.
    if (prev >= 0 && prev < G.n) t2 = top3_init(prev, sqd(lsm_ld(G.xyz, prev), qx, qy, qz), m);
    const float fx = (qx - G.ox) * G.inv_cell, fy = (qy - G.oy) * G.inv_cell_y,
                fz = (qz - G.oz) * G.inv_cell;
    // a query outside the target's box searches around the nearest cell of the box: the
    // box faces that lie on the grid boundary bound nothing (no points beyond them)
    auto clampc = [](float f, int n) { return (int)fminf(fmaxf(floorf(f), 0.f), float(n - 1)); };
    const int cx = clampc(fx, G.nx), cy = clampc(fy, G.ny), cz = clampc(fz, G.nz);
    // box half-width in cells: the warm-start radius (+ f32 slack), else NN_KCOLD
    int K = prm.kcold;
    if (t2.bidx < 0 && prm.cold_seed) {
        // cold start: the middle point of the query's own cell (when it holds any) seeds the
        // search, so the first rows' walks and x-ranges are pruned from the start; the box stays
        // the cold one (NN_KCOLD), and the (d2, index) minimum does not depend on the seed
        const int cl = lsm_cell_lin(G.nbx, G.nby, cx, cy, cz);
        const uint32_t a = lsm_ld(G.cell_start, cl), b = lsm_ld(G.cell_start, cl + 1);
        if (b > a) {
            const int k = int((a + b) >> 1);
            t2 = top3_init(k, sqd(lsm_ld(G.xyz, k), qx, qy, qz), m);
        }
    } else if (t2.bd2 < INFINITY) {
        const float rc = sqrtf(t2.bd2) * G.inv_cell * 1.0001f + 1e-4f;
        // In a pair that keeps iterating (direct_ok: >= NN_DIRECT_ITER updates, the chaotic
        // tail), a query whose previous neighbour lies >= NN_DIRECT_RC cells away needs a wide
        // box, which settles it only when a point turns up within the box's face distance; there
        // such queries (no target surface near them) mostly fail it after walking ~40 rows. They
        // go straight to the fallback with the warm start as their best, which finds the same
        // (d2, index) minimum with 32 lanes over 1.5 m blocks. Early passes keep the box search:
        // after a large first correction (revisit pairs) the surface is often near again, and
        // the fallback, starting from the stale warm start, costs more than the box.
        if (direct_ok && rc >= prm.direct_rc) {
            NN_ST(ns, 7, sub == 0 ? 1 : 0);
            return false;
        }
        K = rc >= float(prm.kmax) ? prm.kmax : max(1, (int)ceilf(rc));
    } else {
        NN_ST(ns, 6, 1);
    }
    NN_ST(ns, 5, K);
    // K cells of `cell` in x and z; in y the same extent in the finer y cells (LSM_YSUB)
    const int Ky = K * LSM_YSUB;
    const int x0 = max(cx - K, 0), x1 = min(cx + K, G.nx - 1);
    const int y0 = max(cy - Ky, 0), y1 = min(cy + Ky, G.ny - 1);
    const int z0 = max(cz - K, 0), z1 = min(cz + K, G.nz - 1);
    const float c2 = G.cell * G.cell * 0.9999f;   // slack: cells assigned by f32 floor
    const float c2y = G.cell_y * G.cell_y * 0.9999f;
    const uint32_t *cs = G.cell_start;
    typedef typename std::conditional<GBUF, BufPts, GlobalPts>::type Rd;
    const Rd gp = [&]() {
        if constexpr (GBUF) return cloud_buf_pts(G);
        else return GlobalPts{G.xyz};
    }();
    const int W = 2 * K + 1, Wy = 2 * Ky + 1;
    // Rows are visited centre-out (offsets 0, -1, 1, -2, 2, ...: |offset| never decreases) and
    // a row at offset d in z (or y) is at least (|d| - 1) cells from the query's slab. Once that
    // bound reaches the pruning radius (which only shrinks) every later row of the loop would
    // be skipped as well, so the loop stops there: the same rows are walked, without iterating
    // over the pruned rest of a 9 x 9 cold box.
#pragma unroll 1
    for (int iz = 0; iz < W; ++iz) {
        const int adz = (iz + 1) >> 1;
        if (adz >= 2 && float((adz - 1) * (adz - 1)) * c2 >= t2.lim) break;
        const int dz = (iz & 1) ? -adz : adz;   // 0, -1, 1, -2, 2 ...
        const int z = cz + dz;
        if (z < z0 || z > z1) continue;
        const float wz = slab_cells2(fz, z) * c2;
        if (wz >= t2.lim) continue;
#pragma unroll 1
        for (int iy = (sub - iz * Wy) & (L - 1); iy < Wy; iy += L) {   // rows t == sub (mod L)
            const int ady = (iy + 1) >> 1;
            if (ady >= 2 && wz + float((ady - 1) * (ady - 1)) * c2y >= t2.lim) break;
            const int dy = (iy & 1) ? -ady : ady;
            const int y = cy + dy;
            if (y < y0 || y > y1) continue;
            const float wyz = wz + slab_cells2(fy, y) * c2y;
            const float lim = t2.lim;
            if (wyz >= lim) continue;
            NN_ST(ns, 1, 1);
            // cells of this row that can still hold a point within the pruning radius
            int xa = x0, xb = x1;
            if (lim < INFINITY) {
                const float ch = sqrtf((lim - wyz) * 1.0002f) * G.inv_cell + 1e-4f;
                xa = max(xa, (int)floorf(fx - ch));
                xb = min(xb, (int)floorf(fx + ch));
            }
            // The row's block parts left to right. (Centre-out with the far parts pruned by
            // their x-slab -- fewer entry searches in the cold pass 0 -- measured slower: nn
            // 81.7 -> 91.3 ms per step, 88.5 with the registers capped back to 7 waves/SIMD.)
            int x = xa;
            while (x <= xb) {
                const int xe = min(xb, x | (LSM_BLKX - 1));   // end of this block's row part
                const uint32_t a = lsm_ld(cs, lsm_cell_lin(G.nbx, G.nby, x, y, z));
                const uint32_t b = lsm_ld(cs, lsm_cell_lin(G.nbx, G.nby, xe, y, z) + 1);
                if (b > a) scan_run(gp, a, b, qx, qy, qz, wyz, t2, prm.lin, ns);
                x = xe + 1;
            }
        }
    }
    // every point outside the searched box is at least `bound` away; sides clipped by the grid
    // hold no points.
    const float bx = fminf(cx - K > 0 ? fx - float(cx - K) : INFINITY,
                           cx + K + 1 < G.nx ? float(cx + K + 1) - fx : INFINITY);
    const float by = fminf(cy - Ky > 0 ? fy - float(cy - Ky) : INFINITY,
                           cy + Ky + 1 < G.ny ? float(cy + Ky + 1) - fy : INFINITY);
    const float bz = fminf(cz - K > 0 ? fz - float(cz - K) : INFINITY,
                           cz + K + 1 < G.nz ? float(cz + K + 1) - fz : INFINITY);
    const float bound = fminf(fminf(bx, bz) * G.cell, by * G.cell_y);
    const float bound2 = bound * bound * 0.99999f;
    if (L > 1) group_top3(t2, L);
    if (!(t2.bd2 <= bound2 || bound >= prm.maxc)) NN_ST(ns, 7, sub == 0 ? 1 : 0);
    if (t2.bd2 <= bound2 || bound >= prm.maxc) {
        if (t2.bidx >= 0 && t2.bd2 < prm.maxc2) {
            result = t2.bidx;
            alt = t2.sidx;
            rho = rho_from(t2.lim, bound);
        } else {
            result = -1;
            rho = rho_from(t2.bd2, bound);
        }
        return true;
    }
    return false;
}

// wave-aggregated append of the lanes with `pending` to the fallback queue
__device__ __forceinline__ void push_fallback(bool pending, int pair, int i, float m,
                                              const Top3 &t2,
                                              FallbackItem *__restrict__ queue,
                                              uint32_t *__restrict__ queue_n, uint32_t queue_cap) {
    const uint64_t bm = __ballot(pending);
    if (!bm) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)bm) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(queue_n, (uint32_t)__popcll(bm));
    base = __shfl(base, leader, LSM_WAVE);
    if (pending) {
        const uint32_t slot = base + __popcll(bm & ((uint64_t(1) << lane) - 1));
        if (slot < queue_cap) queue[slot] = {pair, i, t2.bidx, t2.bd2, t2.sd2, m};
    }
}

// Stability check of one query (passes >= 1). corr[g] is the nearest neighbour the query's last
// search found; rec[g] = (alt | spass << REC_SHIFT, rho) is that search's second point (REC_NONE:
// none), the pass spass it ran in, and its rho (a lower bound on |q_s - t'| for every target
// point t' other than corr[g] and alt; for every point when corr[g] = -1). q_s, the search's f32
// query point, is not stored: it is recomputed from the pair's transform history (hist[spass],
// written by the solve kernel) with transform_point's fixed rounding, so it is the search's point
// bit for bit. For this pass's query point q, every such point is at least rho - D away,
// D = |q - q_s| (triangle inequality, f64 of the f32 points, rounded up). The winner w of
// corr[g] and alt in the exact f32 (d2, index) order is certified when |q - w| (1 + 1e-5) + D
// < rho, i.e. every other point is strictly farther even after the f32 rounding of the search's
// squared distances (relative error < 1e-6); only a swap (alt won) is written, and the record
// keeps the search's pass (so q_s stays the search's point). D is the direct displacement since
// the search, not a sum of per-pass steps, so a pair that oscillates keeps its certificates. A
// query without a neighbour stays without one while rho - D >= max_corr (1 + 1e-5); one whose
// neighbour left max_corr drops it and is re-based at q. Returns false when the query must be
// searched; `m` is then its margin for the search's rho.
__device__ __forceinline__ float motion_margin(const PairState &P, const float4 s,
                                               const NNParams &prm);

__device__ __forceinline__ bool check_query(const PairState &P, const CloudDev &S,
                                           const CloudDev &G, int i, int64_t g,
                                           const NNParams &prm, int32_t *__restrict__ corr,
                                           int2 *__restrict__ rec, const double *hist, int pass,
                                           float &m) {
    const float4 s = lsm_ld(S.xyz, i);
    double x, y, z;
    transform_point(P.T, s, x, y, z);
    const float qx = float(x), qy = float(y), qz = float(z);
    const int2 rc = lsm_ld(rec, g);
    const int spass = int(uint32_t(rc.x) >> REC_SHIFT);
    double xs, ys, zs;   // q_s: the search's query point, from the transform of its pass
    transform_point(hist + size_t(spass) * HIST_STRIDE, s, xs, ys, zs);
    const double ddx = double(qx) - double(float(xs)), ddy = double(qy) - double(float(ys)),
                 ddz = double(qz) - double(float(zs));
    const double delta = sqrt(ddx * ddx + ddy * ddy + ddz * ddz) * (1.0 + 1e-6) + 1e-7;
    const int prev = corr[g];
    const double r = double(__int_as_float(rc.y));
    if (prev >= 0) {
        const uint32_t araw = uint32_t(rc.x) & REC_NONE;
        const int sec = araw == REC_NONE ? -1 : int(araw);
        float4 t = lsm_ld(G.xyz, prev);
        float dt = sqd(t, qx, qy, qz);
        bool swap = false;
        if (sec >= 0) {
            const float4 u = lsm_ld(G.xyz, sec);
            const float du = sqd(u, qx, qy, qz);
            if (better(du, sec, dt, prev)) {
                swap = true;
                t = u;
                dt = du;
            }
        }
        const double ex = double(qx) - double(t.x), ey = double(qy) - double(t.y),
                     ez = double(qz) - double(t.z);
        const double e = sqrt(ex * ex + ey * ey + ez * ez);
        if (e * (1.0 + 1e-5) + delta < r) {
            if (dt >= prm.maxc2) {
                // the neighbour left max_corr: no point is within it, none nearer than e
                corr[g] = -1;
                rec[g] = rec_pack(-1, pass, __double2float_rd(fmin(e * (1.0 - 1e-5), r - delta)));
            } else if (swap) {
                corr[g] = sec;
                rec[g] = make_int2(int(uint32_t(prev) | (uint32_t(spass) << REC_SHIFT)), rc.y);
            }
            return true;
        }
    } else if (prev == -1 && r - delta >= double(prm.maxc) * (1.0 + 1e-5)) {
        return true;
    }
    m = motion_margin(P, s, prm);
    return false;
}

// rho margin of a search in a pass that moved the query by dq (the same value check_query gives)
__device__ __forceinline__ float motion_margin(const PairState &P, const float4 s,
                                               const NNParams &prm) {
    double x, y, z, xp, yp, zp;
    transform_point(P.T, s, x, y, z);
    transform_point(P.Tp, s, xp, yp, zp);
    const double ddx = double(float(x)) - double(float(xp)), ddy = double(float(y)) - double(float(yp)),
                 ddz = double(float(z)) - double(float(zp));
    const double dq = sqrt(ddx * ddx + ddy * ddy + ddz * ddz);
    return float(prm.m_mul * dq + prm.m_add);
}

// per-wave sums of the lanes' statistics into stats[pass * NN_NSTAT + c]
__device__ __forceinline__ void flush_stats(const NNStat &ls, unsigned long long *stats) {
    for (int c = 0; c < NN_NSTAT; ++c) {
        uint32_t v = ls.v[c];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, LSM_WAVE);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(stats + c, (unsigned long long)v);
    }
}

// LSM_NN_WPE=<w>: cap the correspondence kernel's registers for w waves per SIMD. 8 (64 VGPRs,
// 2-4 registers spilled outside the walks) since the walks read the target through a buffer
// descriptor: nn 81.7 -> 73.9 ms per step (7 waves: 76.1; round 2, with 64-bit addresses, the
// same cap spilled in the walks and lost).
#ifndef LSM_NN_WPE
#define LSM_NN_WPE 8
#endif
// LSM_NN_WPE0: the same request for the passes without the stability check (0, 1)
#ifndef LSM_NN_WPE0
#define LSM_NN_WPE0 LSM_NN_WPE
#endif
#if LSM_NN_WPE > 0 && LSM_NN_WPE0 > 0
#define LSM_NN_ATTR __attribute__((amdgpu_waves_per_eu(CHECK ? LSM_NN_WPE : LSM_NN_WPE0)))
#else
#define LSM_NN_ATTR
#endif
template <bool CHECK, bool STATS = false>
__global__ void __launch_bounds__(NN_THREADS) LSM_NN_ATTR
nn_kernel(TaskPlan tp, const PairState *__restrict__ st, const CloudDev *__restrict__ cds,
          NNParams prm, int pass, const double *__restrict__ hist, int32_t *__restrict__ corr,
          int2 *__restrict__ rec, FallbackItem *__restrict__ queue,
          uint32_t *__restrict__ queue_n, uint32_t queue_cap, uint32_t *__restrict__ searched,
          unsigned long long *__restrict__ stats = nullptr,
          const uint8_t *__restrict__ tiled = nullptr) {
    // after nn_tile_kernel (same grid and plan): only the workgroups it did not tile
    if (tiled && tiled[blockIdx.x]) return;
    NNStat ls{};
    NNStat *ns = STATS ? &ls : nullptr;
    // one task per workgroup: the host sizes the grid from an earlier pass's plan, which only
    // shrinks, so waves may retire early (no barrier follows the compaction)
    BlockTask task;
    // the host sizes the grid from a plan it polled; a grid smaller than the current plan would
    // skip correspondence tasks silently, so it is flagged (the host then fails the batch)
    if (blockIdx.x == 0 && threadIdx.x == 0 && int64_t(gridDim.x) < int64_t(tp.plan[1]) * NXCD)
        atomicOr(tp.err, 1);
    if (plan_task(tp, st, blockIdx.x, task) <= 0) return;
    const PairState &P = st[task.pair];
    if (!P.active) return;
    const CloudDev S = cds[P.src];
    const CloudDev G = cds[P.tgt];
    int i = task.start + threadIdx.x;
    bool live = i < S.n;
    float m = prm.m0;
    if (CHECK) {
        __shared__ int32_t s_idx[NN_THREADS];
        __shared__ float s_m[NN_THREADS];
        __shared__ int32_t s_cnt[NN_THREADS / LSM_WAVE];
        bool need = false;
        if (live)
            need = !check_query(P, S, G, i, P.src_off + i, prm, corr, rec,
                                hist + size_t(task.pair) * prm.hmax * HIST_STRIDE, pass, m);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const uint64_t bm = __ballot(need);
        if (lane == 0) s_cnt[w] = __popcll(bm);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int q = 0; q < NN_THREADS / LSM_WAVE; ++q) {
            before += q < w ? s_cnt[q] : 0;
            total += s_cnt[q];
        }
        if (need) {
            const int slot = before + __popcll(bm & ((uint64_t(1) << lane) - 1));
            s_idx[slot] = i;
            s_m[slot] = m;
        }
        __syncthreads();
        if (threadIdx.x == 0 && total > 0) atomicAdd(searched, uint32_t(total));
        // few queries left: L lanes per query (power of two, at most split_max). The loop
        // doubles L only while the doubled groups still fit, so total * L <= NN_THREADS: every
        // uncertified query gets a group (the groups may span all four waves). Round 2's
        // "split-placement" probes broke exactly this bound -- a loop test of total * L <= 256
        // (final total * L up to 512) and a 128-lane offset of groups that may need 256 lanes
        // -- so the queries past the last lane were never searched and kept stale
        // correspondences.
        int L = 1;
        while (L < prm.split_max && total * (2 * L) <= NN_THREADS) L *= 2;
        // LSM_NN_SPLIT_PLACE (tests: the result must not depend on where the groups sit):
        // 0 groups from lane 0 in query order; 1 groups end in the last wave (first group at
        // the highest wave boundary that still fits them); 2 as 0 with the query order reversed
        const int span = total * L;
        const int base = prm.split_place == 1 ? ((NN_THREADS - span) / LSM_WAVE) * LSM_WAVE : 0;
        if ((w + 1) * LSM_WAVE <= base || w * LSM_WAVE >= base + span)
            return;   // this wave has nothing to search (no stats)
        const int rel = int(threadIdx.x) - base;
        int q = rel / L;
        live = rel >= 0 && q < total;
        if (prm.split_place == 2) q = total - 1 - q;
        if (live) {
            i = s_idx[q];
            m = s_m[q];
        }
        const int sub = rel & (L - 1);
        const int64_t g = P.src_off + i;
        int result = -1, a2 = -1;
        float r = 0.f;
        Top3 t2 = top3_init(-1, INFINITY, m);
        bool pending = false;
        float4 qp;
        if (live)
            pending = !nn_query(P.T, S, G, i, corr[g], m, prm, result, a2, r, t2, qp, sub, L, ns,
                                P.iter >= prm.direct_iter);
        const bool lead = live && sub == 0;
        push_fallback(pending && lead, task.pair, i, m, t2, queue, queue_n, queue_cap);
        if (lead) {
            corr[g] = pending ? -2 : result;
            if (!pending) rec[g] = rec_pack(a2, pass, r);
        }
        if (STATS) {
            if (sub != 0) ls.v[0] = 0;   // one search per query
            flush_stats(ls, stats);
        }
        return;
    }
    const int64_t g = P.src_off + i;
    int result = -1, a2 = -1;
    float r = 0.f;
    // a pass >= 1 searched without the check (LSM_NN_CERT_FROM): the search still leaves rho
    // with the margin of this pass's motion, for the next pass's certificate
    if (live && P.iter > 0) m = motion_margin(P, lsm_ld(S.xyz, i), prm);
    Top3 t2 = top3_init(-1, INFINITY, m);
    bool pending = false;
    float4 qp;
    if (live)
        pending = !nn_query(P.T, S, G, i, corr[g], m, prm, result, a2, r, t2, qp, 0, 1, ns,
                            P.iter >= prm.direct_iter);
    push_fallback(pending, task.pair, i, m, t2, queue, queue_n, queue_cap);
    if (live) {
        corr[g] = pending ? -2 : result;
        if (!pending) rec[g] = rec_pack(a2, pass, r);
    }
    if (STATS) flush_stats(ls, stats);
}

// The passes that search every query (nn_kernel<false>'s work) with LQ lanes per query: the rows
// of each query's box are dealt round-robin over its LQ lanes (nn_query's split search, merged by
// group_top3), so a long search chain is shared; LQ * 256 threads per workgroup, one 256-query
// block each. Exact like every split search (test_search_path_variants_bit_identical).
template <int LQ>
__global__ void __launch_bounds__(NN_THREADS * LQ) __attribute__((amdgpu_waves_per_eu(LSM_NN_WPE0)))
nn_full_kernel(TaskPlan tp, const PairState *__restrict__ st, const CloudDev *__restrict__ cds,
               NNParams prm, int pass, int32_t *__restrict__ corr, int2 *__restrict__ rec,
               FallbackItem *__restrict__ queue, uint32_t *__restrict__ queue_n,
               uint32_t queue_cap) {
    BlockTask task;
    if (blockIdx.x == 0 && threadIdx.x == 0 && int64_t(gridDim.x) < int64_t(tp.plan[1]) * NXCD)
        atomicOr(tp.err, 1);
    if (plan_task(tp, st, blockIdx.x, task) <= 0) return;
    const PairState &P = st[task.pair];
    if (!P.active) return;
    const CloudDev S = cds[P.src];
    const CloudDev G = cds[P.tgt];
    const int sub = int(threadIdx.x) & (LQ - 1);
    const int i = task.start + int(threadIdx.x) / LQ;
    const bool live = i < S.n;
    const int64_t g = P.src_off + i;
    float m = prm.m0;
    if (live && P.iter > 0) m = motion_margin(P, lsm_ld(S.xyz, i), prm);
    int result = -1, a2 = -1;
    float r = 0.f;
    Top3 t2 = top3_init(-1, INFINITY, m);
    bool pending = false;
    float4 qp;
    if (live)
        pending = !nn_query(P.T, S, G, i, corr[g], m, prm, result, a2, r, t2, qp, sub, LQ,
                            nullptr, P.iter >= prm.direct_iter);
    const bool lead = live && sub == 0;
    push_fallback(pending && lead, task.pair, i, m, t2, queue, queue_n, queue_cap);
    if (lead) {
        corr[g] = pending ? -2 : result;
        if (!pending) rec[g] = rec_pack(a2, pass, r);
    }
}

// ------------------------------------------------------------------------------------------
// LDS-staged tile search (the passes that search every query: 0 and 1)
// ------------------------------------------------------------------------------------------
// A workgroup's 256 queries are consecutive points of the cell-sorted source, so they occupy a
// few cells. The workgroup stages every target point of the cells within NN_TMARGIN cells of its
// queries' cells into LDS -- one x-sorted run per (y, z) row of the box: a row's block parts
// follow each other in x, and their global indices increase with x, so the row is one run in
// (x, index) order -- and every lane then runs the box search of nn_query against the tile:
// rows centre-out in z and y, pruned by their slab distance, an entry search and two walks per
// row, all in LDS. Each staged point carries its global index (w bits), so the (d2, index) order
// and every result are the global path's. A query is resolved when its best distance is below
// the distance to every face of the staged box that is not the grid's boundary (the points
// outside are farther); the rest continue with nn_query (warm-started from the tile's best) and
// the fallback, so the results are bit-identical to nn_kernel<false> (test_search_path_variants).
// A workgroup whose box holds more than NN_TCAP points (or rows / block parts than the tables
// hold) searches as nn_kernel<false> does. CPU model of the tile sizes: tools/nn_tile_model.py.
// Off by default (LSM_NN_TILE=1 selects it): exact, but slower than the global path.
#ifndef LSM_NN_TCAP
#define LSM_NN_TCAP 4096
#endif
constexpr int NN_TCAP = LSM_NN_TCAP;   // staged points (16 B each)
constexpr int NN_TPARTS = 384;         // staged block parts (a row spans one part per 4 cells)
constexpr int NN_TMARGIN = 1;          // cells staged around the queries' cells

// one x-sorted LDS run [a, b) of a row at slab distance dyz2 (squared): entry search at qx, then
// rightwards and leftwards while dx^2 + dyz2 <= the pruning radius (nn_query's scan_run on LDS;
// each walk reads its next point before testing the current one)
__device__ __forceinline__ void tile_run(const float4 *T, uint32_t a, uint32_t b, float qx,
                                         float qy, float qz, float dyz2, float cap2, Top3 &t2) {
    uint32_t lo = a, hi = b;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T[mid].x < qx) lo = mid + 1;
        else hi = mid;
    }
    if (lo < b) {
        float4 nx = T[lo];
        for (uint32_t k = lo; k < b; ++k) {
            const float4 t = nx;
            if (k + 1 < b) nx = T[k + 1];
            const float dx = t.x - qx;
            if (dx * dx + dyz2 > fminf(t2.lim, cap2)) break;
            top_add(sqd(t, qx, qy, qz), __float_as_int(t.w), t2);
        }
    }
    if (lo > a) {
        float4 nx = T[lo - 1];
        for (int k = int(lo) - 1; k >= int(a); --k) {
            const float4 t = nx;
            if (k > int(a)) nx = T[k - 1];
            const float dx = qx - t.x;
            if (dx * dx + dyz2 > fminf(t2.lim, cap2)) break;
            top_add(sqd(t, qx, qy, qz), __float_as_int(t.w), t2);
        }
    }
}

// workgroup minima of six ints (one barrier pair)
__device__ __forceinline__ void wg_min6(int (&v)[6], int (*red)[NN_THREADS / LSM_WAVE]) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[c] = min(v[c], __shfl_xor(v[c], off, LSM_WAVE));
        if ((threadIdx.x & 63) == 0) red[c][threadIdx.x >> 6] = v[c];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        v[c] = red[c][0];
#pragma unroll
        for (int q = 1; q < NN_THREADS / LSM_WAVE; ++q) v[c] = min(v[c], red[c][q]);
    }
}

__global__ void __launch_bounds__(NN_THREADS)
nn_tile_kernel(TaskPlan tp, const PairState *__restrict__ st, const CloudDev *__restrict__ cds,
               NNParams prm, int pass, int32_t *__restrict__ corr, int2 *__restrict__ rec,
               FallbackItem *__restrict__ box, uint32_t *__restrict__ box_n, uint32_t box_cap,
               uint8_t *__restrict__ tiled_out) {
    __shared__ float4 tile[NN_TCAP];
    __shared__ uint32_t p_a[NN_TPARTS];        // a block part's first global index
    __shared__ uint32_t p_off[NN_TPARTS + 1];  // its first tile slot (exclusive scan)
    __shared__ int red[6][NN_THREADS / LSM_WAVE];
    BlockTask task;
    if (blockIdx.x == 0 && threadIdx.x == 0 && int64_t(gridDim.x) < int64_t(tp.plan[1]) * NXCD)
        atomicOr(tp.err, 1);
    if (plan_task(tp, st, blockIdx.x, task) <= 0) {   // uniform per workgroup
        if (threadIdx.x == 0) tiled_out[blockIdx.x] = 1;   // nothing for nn_kernel either
        return;
    }
    const PairState &P = st[task.pair];
    if (!P.active) {
        if (threadIdx.x == 0) tiled_out[blockIdx.x] = 1;
        return;
    }
    const CloudDev S = cds[P.src];
    const CloudDev G = cds[P.tgt];
    const int i = task.start + threadIdx.x;
    const bool live = i < S.n;
    const int64_t g = P.src_off + i;
    float m = prm.m0;
    if (live && P.iter > 0) m = motion_margin(P, lsm_ld(S.xyz, i), prm);
    // the query point and its cell (clamped to the grid, as nn_query)
    float qx = 0.f, qy = 0.f, qz = 0.f;
    int cx = 0, cy = 0, cz = 0;
    if (live) {
        double x, y, z;
        transform_point(P.T, lsm_ld(S.xyz, i), x, y, z);
        qx = float(x);
        qy = float(y);
        qz = float(z);
    }
    const float fx = (qx - G.ox) * G.inv_cell, fy = (qy - G.oy) * G.inv_cell_y,
                fz = (qz - G.oz) * G.inv_cell;
    auto clampc = [](float f, int n) { return (int)fminf(fmaxf(floorf(f), 0.f), float(n - 1)); };
    if (live && G.n > 0) {
        cx = clampc(fx, G.nx);
        cy = clampc(fy, G.ny);
        cz = clampc(fz, G.nz);
    }
    const bool lq = live && G.n > 0;
    // the staged box: the queries' cells +- NN_TMARGIN, clipped to the grid
    int ext[6] = {lq ? cx : INT_MAX, lq ? -cx : INT_MAX, lq ? cy : INT_MAX,
                  lq ? -cy : INT_MAX, lq ? cz : INT_MAX, lq ? -cz : INT_MAX};
    wg_min6(ext, red);
    const int x0 = max(ext[0] - NN_TMARGIN, 0), x1 = min(-ext[1] + NN_TMARGIN, G.nx - 1);
    const int y0 = max(ext[2] - NN_TMARGIN * LSM_YSUB, 0),
              y1 = min(-ext[3] + NN_TMARGIN * LSM_YSUB, G.ny - 1);
    const int z0 = max(ext[4] - NN_TMARGIN, 0), z1 = min(-ext[5] + NN_TMARGIN, G.nz - 1);
    const bool boxed = G.n > 0 && x0 <= x1 && y0 <= y1 && z0 <= z1;   // some query is live
    const int nyb = boxed ? y1 - y0 + 1 : 0, nzb = boxed ? z1 - z0 + 1 : 0;
    const int np = boxed ? (x1 >> LSM_BLKX_SHIFT) - (x0 >> LSM_BLKX_SHIFT) + 1 : 0;  // per row
    const int64_t nparts64 = int64_t(nyb) * nzb * np;
    bool tiled = boxed && nparts64 <= NN_TPARTS;
    if (!tiled) {   // no query, or too many rows: nn_kernel searches this workgroup
        if (threadIdx.x == 0) tiled_out[blockIdx.x] = boxed ? 0 : 1;
        return;
    }
    if (threadIdx.x == 0) tiled_out[blockIdx.x] = 1;
    int nparts = int(nparts64);
    if (tiled) {
        // part bounds; each thread holds the lengths of two consecutive parts for the scan
        uint32_t len[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int t = 2 * int(threadIdx.x) + h;
            len[h] = 0;
            if (t < nparts) {
                const int r = t / np, j = t - r * np;
                const int y = y0 + r % nyb, z = z0 + r / nyb;
                const int xa = max(x0, ((x0 >> LSM_BLKX_SHIFT) + j) << LSM_BLKX_SHIFT);
                const int xb = min(x1, xa | (LSM_BLKX - 1));
                const uint32_t a = lsm_ld(G.cell_start, lsm_cell_lin(G.nbx, G.nby, xa, y, z));
                const uint32_t b = lsm_ld(G.cell_start, lsm_cell_lin(G.nbx, G.nby, xb, y, z) + 1);
                p_a[t] = a;
                len[h] = b - a;
            }
        }
        // exclusive scan of the part lengths (2 per thread, in part order)
        const uint32_t pair_sum = len[0] + len[1];
        uint32_t x = pair_sum;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int off = 1; off < LSM_WAVE; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, LSM_WAVE);
            if (lane >= off) x += y;
        }
        __shared__ uint32_t wsum[NN_THREADS / LSM_WAVE];
        if (lane == LSM_WAVE - 1) wsum[w] = x;
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int q = 0; q < NN_THREADS / LSM_WAVE; ++q) {
            before += q < w ? wsum[q] : 0;
            total += wsum[q];
        }
        const uint32_t ex = before + x - pair_sum;
        if (2 * int(threadIdx.x) < nparts) p_off[2 * threadIdx.x] = ex;
        if (2 * int(threadIdx.x) + 1 < nparts) p_off[2 * threadIdx.x + 1] = ex + len[0];
        if (threadIdx.x == 0) p_off[nparts] = total;
        tiled = total <= uint32_t(NN_TCAP);
        __syncthreads();
        if (!tiled) {   // too many points: nn_kernel searches this workgroup from global memory
            if (threadIdx.x == 0) tiled_out[blockIdx.x] = 0;
            return;
        }
        {
            // copy: slot s -> its part (binary search over p_off) -> global index; four slots
            // per round, their loads issued together
            for (uint32_t s0 = threadIdx.x; s0 < total; s0 += 4 * NN_THREADS) {
                uint32_t k[4];
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t s = s0 + uint32_t(u) * NN_THREADS;
                    k[u] = 0xffffffffu;
                    if (s < total) {
                        int lo = 0, hi = nparts;   // the last part with p_off <= s
                        while (hi - lo > 1) {
                            const int mid = (lo + hi) >> 1;
                            if (p_off[mid] <= s) lo = mid;
                            else hi = mid;
                        }
                        k[u] = p_a[lo] + (s - p_off[lo]);
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k[u] != 0xffffffffu) v[u] = lsm_ld(G.xyz, k[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k[u] != 0xffffffffu)
                        tile[s0 + uint32_t(u) * NN_THREADS] =
                            make_float4(v[u].x, v[u].y, v[u].z, __int_as_float(int(k[u])));
            }
        }
        __syncthreads();
    }
    int result = -1, a2 = -1, warm = -1;
    float r = 0.f;
    Top3 t2 = top3_init(-1, INFINITY, m);
    bool boxq = false;
    if (live && tiled) {
        const int prev = corr[g];
        if (prev >= 0 && prev < G.n) t2 = top3_init(prev, sqd(lsm_ld(G.xyz, prev), qx, qy, qz), m);
        // every unstaged point is at least `bound` away (faces on the grid boundary bound
        // nothing): the search only needs the points within it (a query with none there goes to
        // the box queue), so its rows and walks are pruned at that radius as well
        const float bx = fminf(x0 > 0 ? fx - float(x0) : INFINITY,
                               x1 + 1 < G.nx ? float(x1 + 1) - fx : INFINITY);
        const float by = fminf(y0 > 0 ? fy - float(y0) : INFINITY,
                               y1 + 1 < G.ny ? float(y1 + 1) - fy : INFINITY);
        const float bz = fminf(z0 > 0 ? fz - float(z0) : INFINITY,
                               z1 + 1 < G.nz ? float(z1 + 1) - fz : INFINITY);
        const float bound = fminf(fminf(bx, bz) * G.cell, by * G.cell_y);
        const float bound2 = bound * bound * 0.99999f;
        const float cap2 = bound * bound * 1.0001f + 1e-6f;   // >= bound2 (f32 slack)
        const float c2 = G.cell * G.cell * 0.9999f;   // slack: cells assigned by f32 floor
        const float c2y = G.cell_y * G.cell_y * 0.9999f;
        const int mz = max(cz - z0, z1 - cz), my = max(cy - y0, y1 - cy);
#pragma unroll 1
        for (int iz = 0; iz <= 2 * mz; ++iz) {
            const int adz = (iz + 1) >> 1;
            if (adz >= 2 && float((adz - 1) * (adz - 1)) * c2 >= fminf(t2.lim, cap2)) break;
            const int z = cz + ((iz & 1) ? -adz : adz);
            if (z < z0 || z > z1) continue;
            const float wz = slab_cells2(fz, z) * c2;
            if (wz >= fminf(t2.lim, cap2)) continue;
#pragma unroll 1
            for (int iy = 0; iy <= 2 * my; ++iy) {
                const int ady = (iy + 1) >> 1;
                if (ady >= 2 && wz + float((ady - 1) * (ady - 1)) * c2y >= fminf(t2.lim, cap2))
                    break;
                const int y = cy + ((iy & 1) ? -ady : ady);
                if (y < y0 || y > y1) continue;
                const float wyz = wz + slab_cells2(fy, y) * c2y;
                if (wyz >= fminf(t2.lim, cap2)) continue;
                const int row = (z - z0) * nyb + (y - y0);
                const uint32_t a = p_off[row * np], b = p_off[(row + 1) * np];
                if (b > a) tile_run(tile, a, b, qx, qy, qz, wyz, cap2, t2);
            }
        }
        if (t2.bd2 <= bound2 || bound >= prm.maxc) {
            if (t2.bidx >= 0 && t2.bd2 < prm.maxc2) {
                result = t2.bidx;
                a2 = t2.sidx;
                r = rho_from(t2.lim, bound);
            } else {
                result = -1;
                r = rho_from(t2.bd2, bound);
            }
        } else {
            boxq = true;   // not settled inside the tile: the global box search, warm from the
            warm = t2.bidx;   // tile's best
        }
    }
    // the global box searches run in nn_box_kernel (full occupancy: this kernel holds a tile),
    // compacted into a queue, warm-started as above
    {
        const uint64_t bm = __ballot(boxq);
        if (bm) {
            const int lane = threadIdx.x & 63;
            const int leader = __ffsll((unsigned long long)bm) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(box_n, (uint32_t)__popcll(bm));
            base = __shfl(base, leader, LSM_WAVE);
            if (boxq) {
                const uint32_t slot = base + __popcll(bm & ((uint64_t(1) << lane) - 1));
                if (slot < box_cap) box[slot] = {task.pair, i, warm, 0.f, 0.f, m};
            }
        }
    }
    if (live && !boxq) {
        corr[g] = result;
        rec[g] = rec_pack(a2, pass, r);
    }
}

// The box searches the tile kernel could not settle: one lane per queued query (nn_query with the
// queued warm start; a wave takes its lanes' pairs one at a time), unresolved ones on to the
// fallback. Grid-stride over the queue (its length is on the device).
#ifndef LSM_NN_BOX_WPE
#define LSM_NN_BOX_WPE 6
#endif
__global__ void __launch_bounds__(NN_THREADS) __attribute__((amdgpu_waves_per_eu(LSM_NN_BOX_WPE)))
nn_box_kernel(const PairState *__restrict__ st, const CloudDev *__restrict__ cds, NNParams prm,
              int pass, int32_t *__restrict__ corr, int2 *__restrict__ rec,
              const FallbackItem *__restrict__ box, const uint32_t *__restrict__ box_n,
              uint32_t box_cap, FallbackItem *__restrict__ queue, uint32_t *__restrict__ queue_n,
              uint32_t queue_cap) {
    const uint32_t n = min(*box_n, box_cap);
    for (uint32_t base = blockIdx.x * NN_THREADS; base < n; base += gridDim.x * NN_THREADS) {
        const uint32_t t = base + threadIdx.x;
        const bool live = t < n;
        FallbackItem it{0, 0, -1, 0.f, 0.f, 0.f};
        if (live) it = box[t];
        int result = -1, a2 = -1;
        float r = 0.f;
        Top3 t2 = top3_init(-1, INFINITY, it.margin);
        bool pending = false;
        int64_t g = 0;
        // one pair at a time (the lanes of a wave usually hold one or two): its target is then
        // wave-uniform and read through a buffer descriptor, as in nn_kernel
        bool todo = live;
        for (uint64_t bm = __ballot(todo); bm; bm = __ballot(todo)) {
            const int lead = __ffsll((unsigned long long)bm) - 1;
            const int pr = __builtin_amdgcn_readfirstlane(__shfl(it.pair, lead, LSM_WAVE));
            if (todo && it.pair == pr) {
                const PairState &P = st[pr];
                const CloudDev S = cds[P.src];
                const CloudDev G = cds[P.tgt];
                g = P.src_off + it.i;
                float4 qp;
                pending = !nn_query(P.T, S, G, it.i, it.best, it.margin, prm, result, a2, r, t2,
                                    qp, 0, 1, nullptr, P.iter >= prm.direct_iter);
                todo = false;
            }
        }
        push_fallback(pending, it.pair, it.i, it.margin, t2, queue, queue_n, queue_cap);
        if (live) {
            corr[g] = pending ? -2 : result;
            if (!pending) rec[g] = rec_pack(a2, pass, r);
        }
    }
}

// ------------------------------------------------------------------------------------------
// exact fallback: one wave per unresolved query, expanding boxes (shells)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float gap2(float q, float lo, float hi) {
    const float d = q < lo ? lo - q : (q > hi ? q - hi : 0.f);
    return d * d;
}

// Blocks in Chebyshev ring r, and in the rings before r.
__device__ __forceinline__ int ring_size(int r) { return r == 0 ? 1 : 24 * r * r + 2; }
__device__ __forceinline__ int ring_prefix(int r) { return r == 0 ? 0 : (2 * r - 1) * (2 * r - 1) * (2 * r - 1); }
constexpr int FB_R0 = 2;   // the fallback's first shell: rings 0 .. FB_R0 (5 x 5 x 5 blocks)
// the first shell's block offsets (dx, dy, dz) centre-out, by |offset|^2: the blocks nearest the
// query are scanned first, so the pruning radius shrinks before the outer blocks are tested
__constant__ int8_t c_shell[3 * 125] = {
    0, 0, 0, 0, 0, -1, 0, -1, 0, -1, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, -1, -1, -1, 0, -1, 1, 0, -1,
    0, 1, -1, -1, -1, 0, 1, -1, 0, -1, 1, 0, 1, 1, 0, 0, -1, 1, -1, 0, 1, 1, 0, 1, 0, 1, 1, -1, -1, -1,
    1, -1, -1, -1, 1, -1, 1, 1, -1, -1, -1, 1, 1, -1, 1, -1, 1, 1, 1, 1, 1, 0, 0, -2, 0, -2, 0, -2, 0, 0,
    2, 0, 0, 0, 2, 0, 0, 0, 2, 0, -1, -2, -1, 0, -2, 1, 0, -2, 0, 1, -2, 0, -2, -1, -2, 0, -1, 2, 0, -1,
    0, 2, -1, -1, -2, 0, 1, -2, 0, -2, -1, 0, 2, -1, 0, -2, 1, 0, 2, 1, 0, -1, 2, 0, 1, 2, 0, 0, -2, 1,
    -2, 0, 1, 2, 0, 1, 0, 2, 1, 0, -1, 2, -1, 0, 2, 1, 0, 2, 0, 1, 2, -1, -1, -2, 1, -1, -2, -1, 1, -2,
    1, 1, -2, -1, -2, -1, 1, -2, -1, -2, -1, -1, 2, -1, -1, -2, 1, -1, 2, 1, -1, -1, 2, -1, 1, 2, -1, -1, -2, 1,
    1, -2, 1, -2, -1, 1, 2, -1, 1, -2, 1, 1, 2, 1, 1, -1, 2, 1, 1, 2, 1, -1, -1, 2, 1, -1, 2, -1, 1, 2,
    1, 1, 2, 0, -2, -2, -2, 0, -2, 2, 0, -2, 0, 2, -2, -2, -2, 0, 2, -2, 0, -2, 2, 0, 2, 2, 0, 0, -2, 2,
    -2, 0, 2, 2, 0, 2, 0, 2, 2, -1, -2, -2, 1, -2, -2, -2, -1, -2, 2, -1, -2, -2, 1, -2, 2, 1, -2, -1, 2, -2,
    1, 2, -2, -2, -2, -1, 2, -2, -1, -2, 2, -1, 2, 2, -1, -2, -2, 1, 2, -2, 1, -2, 2, 1, 2, 2, 1, -1, -2, 2,
    1, -2, 2, -2, -1, 2, 2, -1, 2, -2, 1, 2, 2, 1, 2, -1, 2, 2, 1, 2, 2, -2, -2, -2, 2, -2, -2, -2, 2, -2,
    2, 2, -2, -2, -2, 2, 2, -2, 2, -2, 2, 2, 2, 2, 2,
};

// Chebyshev ring r of blocks around the origin block: t in [0, 24 r^2 + 2) -> offset.
__device__ __forceinline__ void ring_offset(int r, int t, int &dx, int &dy, int &dz) {
    if (r == 0) {
        dx = dy = dz = 0;
        return;
    }
    const int n1 = 2 * r + 1, n2 = 2 * r - 1;
    if (t < 2 * n1 * n1) {                 // z = -r, z = +r faces
        const int f = t / (n1 * n1), u = t % (n1 * n1);
        dz = f ? r : -r;
        dy = u / n1 - r;
        dx = u % n1 - r;
        return;
    }
    t -= 2 * n1 * n1;
    if (t < 2 * n1 * n2) {                 // y = -r, y = +r faces without the z rims
        const int f = t / (n1 * n2), u = t % (n1 * n2);
        dy = f ? r : -r;
        dz = u / n1 - r + 1;
        dx = u % n1 - r;
        return;
    }
    t -= 2 * n1 * n2;                      // x = -r, x = +r faces without y and z rims
    const int f = t / (n2 * n2), u = t % (n2 * n2);
    dx = f ? r : -r;
    dz = u / n2 - r + 1;
    dy = u % n2 - r + 1;
}

// Exact 1-NN for the queries the box search could not resolve: a group of GL aligned lanes per
// query (64 / GL queries per wave) walks Chebyshev rings of 4x4x4-cell virtual blocks outward
// from the query's block. Lanes test GL blocks at a time against the current pruning radius
// (prune2, lower-bound pruning) and the block occupancy bits; the surviving blocks are scanned
// by the whole group (a block's 16 row ranges pruned by their own lower bounds, compacted by a
// prefix sum). Stops when every unscanned point is provably farther than the best, or than
// max_corr. The first shell (rings 0 .. FB_R0, one merge and stop test) is decoded with constant
// divisors. A first-shell survivor block holds ~14 points, so 32 lanes scan it in one step like
// 64 do; queries expected to need wide rings take a whole wave (the `far` split).
template <int GL>
__device__ __forceinline__ void group_top2(Top2 &t) {
#pragma unroll
    for (int off = GL / 2; off > 0; off >>= 1) {
        const float od = __shfl_xor(t.bd2, off, LSM_WAVE);
        const int oi = __shfl_xor(t.bidx, off, LSM_WAVE);
        const float os = __shfl_xor(t.sd2, off, LSM_WAVE);
        if (oi == t.bidx) {
            t.sd2 = fminf(t.sd2, os);
        } else if (better(od, oi, t.bd2, t.bidx)) {
            t.sd2 = fminf(os, t.bd2);
            t.bd2 = od;
            t.bidx = oi;
        } else {
            t.sd2 = fminf(t.sd2, od);
        }
    }
    t.lim = prune2(t.bd2, t.sd2, t.m);
}

// fewest fallback lanes per query: one per row range of a virtual block
constexpr int FB_GL_MIN = LSM_BLKX == 4 || LSM_VB_ROWS <= 16 ? 16 : LSM_VB_ROWS;

#ifndef LSM_FB_U
#define LSM_FB_U 4        // candidate chunks per round (4 x 32: the whole first shell)
#endif
constexpr int FB_U = LSM_FB_U;
#ifndef LSM_FB_WPE
#define LSM_FB_WPE 5      // 94 VGPRs, no spills (6: 10 spilled)
#endif
template <int GL>
__device__ __forceinline__ void
fallback_run(const PairState *__restrict__ st, const CloudDev *__restrict__ cds, const NNParams &prm,
             const FallbackItem *__restrict__ queue, uint32_t total, int32_t *__restrict__ corr,
             int2 *__restrict__ rec, int pass, unsigned long long *__restrict__ fstats, float far2,
             int far, int4 (*__restrict__ s_cand)[LSM_WAVE], float (*__restrict__ s_lbx)[LSM_WAVE]) {
    // far = 0: the items whose box-search best is within sqrt(far2) (or all when far2 = inf);
    // far = 1: the others (expected to need wider rings: more lanes per query)
    // s_cand / s_lbx: the wave's LDS candidate slots ([FB_U][64]: block id, lower bound, y, z /
    // the x part of the lower bound)
    constexpr int NG = LSM_WAVE / GL;
    const int lane = threadIdx.x, sub = lane & (GL - 1), grp = lane / GL;
    const uint64_t gmask = (GL == 64 ? ~0ull : ((1ull << GL) - 1ull)) << (grp * GL);
    // per-pass statistics (diagnostics builds only: the counters cost registers)
#ifdef LSM_DIAG
#define FB_ST(...) __VA_ARGS__
    uint32_t fs[7] = {0, 0, 0, 0, 0, 0, 0};
#else
#define FB_ST(...)
#endif
    for (uint32_t base = blockIdx.x * NG; base < total; base += gridDim.x * NG) {
        const uint32_t it = base + uint32_t(grp);
        if (it >= total) continue;   // whole groups only: the group below stays converged
        const FallbackItem q = queue[it];
        if ((q.best_d2 > far2) != (far != 0)) continue;
        FB_ST(if (sub == 0) fs[0] += 1; const uint32_t chunks0 = fs[2], blocks0 = fs[3];)
        const PairState &P = st[q.pair];
        const CloudDev S = cds[P.src];
        const CloudDev G = cds[P.tgt];
        double qx64, qy64, qz64;
        transform_point(P.T, lsm_ld(S.xyz, q.i), qx64, qy64, qz64);
        const float qx = float(qx64), qy = float(qy64), qz = float(qz64);
        Top2 t2 = top2_init(q.best, q.best_d2, q.second_d2, q.margin);
        // virtual blocks of 4 x LSM_BLKY x 4 cells (cubes of edge 4 cell): one layout block holds
        // 1 << VBS of them side by side in x; a virtual block is NR point ranges (its x-chunk of
        // each of its LSM_VB_ROWS cell rows; one range when the layout block is 4 cells wide)
        constexpr int VBS = LSM_BLKX_SHIFT - 2;
        constexpr int NR = LSM_BLKX == 4 ? 1 : LSM_VB_ROWS;
        constexpr int RL = LSM_BLKX == 4 ? LSM_BLK_CELLS : 4;   // cells per range
        static_assert(NR == 1 || GL >= NR, "a lane per range");
        constexpr bool BOTH = NR > 1 && GL < 2 * NR;   // each lane loads its range's start and end
        const int nvbx = G.nbx << VBS;
        const float B = G.cell * float(LSM_BLK);   // virtual block edge (= cell_y * LSM_BLKY)
        const float gx1 = G.ox + G.nx * G.cell, gy1 = G.oy + G.ny * G.cell_y,
                    gz1 = G.oz + G.nz * G.cell;
        const float box2 = gap2(qx, G.ox, gx1) + gap2(qy, G.oy, gy1) + gap2(qz, G.oz, gz1);
        float fbound = 0.f;
#if LSM_FB_PROBE == 1   // timing probe (diagnostics only, wrong results): item setup alone
        if (G.n > 0) {
            fbound = 0.f;
        } else
#endif
        if (G.n <= 0) {
            fbound = INFINITY;
        } else if (box2 >= prm.maxc2) {
            fbound = sqrtf(box2);
            FB_ST(if (sub == 0) fs[6] += 1;)
        } else {
            const float invB = 1.f / B;
            const int qbx = (int)floorf((qx - G.ox) * invB), qby = (int)floorf((qy - G.oy) * invB),
                      qbz = (int)floorf((qz - G.oz) * invB);
            auto outside = [](int v, int n) { return v < 0 ? -v : (v > n - 1 ? v - (n - 1) : 0); };
            const int r0 = max(outside(qbx, nvbx), max(outside(qby, G.nby), outside(qbz, G.nbz)));
            const uint32_t *cs = G.cell_start;
            const int gl0 = grp * GL, rr = NR == 1 ? 0 : (sub & (NR - 1));
            // this lane's cell-table words of a virtual block: range rr (row z rr / LSM_BLKY, y
            // rr % LSM_BLKY)'s start (sub & NR == 0) or end; both when the group has fewer than
            // 2 NR lanes
            const int roff = (NR == 1 ? 0 : (rr / LSM_BLKY) * LSM_BLKY * LSM_BLKX +
                                                (rr % LSM_BLKY) * LSM_BLKX) +
                             (BOTH ? 0 : ((sub / NR) & 1) * RL);
            auto vb_word = [&](uint32_t vid) {
                const size_t c = size_t(vid >> VBS) * LSM_BLK_CELLS +
                                 ((vid & ((1u << VBS) - 1u)) << 2) + uint32_t(roff);
                return make_uint2(lsm_ld(cs, c), BOTH ? lsm_ld(cs, c + RL) : 0u);
            };
            int ra = r0, rb = r0 == 0 ? FB_R0 : r0;
            for (;;) {
                FB_ST(if (sub == 0) fs[1] += 1;)
                const bool cube = ra == 0;   // rings 0 .. FB_R0 as one (2 FB_R0 + 1)^3 cube
                const int nitems = ring_prefix(rb + 1) - ring_prefix(ra);
                // FB_U chunks of GL candidates per round: their occupancy-bit loads are in
                // flight together; the candidates wait in LDS for the survivor scan
                for (int b0 = 0; b0 < nitems; b0 += GL * FB_U) {
                    uint64_t masks[FB_U];
                    {
                        int bid_[FB_U];
                        uint32_t bw[FB_U];
#pragma unroll
                        for (int u = 0; u < FB_U; ++u) {
                            FB_ST(if (sub == 0 && b0 + u * GL < nitems) fs[2] += 1;)
                            const int t = b0 + u * GL + sub;
                            bid_[u] = -1;
                            int by_ = 0, bz_ = 0;
                            float lb_ = INFINITY;   // lower bound of the block's squared distances
                            float lbx_ = 0.f;
                            bw[u] = 0u;
                            if (t < nitems) {
                                int dx, dy, dz;
                                if (cube) {
                                    dx = c_shell[3 * t];
                                    dy = c_shell[3 * t + 1];
                                    dz = c_shell[3 * t + 2];
                                } else {
                                    int r = ra, v = t;
                                    while (v >= ring_size(r)) v -= ring_size(r++);
                                    ring_offset(r, v, dx, dy, dz);
                                }
                                const int bx = qbx + dx, by = qby + dy, bz = qbz + dz;
                                if (bx >= 0 && bx < nvbx && by >= 0 && by < G.nby && bz >= 0 &&
                                    bz < G.nbz) {
                                    const float gx = gap2(qx, G.ox + bx * B, G.ox + (bx + 1) * B);
                                    const float lb2 =
                                        gx + gap2(qy, G.oy + by * B, G.oy + (by + 1) * B) +
                                        gap2(qz, G.oz + bz * B, G.oz + (bz + 1) * B);
                                    if (lb2 * 0.9999f < t2.lim) {
                                        bid_[u] = (bz * G.nby + by) * nvbx + bx;
                                        by_ = by;
                                        bz_ = bz;
                                        lb_ = lb2;
                                        lbx_ = gx;
                                    }
                                }
                            }
                            // empty blocks (most of a far query's rings) end at the occupancy
                            // bit, an L1 hit, without cell-table loads
                            if (bid_[u] >= 0) bw[u] = lsm_ld(G.bmask, bid_[u] >> 5);
                            s_cand[u][lane] = make_int4(bid_[u], __float_as_int(lb_), by_, bz_);
                            s_lbx[u][lane] = lbx_;
                        }
#pragma unroll
                        for (int u = 0; u < FB_U; ++u)
                            masks[u] = __ballot(bid_[u] >= 0 && ((bw[u] >> (bid_[u] & 31)) & 1u)) &
                                       gmask;
                        // the wave's own LDS writes, read back by other lanes below
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
#pragma unroll
                    for (int u = 0; u < FB_U; ++u) {
                    // survivor blocks one after another; the next block's cell-table words are
                    // loaded while the current block is scanned
#if LSM_FB_PROBE == 2   // timing probe (diagnostics only, wrong results): no survivor scans
                    uint64_t mask = 0 & masks[u];
#else
                    uint64_t mask = masks[u];
#endif
                    if (mask) {
                        int src = __ffsll((unsigned long long)mask) - 1;
                        mask &= mask - 1;
                        uint2 w = vb_word(uint32_t(s_cand[u][src].x));
                        int csrc = src;
                        for (;;) {
                            // the next survivor still within the group leader's pruning radius
                            // (it only shrinks; skipping a block beyond one lane's radius leaves
                            // the merged nearest point and rho unchanged, as the first test does)
                            const float lim0 = __shfl(t2.lim, gl0, LSM_WAVE);
                            bool more = false;   // uniform in the group
                            while (mask) {
                                src = __ffsll((unsigned long long)mask) - 1;
                                mask &= mask - 1;
                                if (__int_as_float(s_cand[u][src].y) * 0.9999f < lim0) {
                                    more = true;
                                    break;
                                }
                            }
                            uint2 wn = w;
                            if (more) wn = vb_word(uint32_t(s_cand[u][src].x));
                            // the current block's ranges, each pruned by its rows' lower bound
                            const uint32_t pa = BOTH ? w.x : __shfl(w.x, gl0 + rr, LSM_WAVE),
                                           pb = BOTH ? w.y : __shfl(w.x, gl0 + NR + rr, LSM_WAVE);
                            uint32_t n = pb - pa;
                            if (NR > 1) {
                                const int4 cc = s_cand[u][csrc];
                                const float cx = s_lbx[u][csrc];
                                const int y = cc.z * LSM_BLKY + (rr % LSM_BLKY),
                                          z = cc.w * LSM_BLK + rr / LSM_BLKY;
                                const float rlb =
                                    cx + gap2(qy, G.oy + y * G.cell_y, G.oy + (y + 1) * G.cell_y) +
                                    gap2(qz, G.oz + z * G.cell, G.oz + (z + 1) * G.cell);
                                if (!(rlb * 0.9999f < lim0)) n = 0;
                            }
                            uint32_t inc = n;   // inclusive prefix over the NR ranges
                            if (NR > 1) {
#pragma unroll
                                for (int off = 1; off < NR; off <<= 1) {
                                    const uint32_t o = __shfl_up(inc, off, NR);
                                    if (rr >= off) inc += o;
                                }
                            }
                            const uint32_t T = NR > 1 ? __shfl(inc, gl0 + NR - 1, LSM_WAVE) : n;
                            const uint32_t ex = inc - n;
                            FB_ST(if (sub == 0) {
                                fs[3] += 1;
                                fs[4] += T;
                            })
                            for (uint32_t t0 = 0; t0 < T; t0 += GL) {
                                const uint32_t tt = t0 + uint32_t(sub);
                                uint32_t k = pa + tt;
                                if (NR > 1) {   // the range holding point tt (all lanes shuffle)
                                    int lo = 0;
#pragma unroll
                                    for (int step = NR / 2; step > 0; step >>= 1)
                                        if (__shfl(inc, gl0 + lo + step - 1, LSM_WAVE) <= tt)
                                            lo += step;
                                    lo = min(lo, NR - 1);
                                    k = __shfl(pa, gl0 + lo, LSM_WAVE) +
                                        (tt - __shfl(ex, gl0 + lo, LSM_WAVE));
                                }
                                if (tt < T) top2_add(sqd(lsm_ld(G.xyz, k), qx, qy, qz), int(k), t2);
                            }
                            if (!more) break;
                            w = wn;
                            csrc = src;
                        }
                    }
                    }
                }
                group_top2<GL>(t2);
                const int r = rb;
                float bound = INFINITY;
                if (qbx - r > 0) bound = fminf(bound, qx - (G.ox + (qbx - r) * B));
                if (qbx + r + 1 < nvbx) bound = fminf(bound, G.ox + (qbx + r + 1) * B - qx);
                if (qby - r > 0) bound = fminf(bound, qy - (G.oy + (qby - r) * B));
                if (qby + r + 1 < G.nby) bound = fminf(bound, G.oy + (qby + r + 1) * B - qy);
                if (qbz - r > 0) bound = fminf(bound, qz - (G.oz + (qbz - r) * B));
                if (qbz + r + 1 < G.nbz) bound = fminf(bound, G.oz + (qbz + r + 1) * B - qz);
                if (bound == INFINITY || t2.bd2 <= bound * bound * 0.99999f ||
                    bound >= prm.maxc || rb >= 4095) {
                    fbound = bound;
                    break;
                }
                ra = rb + 1;
                rb = ra;
            }
        }
        if (sub == 0) {
            const int64_t g = P.src_off + q.i;
            const bool hit = t2.bidx >= 0 && t2.bd2 < prm.maxc2;
            FB_ST(fs[5] += hit ? 1 : 0;)
            corr[g] = hit ? t2.bidx : -1;
            rec[g] = rec_pack(-1, pass, hit ? rho_from(t2.lim, fbound) : rho_from(t2.bd2, fbound));
            FB_ST(if (fstats)   // the pass's costliest item: chunks << 32 | survivor blocks
                atomicMax(fstats + 7, ((unsigned long long)(fs[2] - chunks0) << 32) |
                                          (unsigned long long)(fs[3] - blocks0));)
        }
    }
    FB_ST(if (fstats && sub == 0) for (int c = 0; c < 7; ++c) if (fs[c])
              atomicAdd(fstats + c, (unsigned long long)fs[c]);)
#undef FB_ST
}

template <int GL>
__global__ void __launch_bounds__(LSM_WAVE) __attribute__((amdgpu_waves_per_eu(LSM_FB_WPE)))
nn_fallback_g(const PairState *__restrict__ st, const CloudDev *__restrict__ cds, NNParams prm,
              const FallbackItem *__restrict__ queue, const uint32_t *__restrict__ queue_n,
              uint32_t queue_cap, int32_t *__restrict__ corr, int2 *__restrict__ rec, int pass,
              unsigned long long *__restrict__ fstats, float far2, int far) {
    __shared__ int4 s_cand[FB_U][LSM_WAVE];
    __shared__ float s_lbx[FB_U][LSM_WAVE];
    fallback_run<GL>(st, cds, prm, queue, min(*queue_n, queue_cap), corr, rec, pass, fstats, far2,
                     far, s_cand, s_lbx);
}

// The fallback with its lanes per query chosen on the device from the pass's queue length: a
// whole wave per query for a queue of at most wide_max (the later passes, and the few but far
// queries of revisit pairs), 32 lanes for a longer one (the first passes of a sequence, where two
// queries per wave keep more of them in flight).
__global__ void __launch_bounds__(LSM_WAVE) __attribute__((amdgpu_waves_per_eu(LSM_FB_WPE)))
nn_fallback_auto(const PairState *__restrict__ st, const CloudDev *__restrict__ cds, NNParams prm,
                 const FallbackItem *__restrict__ queue, const uint32_t *__restrict__ queue_n,
                 uint32_t queue_cap, int32_t *__restrict__ corr, int2 *__restrict__ rec, int pass,
                 unsigned long long *__restrict__ fstats, uint32_t wide_max) {
    __shared__ int4 s_cand[FB_U][LSM_WAVE];
    __shared__ float s_lbx[FB_U][LSM_WAVE];
    const uint32_t total = min(*queue_n, queue_cap);
    if (total <= wide_max)
        fallback_run<64>(st, cds, prm, queue, total, corr, rec, pass, fstats, INFINITY, 0, s_cand, s_lbx);
    else
        fallback_run<32>(st, cds, prm, queue, total, corr, rec, pass, fstats, INFINITY, 0, s_cand, s_lbx);
}

// ------------------------------------------------------------------------------------------
// residual / Jacobian accumulation (deterministic block partials)
// ------------------------------------------------------------------------------------------
// Wave sums of 16 per-lane values with 16 shuffles instead of 16 x 6: at each butterfly step the
// lane pair (l, l ^ off) splits the values it still carries, each half keeping one half of the
// indices summed over both lanes. After the steps with off = 32 .. 4 and the final off = 2, 1
// sums, lane l holds the full wave sum of index l >> 2. Fixed tree: deterministic.
__device__ __forceinline__ double wave_transpose_sum16(double (&v)[16], int lane) {
#define LSM_TSTEP(OFF, H)                                                     \
    {                                                                         \
        const bool up = (lane & (OFF)) != 0;                                  \
        _Pragma("unroll") for (int k = 0; k < (H); ++k) {                     \
            const double send = up ? v[k] : v[k + (H)];                       \
            const double recv = __shfl_xor(send, (OFF), LSM_WAVE);            \
            v[k] = (up ? v[k + (H)] : v[k]) + recv;                           \
        }                                                                     \
    }
    LSM_TSTEP(32, 8)
    LSM_TSTEP(16, 4)
    LSM_TSTEP(8, 2)
    LSM_TSTEP(4, 1)
#undef LSM_TSTEP
    const double s = v[0] + __shfl_xor(v[0], 2, LSM_WAVE);
    return s + __shfl_xor(s, 1, LSM_WAVE);
}

// Accumulator k (LSM_ACC layout) of one correspondence. P2Plane: J^T J (upper triangle, row
// by row: 0-20), J^T r (21-26), r^2 (27); P2P: source (0-2) and target (3-5) sums, t s^T
// (6-14); both: squared distance (28), count (29).
template <int METHOD>
__device__ __forceinline__ double acc_value(int k, const double (&J)[6], double r,
                                            const double (&sv)[3], const double (&tv)[3],
                                            double e2) {
    if (k == 28) return e2;
    if (k == 29) return 1.0;
    if (METHOD == LSM_P2PLANE) {
        constexpr int JA[21] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 5};
        constexpr int JB[21] = {0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5, 2, 3, 4, 5, 3, 4, 5, 4, 5, 5};
        if (k < 21) return J[JA[k]] * J[JB[k]];
        if (k < 27) return J[k - 21] * r;
        return k == 27 ? r * r : 0.0;
    }
    if (k < 3) return sv[k];
    if (k < 6) return tv[k - 3];
    if (k < 15) return tv[(k - 6) / 3] * sv[(k - 6) % 3];
    return 0.0;
}

template <int METHOD>
__device__ __forceinline__ void accumulate_task(const BlockTask task,
                                                const PairState *__restrict__ st,
                                                const CloudDev *__restrict__ cds,
                                                const int32_t *__restrict__ corr,
                                                double *__restrict__ partials) {
    const PairState &P = st[task.pair];
    if (!P.active) return;
    const CloudDev S = cds[P.src];
    const CloudDev G = cds[P.tgt];
    const int i = task.start + threadIdx.x;
    // the correspondence's terms; an invalid lane contributes zeros
    double J[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, sv[3] = {0.0, 0.0, 0.0}, tv[3] = {0.0, 0.0, 0.0};
    double r = 0.0, e2 = 0.0;
    bool valid = false;
    if (i < S.n) {
        const int idx = corr[P.src_off + i];
        if (idx >= 0) {
            valid = true;
            double x, y, z;
            transform_point(P.T, lsm_ld(S.xyz, i), x, y, z);
            const float4 t = lsm_ld(G.xyz, idx);
            const double tx = t.x, ty = t.y, tz = t.z;
            const double ex = x - tx, ey = y - ty, ez = z - tz;
            e2 = (ex * ex + ey * ey) + ez * ez;
            if (METHOD == LSM_P2PLANE) {
                const float4 nf = lsm_ld(G.nrm, idx);
                const double nx = nf.x, ny = nf.y, nz = nf.z;
                r = (ex * nx + ey * ny) + ez * nz;
                J[0] = y * nz - z * ny;
                J[1] = z * nx - x * nz;
                J[2] = x * ny - y * nx;
                J[3] = nx;
                J[4] = ny;
                J[5] = nz;
            } else {
                sv[0] = x;
                sv[1] = y;
                sv[2] = z;
                tv[0] = tx;
                tv[1] = ty;
                tv[2] = tz;
            }
        }
    }
    // two halves of 16 accumulators: a transposed wave sum each (fewer live registers than one
    // of 32), per-wave sums in LDS, then the fixed-order sum over the waves
    __shared__ double red[NN_THREADS / LSM_WAVE][32];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = valid ? acc_value<METHOD>(16 * h + k, J, r, sv, tv, e2) : 0.0;
        const double sum = wave_transpose_sum16(v, lane);   // lane l: wave sum of index l >> 2
        if ((lane & 3) == 0) red[w][16 * h + (lane >> 2)] = sum;
        __builtin_amdgcn_sched_barrier(0);   // keep the halves apart (register pressure)
    }
    __syncthreads();
    if (threadIdx.x < 30) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < NN_THREADS / LSM_WAVE; ++q) s += red[q][threadIdx.x];
        partials[size_t(task.slot) * LSM_ACC + threadIdx.x] = s;
    }
}

template <int METHOD>
__global__ void __launch_bounds__(NN_THREADS)
accumulate_kernel(TaskPlan tp, const PairState *__restrict__ st, const CloudDev *__restrict__ cds,
                  const int32_t *__restrict__ corr, double *__restrict__ partials) {
    for (int t = blockIdx.x;; t += gridDim.x) {
        BlockTask task;
        const int r = plan_task(tp, st, t, task);
        if (r < 0) break;
        if (r > 0) accumulate_task<METHOD>(task, st, cds, corr, partials);
        __syncthreads();   // the task's LDS reduction buffer is reused by the next task
    }
}

// ------------------------------------------------------------------------------------------
// solve: one wave per pair
// ------------------------------------------------------------------------------------------
// Eigen::LDLT (diagonal pivoting on the not-yet-updated diagonal, left-looking) + solve with the
// pseudo-inverse of D (|D_i| <= DBL_MIN -> 0), as SolveLinearSystemPSD(JTJ, -JTr).
__device__ void ldlt_solve6(double A[6][6], double b[6], double x[6]) {
    int tr[6];
    double diag_tmp[6];
    for (int k = 0; k < 6; ++k) {
        int j = k;
        double best = fabs(A[k][k]);
        for (int q = k + 1; q < 6; ++q)
            if (fabs(A[q][q]) > best) {
                best = fabs(A[q][q]);
                j = q;
            }
        tr[k] = j;
        if (j != k) {
            for (int c = 0; c < 6; ++c) {
                double t = A[k][c];
                A[k][c] = A[j][c];
                A[j][c] = t;
            }
            for (int r = 0; r < 6; ++r) {
                double t = A[r][k];
                A[r][k] = A[r][j];
                A[r][j] = t;
            }
        }
        if (k > 0) {
            for (int c = 0; c < k; ++c) diag_tmp[c] = A[c][c] * A[k][c];
            double s = 0.0;
            for (int c = 0; c < k; ++c) s += A[k][c] * diag_tmp[c];
            A[k][k] -= s;
            for (int r = k + 1; r < 6; ++r) {
                double t = 0.0;
                for (int c = 0; c < k; ++c) t += A[r][c] * diag_tmp[c];
                A[r][k] -= t;
            }
        }
        const double akk = A[k][k];
        if (k == 0 && akk == 0.0) {
            for (int q = 0; q < 6; ++q) x[q] = 0.0;
            return;
        }
        if (akk != 0.0)
            for (int r = k + 1; r < 6; ++r) A[r][k] /= akk;
    }
    double y[6];
    for (int q = 0; q < 6; ++q) y[q] = b[q];
    for (int k = 0; k < 6; ++k) {
        double t = y[k];
        y[k] = y[tr[k]];
        y[tr[k]] = t;
    }
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < r; ++c) y[r] -= A[r][c] * y[c];
    for (int r = 0; r < 6; ++r) y[r] = fabs(A[r][r]) > 2.2250738585072014e-308 ? y[r] / A[r][r] : 0.0;
    for (int r = 5; r >= 0; --r)
        for (int c = r + 1; c < 6; ++c) y[r] -= A[c][r] * y[c];
    for (int k = 5; k >= 0; --k) {
        double t = y[k];
        y[k] = y[tr[k]];
        y[tr[k]] = t;
    }
    for (int q = 0; q < 6; ++q) x[q] = y[q];
}

// TransformVector6dToMatrix4d: R = Rz(x2) * Ry(x1) * Rx(x0), t = x3..5.
__device__ void vec6_to_mat4(const double x[6], double D[16]) {
    const double ca = cos(x[0]), sa = sin(x[0]), cb = cos(x[1]), sb = sin(x[1]), cg = cos(x[2]),
                 sg = sin(x[2]);
    D[0] = cg * cb;
    D[1] = cg * sb * sa - sg * ca;
    D[2] = cg * sb * ca + sg * sa;
    D[4] = sg * cb;
    D[5] = sg * sb * sa + cg * ca;
    D[6] = sg * sb * ca - cg * sa;
    D[8] = -sb;
    D[9] = cb * sa;
    D[10] = cb * ca;
    D[3] = x[3];
    D[7] = x[4];
    D[11] = x[5];
    D[12] = D[13] = D[14] = 0.0;
    D[15] = 1.0;
}

__global__ void __launch_bounds__(LSM_WAVE)
solve_kernel(PairState *__restrict__ st, const double *__restrict__ partials, NNParams prm,
             int pass, const double *__restrict__ pair_bytes, uint32_t *__restrict__ active_next,
             double *__restrict__ bytes_next, unsigned long long *__restrict__ src_next,
             int32_t *__restrict__ flags, double *__restrict__ hist) {
    PairState &P = st[blockIdx.x];
    if (!P.active) return;
    __shared__ double tot[32];
    const int lane = threadIdx.x;
    // lane l sums blocks l, l+64, ... for every component; then a fixed-tree wave reduction per
    // component (deterministic for a given block count)
    double part[30];
#pragma unroll
    for (int k = 0; k < 30; ++k) part[k] = 0.0;
    for (int b = lane; b < P.nblk; b += LSM_WAVE) {
        const double *src = partials + size_t(P.blk0 + b) * LSM_ACC;
#pragma unroll
        for (int k = 0; k < 30; ++k) part[k] += src[k];
    }
#pragma unroll
    for (int k = 0; k < 30; ++k) {
        const double v = lsm_wave_sum(part[k]);
        if (lane == 0) tot[k] = v;
    }
    __syncthreads();
    if (lane != 0) return;
    const double cnt = tot[29];
    const double nsrc = double(P.nsrc);
    const double fitness = cnt > 0 ? cnt / nsrc : 0.0;
    const double rmse = cnt > 0 ? sqrt(tot[28] / cnt) : 0.0;
    bool done = false;
    if (pass >= 1 && fabs(P.prev_fitness - fitness) < prm.rel_fit &&
        fabs(P.prev_rmse - rmse) < prm.rel_rmse)
        done = true;
    else if (pass >= prm.max_iter)
        done = true;
    P.fitness = fitness;
    P.rmse = rmse;
    P.ncorr = int32_t(cnt);
    if (done) {
        P.active = 0;
        flags[blockIdx.x] = 0;
        return;
    }
    double D[16];
    if (cnt <= 0) {
        for (int k = 0; k < 16; ++k) D[k] = (k % 5 == 0) ? 1.0 : 0.0;
    } else if (prm.method == LSM_P2PLANE) {
        double A[6][6], b[6], x[6];
        int k = 0;
        for (int a = 0; a < 6; ++a)
            for (int c = a; c < 6; ++c) {
                A[a][c] = tot[k];
                A[c][a] = tot[k];
                ++k;
            }
        for (int a = 0; a < 6; ++a) b[a] = -tot[21 + a];
        ldlt_solve6(A, b, x);
        vec6_to_mat4(x, D);
    } else {
        lsm::umeyama_update(tot, D);
    }
    double T[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += D[4 * r + k] * P.T[4 * k + c];
            T[4 * r + c] = s;
        }
    for (int k = 0; k < 16; ++k) {
        P.Tp[k] = P.T[k];
        P.T[k] = T[k];
    }
    if (hist) {   // null when no pass checks certificates
        double *h = hist + (size_t(blockIdx.x) * prm.hmax + pass + 1) * HIST_STRIDE;  // pass + 1's T
        for (int k = 0; k < HIST_STRIDE; ++k) h[k] = T[k];
    }
    P.iter = pass + 1;
    P.prev_fitness = fitness;
    P.prev_rmse = rmse;
    atomicAdd(active_next, 1u);
    atomicAdd(bytes_next, pair_bytes[blockIdx.x]);
    atomicAdd(src_next, (unsigned long long)P.nsrc);
}

// slot 0 of every pair's transform history: the initial transform
__global__ void hist_init_kernel(const PairState *__restrict__ st, int npairs, int hmax,
                                 double *__restrict__ hist) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npairs) return;
    for (int q = 0; q < HIST_STRIDE; ++q) hist[size_t(k) * hmax * HIST_STRIDE + q] = st[k].T[q];
}

// a pair's final correspondences as a dense array in reference order (for
// lsm_icp_last_correspondences): dense[src_perm[i]] = tgt_perm[corr[i]] or -1
__global__ void corr_to_ref(const int32_t *corr, int n, const uint32_t *src_perm,
                            const uint32_t *tgt_perm, int32_t *dense) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = corr[i];
    dense[src_perm[i]] = c >= 0 ? int32_t(tgt_perm[c]) : -1;
}

template <typename T>
int upload(lsm_ctx *ctx, const char *name, const std::vector<T> &v, T **out) {
    T *d = static_cast<T *>(ctx->buf(name, std::max<size_t>(v.size(), 1) * sizeof(T)));
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

}  // namespace

int lsm_icp_run(lsm_ctx *ctx, int64_t npairs, Cloud **src, Cloud **tgt, const double *init,
                const lsm_icp_params &p, lsm_icp_result *out) {
    hipStream_t st = ctx->stream;
    int rc;
    // unique clouds -> CloudDev table
    std::vector<Cloud *> uniq;
    std::vector<int32_t> si(npairs), ti(npairs);
    auto slot_of = [&](Cloud *c) {
        for (size_t k = 0; k < uniq.size(); ++k)
            if (uniq[k] == c) return int32_t(k);
        uniq.push_back(c);
        return int32_t(uniq.size() - 1);
    };
    if (npairs > 64) {
        // hash lookup for big batches
        std::unordered_map<Cloud *, int32_t> m;
        for (int64_t k = 0; k < npairs; ++k) {
            for (Cloud *c : {src[k], tgt[k]})
                if (!m.count(c)) {
                    m[c] = int32_t(uniq.size());
                    uniq.push_back(c);
                }
            si[k] = m[src[k]];
            ti[k] = m[tgt[k]];
        }
    } else {
        for (int64_t k = 0; k < npairs; ++k) {
            si[k] = slot_of(src[k]);
            ti[k] = slot_of(tgt[k]);
        }
    }
    std::vector<CloudDev> cdev(uniq.size());
    for (size_t k = 0; k < uniq.size(); ++k) cdev[k] = uniq[k]->dev;
    // lazy-normal targets of a P2Plane batch (LSM_NORMALS_LAZY): every pending normal of a
    // target is computed before the first pass, in one launch of full, cell-ordered workgroups,
    // so the clouds that are never a P2Plane target (the sources of loop-closure or multi-scale
    // batches) never compute theirs. (Computing, pass by pass, only the normals the
    // correspondences reach was bit-identical but slower: DESIGN.md §7.)
    if (p.method == LSM_P2PLANE) {
        std::vector<char> is_tgt(uniq.size(), 0);
        for (int64_t k = 0; k < npairs; ++k) is_tgt[size_t(ti[k])] = 1;
        std::vector<Cloud *> pending;
        for (size_t k = 0; k < uniq.size(); ++k)
            if (is_tgt[k] && uniq[k]->lazy) pending.push_back(uniq[k]);
        if (!pending.empty() && (rc = lsm_normals_complete(ctx, pending))) return rc;
    }

    // pair states; block tasks are rebuilt for the active pairs of each pass (XCD-grouped: all
    // blocks of a pair on one XCD's L2, lanes balanced by block count)
    std::vector<PairState> ps(npairs);
    std::vector<double> pbytes(npairs);
    int64_t src_off = 0;
    int32_t slot = 0;
    double bytes0 = 0.0;
    for (int64_t k = 0; k < npairs; ++k) {
        PairState &P = ps[k];
        std::memset(&P, 0, sizeof(P));
        if (init) std::memcpy(P.T, init + 16 * k, 16 * sizeof(double));
        else
            for (int q = 0; q < 16; ++q) P.T[q] = (q % 5 == 0) ? 1.0 : 0.0;
        const int nsrc = int(src[k]->n);
        P.active = 1;
        P.nsrc = nsrc;
        P.src = si[k];
        P.tgt = ti[k];
        P.src_off = src_off;
        P.blk0 = slot;
        P.nblk = (nsrc + NN_THREADS - 1) / NN_THREADS;
        slot += P.nblk;
        src_off += nsrc;
        // SURVEY.md §8d algorithmic bytes of one NN pass of this pair
        pbytes[k] = double(nsrc) * 12.0 + double(tgt[k]->n) * 12.0 +
                    double(tgt[k]->nonempty_cells) * 8.0 + double(nsrc) * 8.0;
        bytes0 += pbytes[k];
    }
    const int max_iter = p.max_iteration;
    CloudDev *d_cd;
    PairState *d_ps;
    double *d_pbytes;
    if ((rc = upload(ctx, "i_cd", cdev, &d_cd))) return rc;
    if ((rc = upload(ctx, "i_ps", ps, &d_ps))) return rc;
    if ((rc = upload(ctx, "i_pbytes", pbytes, &d_pbytes))) return rc;
    const size_t nsrc_tot = size_t(std::max<int64_t>(src_off, 1));
    int32_t *d_corr = (int32_t *)ctx->buf("i_corr", nsrc_tot * 4);
    int2 *d_rec = (int2 *)ctx->buf("i_rec", nsrc_tot * 8);
    // every pair's transform at every pass (the certificates' search points): slot 0 is the
    // initial transform, slot k + 1 the one solve k leaves. The certificate record holds the
    // search pass in 8 bits and alt in 24: beyond those bounds (or with LSM_NN_NOCERT) every pass
    // searches every query, and no history is kept.
    const int hmax = max_iter + 2;
    int64_t max_tgt = 0;
    for (int64_t k = 0; k < npairs; ++k) max_tgt = std::max<int64_t>(max_tgt, tgt[k]->n);
    const bool nocert = lsm_knob("LSM_NN_NOCERT", 0) != 0.0 || hmax > 256 ||
                        max_tgt >= int64_t(REC_NONE);
    double *d_hist = nullptr;
    if (!nocert) {
        d_hist = (double *)ctx->buf("i_hist", size_t(npairs) * hmax * HIST_STRIDE * 8);
        if (!d_hist) {
            ctx->set_error("scratch allocation failed: i_hist");
            return LSM_ENOMEM;
        }
        hist_init_kernel<<<int((npairs + 255) / 256), 256, 0, st>>>(d_ps, int(npairs), hmax,
                                                                    d_hist);
    }
    const uint32_t qcap = uint32_t(nsrc_tot);
    FallbackItem *d_q = (FallbackItem *)ctx->buf("i_queue", size_t(qcap) * sizeof(FallbackItem));
    // the box-search queue of the tiled passes (nn_tile_kernel -> nn_box_kernel)
    FallbackItem *d_bq = (FallbackItem *)ctx->buf("i_boxq", size_t(qcap) * sizeof(FallbackItem));
    uint8_t *d_tiled = nullptr;   // per grid slot: 1 = nn_tile_kernel settled the workgroup
    double *d_part = (double *)ctx->buf("i_part", size_t(std::max(slot, 1)) * LSM_ACC * 8);
    const int ncnt = max_iter + 2;
    uint32_t *d_counters = (uint32_t *)ctx->buf("i_counters", size_t(ncnt) * 4 * 4);
    double *d_bytes = (double *)ctx->buf("i_bytes", size_t(ncnt) * 8);
    unsigned long long *d_srcn = (unsigned long long *)ctx->buf("i_srcn", size_t(ncnt) * 8);
    int32_t *d_pref = (int32_t *)ctx->buf("i_pref", size_t(npairs + 1) * 4);
    int64_t nblk_all = 0;
    for (int64_t k = 0; k < npairs; ++k) nblk_all += ps[k].nblk;
    int4 *d_coarse = (int4 *)ctx->buf("i_coarse", size_t(nblk_all / PLAN_COARSE + 2) * 16);
    int32_t *d_plan = (int32_t *)ctx->buf("i_plan", size_t(ncnt + 1) * 2 * 4);
    int32_t *d_flags = (int32_t *)ctx->buf("i_flags", size_t(std::max<int64_t>(npairs, 1)) * 4);
    int32_t *d_err = (int32_t *)ctx->buf("i_err", 4);
    if (!d_corr || !d_rec || !d_q || !d_bq || !d_part || !d_counters || !d_bytes || !d_srcn || !d_pref ||
        !d_plan || !d_flags || !d_err || !d_coarse) {
        ctx->set_error("scratch allocation failed (icp)");
        return LSM_ENOMEM;
    }
    uint32_t *d_qn = d_counters;            // [ncnt] fallback queue sizes per pass
    uint32_t *d_active = d_counters + ncnt; // [ncnt] active pairs after each pass
    uint32_t *d_sqn = d_counters + 2 * ncnt; // [ncnt] uncertified queries per pass
    uint32_t *d_bqn = d_counters + 3 * ncnt; // [ncnt] box-search queue sizes (tiled passes)
    LSM_HIP_TRY(ctx, hipMemsetAsync(d_counters, 0, size_t(ncnt) * 4 * 4, st));
    LSM_HIP_TRY(ctx, hipMemsetAsync(d_err, 0, 4, st));
    LSM_HIP_TRY(ctx, hipMemsetAsync(d_bytes, 0, size_t(ncnt) * 8, st));
    LSM_HIP_TRY(ctx, hipMemsetAsync(d_srcn, 0, size_t(ncnt) * 8, st));
    if (src_off > 0) {
        LSM_HIP_TRY(ctx, hipMemsetAsync(d_corr, 0xff, size_t(src_off) * 4, st));
        LSM_HIP_TRY(ctx, hipMemsetAsync(d_rec, 0xff, size_t(src_off) * 8, st));
    }

    NNParams prm;
    prm.maxc = float(p.max_correspondence_distance);
    prm.hmax = hmax;
    prm.maxc2 = float(p.max_correspondence_distance * p.max_correspondence_distance);
    prm.method = p.method;
    prm.max_iter = max_iter;
    prm.rel_fit = p.relative_fitness;
    prm.rel_rmse = p.relative_rmse;
    // Search-path knobs (lsm_knob: test knobs, read per call; the tests switch them to prove
    // every search path exact -- the shipped values are the defaults):
    {   // LSM_NN_SPLIT: lanes per split box search (1 = one lane per query), LSM_NN_SPLIT_PLACE
        const int v = int(lsm_knob("LSM_NN_SPLIT", 8));
        int l = 1;
        while (l * 2 <= v && l < 64) l *= 2;
        prm.split_max = l;
    }
    prm.split_place = int(lsm_knob("LSM_NN_SPLIT_PLACE", 0));
    // certificate margin m = m_mul * delta + m_add (sweeps: DESIGN.md §7), pass-0 margin m0,
    // entry searches linear below `lin` points
    prm.m0 = 0.f;
    prm.lin = 8;
    prm.m_mul = 1.0;
    prm.m_add = 1e-3;
    {   // LSM_NN_DIRECT: warm-start distance in cells from which a query goes straight to the
        // fallback (<= 0: off) once a pair has made LSM_NN_DIRECT_ITER updates; LSM_NN_KCOLD /
        // LSM_NN_KMAX: the cold / warm box caps
        const double d = lsm_knob("LSM_NN_DIRECT", NN_DIRECT_RC);
        prm.direct_rc = d > 0.0 ? float(d) : INFINITY;
        prm.direct_iter = int(lsm_knob("LSM_NN_DIRECT_ITER", NN_DIRECT_ITER));
        prm.kcold = std::max(1, int(lsm_knob("LSM_NN_KCOLD", NN_KCOLD)));
        prm.kmax = std::max(1, int(lsm_knob("LSM_NN_KMAX", NN_KMAX)));
        prm.cold_seed = int(lsm_knob("LSM_NN_COLD_SEED", 1));
    }

    // Passes are launched back to back; the plan of each pass is rebuilt on the device after the
    // solve (plan_kernel), and kernels past the plan's end exit at once. The host only polls,
    // without waiting, the active-pair counts that already arrived in pinned memory: to stop
    // launching once every pair has converged and to shrink the grid of later passes.
    int64_t total_blk = 0;
    for (int64_t k = 0; k < npairs; ++k) total_blk += ps[k].nblk;
    const int64_t per0 = (total_blk + NXCD - 1) / NXCD;
    int grid = int(std::max<int64_t>(per0 * NXCD, NXCD));
    d_tiled = (uint8_t *)ctx->buf("i_tiled", size_t(grid));   // the grid only shrinks
    if (!d_tiled) {
        ctx->set_error("scratch allocation failed: i_tiled");
        return LSM_ENOMEM;
    }
    int32_t *h_poll = (int32_t *)ctx->host_pinned(size_t(ncnt) * 3 * 4);
    if (!h_poll) {
        ctx->set_error("pinned allocation failed (icp poll words)");
        return LSM_ENOMEM;
    }
    // plan_kernel stores the poll words into this mapped pinned buffer (no copy dispatches)
    int32_t *d_poll = nullptr;
    std::memset(h_poll, 0xff, size_t(ncnt) * 3 * 4);
    LSM_HIP_TRY(ctx, hipHostGetDevicePointer((void **)&d_poll, h_poll, 0));
    std::vector<hipEvent_t> pass_ev(size_t(ncnt), nullptr);
    int passes = 0, polled = 0;
    // the recorded pass events go back to the context's pool on every return, early ones included
    struct EventReturn {
        lsm_ctx *ctx;
        std::vector<hipEvent_t> &ev;
        const int &n;
        ~EventReturn() {
            for (int k = 0; k < n; ++k) ctx->event_pool.push_back(ev[size_t(k)]);
        }
    } ev_return{ctx, pass_ev, passes};
    // the fallback: GL lanes per queued query (LSM_FB_GL 16 / 32), LSM_FB_WAVES one-wave
    // workgroups per CU (grid-stride over the queue)
    // LSM_FB_GL 0 (default): chosen per pass on the device (nn_fallback_auto, LSM_FB_WIDE_MAX)
    // (16 lanes cannot hold a lane per range of a virtual block with more than 16 rows: 32 then)
    const int fb_gl = int(lsm_knob("LSM_FB_GL", 0)) == 16 ? FB_GL_MIN : int(lsm_knob("LSM_FB_GL", 0));
    // whole-wave queries only where the fallback can search far: max_corr >= LSM_FB_WIDE_MAXC m
    // (C3 / C4's 10 m; a multi-scale ladder's <= 2 m searches are short and cheaper at 32 lanes)
    const uint32_t fb_wide_max =
        p.max_correspondence_distance >= lsm_knob("LSM_FB_WIDE_MAXC", 4.0)
            ? uint32_t(lsm_knob("LSM_FB_WIDE_MAX", 200000)) : 0u;
    const int fb_wide_from = int(lsm_knob("LSM_FB_WIDE_FROM", 1 << 20));   // GL 64 from this pass
    const float fb_far = float(lsm_knob("LSM_FB_FAR", 0.0));   // far split (m; 0: off)
    const int fb_grid = std::max(1, std::min(ctx->num_cus * int(lsm_knob("LSM_FB_WAVES", 20)), 16384));
    const int box_grid = std::max(1, ctx->num_cus * 8);   // nn_box_kernel: grid-stride
    constexpr int PASS_LAG = 2;   // passes queued ahead of the last one read back
    // LSM_NN_NOCERT=1: search every query in every pass (no stability certificate) -- the
    // tests' proof that certified passes return bit-identical correspondences
    // passes before LSM_NN_CERT_FROM search every query without the stability check: pass 1
    // follows the first update, which moves the scans by centimetres to decimetres -- beyond
    // nearly every certificate -- so the check would only add its loads before the search
    const int CERT_FROM = std::max(1, int(lsm_knob("LSM_NN_CERT_FROM", 2)));
    // LSM_NN_TILE=1: the passes that search every query stage each workgroup's target cells in
    // LDS (nn_tile_kernel + nn_box_kernel); default 0: nn_kernel<false> reads the target from
    // global memory. Measured slower (nn 72.9 ms per C3 step global, 82.2 / 93.1 /
    // 119.8 with tiles of 2048 / 3072 / 4096 points): an option, proven exact by the tests.
    const bool tile_search = lsm_knob("LSM_NN_TILE", 0) != 0.0;
    // LSM_NN_FULL_L: lanes per query in the passes that search every query (1, 2 or 4)
    const int full_l = int(lsm_knob("LSM_NN_FULL_L", 1));
    double ms0 = 0.0;
    for (const char *k : {"nn", "nn_fallback"}) ms0 += ctx->stats[k].ms;
    unsigned long long *d_nst = nullptr;
#ifdef LSM_DIAG
    // diagnostics builds: per-pass search statistics to stderr (LSM_NN_STATS)
    static const bool nn_stats = getenv("LSM_NN_STATS") != nullptr;
#else
    constexpr bool nn_stats = false;
#endif
    if (nn_stats) {
        d_nst = (unsigned long long *)ctx->buf("i_nnstats", size_t(ncnt) * (NN_NSTAT + 8) * 8);
        if (!d_nst) return LSM_ENOMEM;
        LSM_HIP_TRY(ctx, hipMemsetAsync(d_nst, 0, size_t(ncnt) * (NN_NSTAT + 8) * 8, st));
    }
    plan_kernel<<<1, PLAN_THREADS, 0, st>>>(d_ps, int(npairs), d_pref, d_coarse, d_plan);
    const TaskPlan tp{d_plan, d_pref, d_coarse, int(npairs), d_err};
    int64_t queries = 0, queries0 = 0;   // source points searched (timing mode only)
    for (int pass = 0; pass <= max_iter; ++pass) {
        // newest active-pair counts that have landed; waits only to keep at most PASS_LAG
        // passes queued ahead of the last one read back
        bool done = false;
        while (polled < passes) {
            if (passes - polled > PASS_LAG) {
                LSM_HIP_TRY(ctx, hipEventSynchronize(pass_ev[size_t(polled)]));
            } else if (hipEventQuery(pass_ev[size_t(polled)]) != hipSuccess) {
                break;
            }
            const int32_t blocks_left = h_poll[3 * polled + 1];
            if (h_poll[3 * polled] == 0) done = true;
            // the plan only shrinks; a word that has not landed (-1 sentinel) keeps the grid
            if (blocks_left >= 0)
                grid = int(std::max<int64_t>(((int64_t(blocks_left) + NXCD - 1) / NXCD) * NXCD,
                                             NXCD));
            ++polled;
        }
        if (done) break;
        hipEvent_t ev;
        ctx->tic("nn", &ev);
        if (d_nst) {
            unsigned long long *sp = d_nst + size_t(pass) * NN_NSTAT;
            if (pass < CERT_FROM || nocert)
                nn_kernel<false, true><<<grid, NN_THREADS, 0, st>>>(
                    tp, d_ps, d_cd, prm, pass, d_hist, d_corr, d_rec, d_q, d_qn + pass, qcap, d_sqn + pass, sp);
            else
                nn_kernel<true, true><<<grid, NN_THREADS, 0, st>>>(
                    tp, d_ps, d_cd, prm, pass, d_hist, d_corr, d_rec, d_q, d_qn + pass, qcap, d_sqn + pass, sp);
        } else if ((pass < CERT_FROM || nocert) && tile_search) {
            nn_tile_kernel<<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_corr, d_rec,
                                                        d_bq, d_bqn + pass, qcap, d_tiled);
            nn_kernel<false><<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_hist, d_corr,
                                                          d_rec, d_q, d_qn + pass, qcap,
                                                          d_sqn + pass, nullptr, d_tiled);
            nn_box_kernel<<<box_grid, NN_THREADS, 0, st>>>(d_ps, d_cd, prm, pass, d_corr, d_rec,
                                                           d_bq, d_bqn + pass, qcap, d_q,
                                                           d_qn + pass, qcap);
        } else if ((pass < CERT_FROM || nocert) && full_l == 2)
            nn_full_kernel<2><<<grid, NN_THREADS * 2, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_corr,
                                                               d_rec, d_q, d_qn + pass, qcap);
        else if ((pass < CERT_FROM || nocert) && full_l == 4)
            nn_full_kernel<4><<<grid, NN_THREADS * 4, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_corr,
                                                               d_rec, d_q, d_qn + pass, qcap);
        else if (pass < CERT_FROM || nocert)
            nn_kernel<false><<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_hist, d_corr,
                                                                d_rec, d_q, d_qn + pass, qcap,
                                                                d_sqn + pass);
        else
            nn_kernel<true><<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, prm, pass, d_hist, d_corr,
                                                               d_rec, d_q, d_qn + pass, qcap,
                                                               d_sqn + pass);
        ctx->toc("nn", ev);
        ctx->tic("nn_fallback", &ev);
        {
            unsigned long long *fst = d_nst ? d_nst + size_t(ncnt) * NN_NSTAT + size_t(pass) * 8
                                            : nullptr;
            // from pass fb_wide_from on (the non-converging pairs' tail: few, costly queries) a
            // whole wave per query
            const int gl = pass >= fb_wide_from ? 64 : fb_gl;
            if (fb_gl == 0 && pass < fb_wide_from) {
                nn_fallback_auto<<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass, qcap,
                                                               d_corr, d_rec, pass, fst, fb_wide_max);
            } else if (gl != 64 && fb_far > 0.f) {
                // the far split: queries whose box-search best lies beyond fb_far (or that have
                // none) take a whole wave, the rest GL lanes
                const float f2 = fb_far * fb_far;
                if (gl == 16)
                    nn_fallback_g<FB_GL_MIN><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                    qcap, d_corr, d_rec, pass, fst, f2, 0);
                else
                    nn_fallback_g<32><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                    qcap, d_corr, d_rec, pass, fst, f2, 0);
                nn_fallback_g<64><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                qcap, d_corr, d_rec, pass, fst, f2, 1);
            } else if (gl == 16)
                nn_fallback_g<FB_GL_MIN><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                qcap, d_corr, d_rec, pass, fst, INFINITY, 0);
            else if (gl == 64)
                nn_fallback_g<64><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                qcap, d_corr, d_rec, pass, fst, INFINITY, 0);
            else
                nn_fallback_g<32><<<fb_grid, LSM_WAVE, 0, st>>>(d_ps, d_cd, prm, d_q, d_qn + pass,
                                                                qcap, d_corr, d_rec, pass, fst, INFINITY, 0);
        }
        ctx->toc("nn_fallback", ev);
        ctx->tic("accumulate", &ev);
        // the normals' side-stream refine (pre-processing or the lazy targets above) has
        // overlapped this pass's correspondence search; the accumulation reads the normals
        ctx->join_side_device();
        if (p.method == LSM_P2PLANE)
            accumulate_kernel<LSM_P2PLANE><<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, d_corr,
                                                                        d_part);
        else
            accumulate_kernel<LSM_P2P><<<grid, NN_THREADS, 0, st>>>(tp, d_ps, d_cd, d_corr,
                                                                    d_part);
        ctx->toc("accumulate", ev);
        ctx->tic("solve", &ev);
        solve_kernel<<<int(npairs), LSM_WAVE, 0, st>>>(d_ps, d_part, prm, pass, d_pbytes,
                                                       d_active + pass, d_bytes + pass,
                                                       d_srcn + pass, d_flags, d_hist);
        ctx->toc("solve", ev);
        plan_kernel<<<1, PLAN_THREADS, 0, st>>>(d_ps, int(npairs), d_pref, d_coarse, d_plan,
                                                d_active + pass, d_poll + 3 * pass);
        pass_ev[size_t(pass)] = ctx->get_event();
        LSM_HIP_TRY(ctx, hipEventRecord(pass_ev[size_t(pass)], st));
        ++passes;
    }
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    {
        int32_t herr = 0;
        LSM_HIP_TRY(ctx, hipMemcpy(&herr, d_err, 4, hipMemcpyDeviceToHost));
        if (herr) {
            ctx->set_error("internal: correspondence pass launched on a grid smaller than its plan");
            return LSM_EHIP;
        }
    }
    if (d_nst) {   // per pass: searched, rows, runs, bsearch steps, points, K, cold, pending
        std::vector<unsigned long long> h(size_t(ncnt) * (NN_NSTAT + 8));
        LSM_HIP_TRY(ctx, hipMemcpy(h.data(), d_nst, h.size() * 8, hipMemcpyDeviceToHost));
        for (int k = 0; k < passes; ++k) {
            const unsigned long long *v = h.data() + size_t(k) * NN_NSTAT;
            const double q = double(std::max(v[0], 1ull));
            fprintf(stderr,
                    "nnstat pass %2d: searched %9llu rows %.2f runs %.2f bsearch %.2f points %.2f "
                    "K %.2f cold %.3f pending %.4f\n",
                    k, v[0], v[1] / q, v[2] / q, v[3] / q, v[4] / q, v[5] / q, v[6] / q, v[7] / q);
            const unsigned long long *f = h.data() + size_t(ncnt) * NN_NSTAT + size_t(k) * 8;
            const double fq = double(std::max(f[0], 1ull));
            fprintf(stderr,
                    "fbstat pass %2d: queries %8llu rings %.2f chunks %.2f blocks %.2f points "
                    "%.1f hits %.3f outside %.3f max-item chunks %llu blocks %llu\n",
                    k, f[0], f[1] / fq, f[2] / fq, f[3] / fq, f[4] / fq, f[5] / fq, f[6] / fq,
                    f[7] >> 32, f[7] & 0xffffffffull);
        }
    }
    double nn_bytes = 0.0;
    {
        std::vector<double> hb(size_t(passes) + 1, 0.0);
        LSM_HIP_TRY(ctx, hipMemcpy(hb.data(), d_bytes, size_t(passes) * 8, hipMemcpyDeviceToHost));
        nn_bytes = bytes0;   // pass 0: every pair
        for (int k = 0; k + 1 < passes; ++k) nn_bytes += hb[size_t(k)];
        if (ctx->timing) {   // source points searched: all of them, then the active pairs'
            std::vector<unsigned long long> sn(size_t(passes), 0ull);
            LSM_HIP_TRY(ctx, hipMemcpy(sn.data(), d_srcn, size_t(passes) * 8,
                                       hipMemcpyDeviceToHost));
            queries0 = src_off;
            queries = src_off;
            for (int k = 0; k + 1 < passes; ++k) queries += int64_t(sn[size_t(k)]);
        }
    }
    LSM_HIP_TRY(ctx, hipGetLastError());
    // results
    LSM_HIP_TRY(ctx, hipMemcpyAsync(ps.data(), d_ps, ps.size() * sizeof(PairState),
                                    hipMemcpyDeviceToHost, st));
    // pair 0 correspondences in reference order, left on the device until asked for
    {
        const int n0 = int(src[0]->n);
        int32_t *d_dense = (int32_t *)ctx->buf("i_lastcorr_dense", size_t(std::max(n0, 1)) * 4);
        if (!d_dense) return LSM_ENOMEM;
        if (n0 > 0)
            corr_to_ref<<<(n0 + 255) / 256, 256, 0, st>>>(d_corr, n0, src[0]->d_perm,
                                                         tgt[0]->d_perm, d_dense);
        ctx->last_corr_dense_n = n0;
        ctx->last_corr_pending = true;
        ctx->last_corr.clear();
    }
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    ctx->collect_timings();
    if (ctx->timing) {
        ctx->stats["nn"].algo_bytes += nn_bytes;
        // the whole correspondence pass (check + search + fallback) of every pass
        double ms1 = 0.0;
        for (const char *k : {"nn", "nn_fallback"}) ms1 += ctx->stats[k].ms;
        KStat &np = ctx->stats["nn_pass"];
        np.launches += passes;
        np.ms += ms1 - ms0;
        np.algo_bytes += nn_bytes;
        std::vector<uint32_t> sq(passes);
        LSM_HIP_TRY(ctx, hipMemcpy(sq.data(), d_sqn, size_t(passes) * 4, hipMemcpyDeviceToHost));
        int64_t searched = 0;
        for (int k = 1; k < passes; ++k) searched += sq[k];
        ctx->stats["nn_uncertified"].launches += searched;
        // search statistics: queries and the ones the fast path left to the fallback
        std::vector<uint32_t> qn(passes);
        LSM_HIP_TRY(ctx, hipMemcpy(qn.data(), d_qn, size_t(passes) * 4, hipMemcpyDeviceToHost));
        int64_t pend = 0;
        for (int k = 0; k < passes; ++k) pend += qn[k];
        ctx->stats["nn_queries"].launches += queries;
        ctx->stats["nn_queries_first_pass"].launches += queries0;
        ctx->stats["nn_pending"].launches += pend;
        ctx->stats["nn_pending_first_pass"].launches += passes > 0 ? qn[0] : 0;
#ifdef LSM_DIAG
        if (getenv("LSM_DEBUG_PASSES")) {   // per pass: active pairs, searched, fallback
            std::vector<uint32_t> act(passes);
            LSM_HIP_TRY(ctx, hipMemcpy(act.data(), d_active, size_t(passes) * 4,
                                       hipMemcpyDeviceToHost));
            for (int k = 0; k < passes; ++k)
                fprintf(stderr, "pass %2d: active-after %4u  searched %8u  fallback %7u\n", k,
                        act[k], sq[k], qn[k]);
        }
#endif
    }
    for (int64_t k = 0; k < npairs; ++k) {
        const PairState &P = ps[k];
        lsm_icp_result &R = out[k];
        std::memcpy(R.transformation, P.T, sizeof(R.transformation));
        R.fitness = P.fitness;
        R.inlier_rmse = P.rmse;
        R.correspondences = P.ncorr;
        R.iterations = P.iter;
        R.status = 0;
    }
    return LSM_OK;
}
