// plane.hip -- the 'icp2planes' pre-processing on the device:
//
//   KeyFrame.calculate_plane (keyframe.py:417-437): points with z < height -> [O3D]
//       PointCloud.segment_plane(distance_threshold, ransac_n = 3, num_iterations) (RANSAC)
//   KeyFrame.segment_plane   (keyframe.py:439-461): |a x + b y + c z + d| / |(a, b, c)| < thr
//       -> ground / non-ground clouds (select_by_index keeps the index order)
//
// RANSAC as Open3D's SegmentPlane restates it (sequential form): candidate planes from three
// distinct sampled points (TriangleMesh::ComputeTrianglePlane), scored by inlier count
// (|plane . (p, 1)| <= thr) then error / sqrt(count); the sampling loop stops once the number of
// evaluated candidates exceeds log(1 - probability) / log(1 - fitness^3) of the best so far;
// the winner is refit to its inliers (GetPlaneFromPoints: centroid + determinant-form normal).
// The reference's sampler is Open3D's unseeded RNG (not reproducible even by the reference);
// here the samples come from splitmix64(seed) on the host (lsm_plane.h), restated by the oracle.
//
// One call handles one keyframe: every candidate plane is scored by one lane that walks the
// subset in index order (the same f64 sums as the sequential loop: bit-exact counts and
// errors); the refit and the split run in one workgroup.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>

#include "lsm_ctx.h"
#include "lsm_umeyama.h"

namespace {

constexpr int CT = 1024;   // single-workgroup compaction / reduction width

// sorted float4 cloud -> reference-order f64 rows (filter order)
__global__ void ref_points_kernel(const float4 *__restrict__ xyz, const uint32_t *__restrict__ perm,
                                  int n, double *__restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const float4 p = xyz[j];
    const size_t r = perm[j];
    out[3 * r] = p.x;
    out[3 * r + 1] = p.y;
    out[3 * r + 2] = p.z;
}

// Order-preserving compaction in one workgroup: rank of every flagged element among the flagged
// ones, by wave ballots and an LDS prefix of the wave totals, chunk by chunk.
template <typename Pred, typename Emit>
__device__ void compact_block(int n, Pred pred, Emit emit, uint32_t &total) {
    __shared__ uint32_t wcnt[CT / LSM_WAVE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += CT) {
        const int i = base + int(threadIdx.x);
        const int f = (i < n) ? pred(i) : -1;   // -1: not flagged; >= 0: output class
        const bool on = f >= 0;
        const uint64_t m = __ballot(on);
        if (lane == 0) wcnt[w] = __popcll(m);
        __syncthreads();
        uint32_t before = carry, tot = 0;
        for (int q = 0; q < CT / LSM_WAVE; ++q) {
            before += q < w ? wcnt[q] : 0u;
            tot += wcnt[q];
        }
        if (on) emit(i, f, before + __popcll(m & ((uint64_t(1) << lane) - 1)));
        carry += tot;
        __syncthreads();
    }
    total = carry;
}

__device__ __forceinline__ double dot4(const double *pl, double x, double y, double z) {
    // ((a x + b y) + c z) + d, every product and sum rounded (no contraction)
    return lsm_dadd(lsm_dadd(lsm_dadd(lsm_dmul(pl[0], x), lsm_dmul(pl[1], y)),
                             lsm_dmul(pl[2], z)), pl[3]);
}

// sorted normals -> reference order
__global__ void ref_normals_kernel(const float4 *__restrict__ nrm, const uint32_t *__restrict__ perm,
                                   int n, float4 *__restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[perm[j]] = nrm[j];
}

// z < height subset of the reference-order points, in order
__global__ void __launch_bounds__(CT)
subset_below_kernel(const double *__restrict__ P, int n, double height, double *__restrict__ sub,
                    uint32_t *__restrict__ n_sub) {
    uint32_t tot = 0;
    compact_block(
        n, [&](int i) { return P[3 * i + 2] < height ? 0 : -1; },
        [&](int i, int, uint32_t slot) {
            sub[3 * slot] = P[3 * i];
            sub[3 * slot + 1] = P[3 * i + 1];
            sub[3 * slot + 2] = P[3 * i + 2];
        },
        tot);
    if (threadIdx.x == 0) *n_sub = tot;
}

// TriangleMesh::ComputeTrianglePlane: abc = (p1 - p0) x (p2 - p0) / |.|, d = -abc . p0
__device__ bool triangle_plane(const double *p0, const double *p1, const double *p2, double *pl) {
    const double e0[3] = {lsm_dsub(p1[0], p0[0]), lsm_dsub(p1[1], p0[1]), lsm_dsub(p1[2], p0[2])};
    const double e1[3] = {lsm_dsub(p2[0], p0[0]), lsm_dsub(p2[1], p0[1]), lsm_dsub(p2[2], p0[2])};
    double a = lsm_dsub(lsm_dmul(e0[1], e1[2]), lsm_dmul(e0[2], e1[1]));
    double b = lsm_dsub(lsm_dmul(e0[2], e1[0]), lsm_dmul(e0[0], e1[2]));
    double c = lsm_dsub(lsm_dmul(e0[0], e1[1]), lsm_dmul(e0[1], e1[0]));
    const double nrm = sqrt(lsm_dadd(lsm_dadd(lsm_dmul(a, a), lsm_dmul(b, b)), lsm_dmul(c, c)));
    if (nrm == 0.0) return false;
    a = lsm_ddiv(a, nrm);
    b = lsm_ddiv(b, nrm);
    c = lsm_ddiv(c, nrm);
    const double d = -lsm_dadd(lsm_dadd(lsm_dmul(a, p0[0]), lsm_dmul(b, p0[1])), lsm_dmul(c, p0[2]));
    pl[0] = a;
    pl[1] = b;
    pl[2] = c;
    pl[3] = d;
    return true;
}

// one lane per candidate: its plane, inlier count and error sum in subset order
__global__ void __launch_bounds__(LSM_WAVE)
ransac_eval_kernel(const double *__restrict__ sub, int n_sub, const int32_t *__restrict__ samples,
                   int iters, double thr, double *__restrict__ models,
                   uint32_t *__restrict__ counts, double *__restrict__ errs,
                   int32_t *__restrict__ valid) {
    const int it = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = it < iters;
    double pl[4] = {0.0, 0.0, 0.0, 0.0};
    bool ok = false;
    if (live) {
        const int32_t *s = samples + 3 * it;
        ok = triangle_plane(sub + 3 * s[0], sub + 3 * s[1], sub + 3 * s[2], pl);
    }
    uint32_t cnt = 0;
    double err = 0.0;
    if (__ballot(ok)) {
        for (int i = 0; i < n_sub; ++i) {   // every lane reads the same point: broadcast
            const double dist = fabs(dot4(pl, sub[3 * i], sub[3 * i + 1], sub[3 * i + 2]));
            if (ok && dist <= thr) {
                ++cnt;
                err = lsm_dadd(err, dist);
            }
        }
    }
    if (live) {
        for (int k = 0; k < 4; ++k) models[4 * it + k] = pl[k];
        counts[it] = cnt;
        errs[it] = err;
        valid[it] = ok ? 1 : 0;
    }
}

// Sequential selection (lane 0) + GetPlaneFromPoints refit of the winner's inliers (fixed-tree
// f64 sums over the workgroup) -> out[0..3] plane, out[4] inliers (as double), out[5] winner.
__global__ void __launch_bounds__(CT)
ransac_finish_kernel(const double *__restrict__ sub, int n_sub, const double *__restrict__ models,
                     const uint32_t *__restrict__ counts, const double *__restrict__ errs,
                     const int32_t *__restrict__ valid, int iters, double thr, double probability,
                     double *__restrict__ out) {
    __shared__ double best[4];
    __shared__ int s_win;
    __shared__ double red[CT / LSM_WAVE][9];
    if (threadIdx.x == 0) {
        double bfit = 0.0, brmse = 0.0;
        int win = -1;
        double break_it = INFINITY;
        long count = 0;
        for (int it = 0; it < iters; ++it) {
            if (double(count) > break_it) continue;
            if (!valid[it]) continue;
            const double fit = counts[it] ? double(counts[it]) / double(n_sub) : 0.0;
            const double rmse = counts[it] ? errs[it] / sqrt(double(counts[it])) : 0.0;
            if (fit > bfit || (fit == bfit && rmse < brmse)) {
                bfit = fit;
                brmse = rmse;
                win = it;
                break_it = fit < 1.0 ? fmin(log(1.0 - probability) / log(1.0 - pow(fit, 3.0)),
                                            double(iters))
                                     : 0.0;
            }
            ++count;
        }
        s_win = win;
        for (int k = 0; k < 4; ++k) best[k] = win >= 0 ? models[4 * win + k] : 0.0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool have = s_win >= 0;
    // pass 1: inlier count and coordinate sums; pass 2: centred second moments
    double v[9];
    auto reduce = [&](int nv) {
        for (int k = 0; k < nv; ++k) {
            double x = v[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, LSM_WAVE);
            if (lane == 0) red[w][k] = x;
        }
        __syncthreads();
        for (int k = 0; k < nv; ++k) {
            double x = 0.0;
            for (int q = 0; q < CT / LSM_WAVE; ++q) x += red[q][k];
            v[k] = x;
        }
        __syncthreads();
    };
    for (int k = 0; k < 9; ++k) v[k] = 0.0;
    for (int i = threadIdx.x; have && i < n_sub; i += CT) {
        const double *p = sub + 3 * i;
        if (fabs(dot4(best, p[0], p[1], p[2])) <= thr) {
            v[0] += 1.0;
            v[1] += p[0];
            v[2] += p[1];
            v[3] += p[2];
        }
    }
    reduce(4);
    const double n_in = v[0];
    const double cx = n_in > 0 ? v[1] / n_in : 0.0, cy = n_in > 0 ? v[2] / n_in : 0.0,
                 cz = n_in > 0 ? v[3] / n_in : 0.0;
    for (int k = 0; k < 9; ++k) v[k] = 0.0;
    for (int i = threadIdx.x; have && i < n_sub; i += CT) {
        const double *p = sub + 3 * i;
        if (fabs(dot4(best, p[0], p[1], p[2])) <= thr) {
            const double rx = p[0] - cx, ry = p[1] - cy, rz = p[2] - cz;
            v[0] += rx * rx;
            v[1] += rx * ry;
            v[2] += rx * rz;
            v[3] += ry * ry;
            v[4] += ry * rz;
            v[5] += rz * rz;
        }
    }
    reduce(6);
    if (threadIdx.x != 0) return;
    const double xx = v[0], xy = v[1], xz = v[2], yy = v[3], yz = v[4], zz = v[5];
    const double det_x = yy * zz - yz * yz, det_y = xx * zz - xz * xz, det_z = xx * yy - xy * xy;
    double a, b, c;
    if (det_x > det_y && det_x > det_z) {
        a = det_x;
        b = xz * yz - xy * zz;
        c = xy * yz - xz * yy;
    } else if (det_y > det_z) {
        a = xz * yz - xy * zz;
        b = det_y;
        c = xy * xz - yz * xx;
    } else {
        a = xy * yz - xz * yy;
        b = xy * xz - yz * xx;
        c = det_z;
    }
    const double nrm = sqrt(a * a + b * b + c * c);
    if (!have || n_in <= 0 || nrm == 0.0) {
        out[0] = out[1] = out[2] = out[3] = 0.0;
    } else {
        a /= nrm;
        b /= nrm;
        c /= nrm;
        out[0] = a;
        out[1] = b;
        out[2] = c;
        out[3] = -(a * cx + b * cy + c * cz);
    }
    out[4] = n_in;
    out[5] = double(s_win);
}

// segment_plane: |a x + b y + c z + d| / sqrt(a a + b b + c c) < thr (numpy's evaluation order)
__global__ void __launch_bounds__(CT)
split_kernel(const double *__restrict__ P, const float4 *__restrict__ N, int n,
             const double *__restrict__ plane, double thr, float *__restrict__ ground,
             float *__restrict__ rest, float4 *__restrict__ gN, float4 *__restrict__ rN,
             uint32_t *__restrict__ counts) {
    const double a = plane[0], b = plane[1], c = plane[2], d = plane[3];
    const double den = sqrt(lsm_dadd(lsm_dadd(lsm_dmul(a, a), lsm_dmul(b, b)), lsm_dmul(c, c)));
    uint32_t tg = 0, tr = 0;
    auto is_ground = [&](int i) {
        const double num = fabs(lsm_dadd(lsm_dadd(lsm_dadd(lsm_dmul(a, P[3 * i]),
                                                           lsm_dmul(b, P[3 * i + 1])),
                                                  lsm_dmul(c, P[3 * i + 2])), d));
        return lsm_ddiv(num, den) < thr;
    };
    compact_block(
        n, [&](int i) { return is_ground(i) ? 0 : -1; },
        [&](int i, int, uint32_t slot) {
            ground[3 * slot] = float(P[3 * i]);
            ground[3 * slot + 1] = float(P[3 * i + 1]);
            ground[3 * slot + 2] = float(P[3 * i + 2]);
            if (N) gN[slot] = N[i];
        },
        tg);
    compact_block(
        n, [&](int i) { return is_ground(i) ? -1 : 0; },
        [&](int i, int, uint32_t slot) {
            rest[3 * slot] = float(P[3 * i]);
            rest[3 * slot + 1] = float(P[3 * i + 1]);
            rest[3 * slot + 2] = float(P[3 * i + 2]);
            if (N) rN[slot] = N[i];
        },
        tr);
    if (threadIdx.x == 0) {
        counts[0] = tg;
        counts[1] = tr;
    }
}

// Feature-RANSAC hypotheses (RegistrationRANSACBasedOnCorrespondence, ransac_n = 3): one lane
// per iteration -- the sampled correspondences' Umeyama transform, the edge-length (similarity)
// and distance checkers, and the correspondence inlier ratio (|T s - t|^2 < max_corr^2 over all
// correspondences) that drives the early exit.
__global__ void __launch_bounds__(LSM_WAVE)
ransac_hyp_kernel(const double *__restrict__ S, const double *__restrict__ Tg,
                  const int32_t *__restrict__ corr, int ncorr, const int32_t *__restrict__ samples,
                  int iters, double max_corr, double edge, double *__restrict__ T,
                  int32_t *__restrict__ valid, double *__restrict__ ratio) {
    const int it = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = it < iters;
    double D[16];
    double ps[3][3], pt[3][3];
    if (ok) {
        for (int r = 0; r < 3; ++r) {
            const int c = samples[3 * it + r];
            const int i = corr[2 * c], j = corr[2 * c + 1];
            for (int d = 0; d < 3; ++d) {
                ps[r][d] = S[3 * i + d];
                pt[r][d] = Tg[3 * j + d];
            }
        }
        double tot[32];
        for (int k = 0; k < 32; ++k) tot[k] = 0.0;
        for (int r = 0; r < 3; ++r) {
            for (int d = 0; d < 3; ++d) {
                tot[d] += ps[r][d];
                tot[3 + d] += pt[r][d];
            }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) tot[6 + 3 * a + b] += pt[r][a] * ps[r][b];
        }
        tot[29] = 3.0;
        lsm::umeyama_update(tot, D);
        for (int i = 0; i < 3 && ok; ++i)
            for (int j = i + 1; j < 3; ++j) {
                const double ex = ps[i][0] - ps[j][0], ey = ps[i][1] - ps[j][1], ez = ps[i][2] - ps[j][2];
                const double fx = pt[i][0] - pt[j][0], fy = pt[i][1] - pt[j][1], fz = pt[i][2] - pt[j][2];
                const double ds = sqrt((ex * ex + ey * ey) + ez * ez);
                const double dt = sqrt((fx * fx + fy * fy) + fz * fz);
                if (ds < dt * edge || dt < ds * edge) ok = false;
            }
        for (int r = 0; r < 3 && ok; ++r) {
            const double x = D[0] * ps[r][0] + D[1] * ps[r][1] + D[2] * ps[r][2] + D[3];
            const double y = D[4] * ps[r][0] + D[5] * ps[r][1] + D[6] * ps[r][2] + D[7];
            const double z = D[8] * ps[r][0] + D[9] * ps[r][1] + D[10] * ps[r][2] + D[11];
            const double ex = pt[r][0] - x, ey = pt[r][1] - y, ez = pt[r][2] - z;
            if (sqrt((ex * ex + ey * ey) + ez * ez) > max_corr) ok = false;
        }
    }
    uint32_t in = 0;
    if (__ballot(ok)) {
        const double m2 = max_corr * max_corr;
        for (int c = 0; c < ncorr; ++c) {   // every lane reads the same correspondence
            const int i = corr[2 * c], j = corr[2 * c + 1];
            if (!ok) continue;
            const double sx = S[3 * i], sy = S[3 * i + 1], sz = S[3 * i + 2];
            const double x = D[0] * sx + D[1] * sy + D[2] * sz + D[3];
            const double y = D[4] * sx + D[5] * sy + D[6] * sz + D[7];
            const double z = D[8] * sx + D[9] * sy + D[10] * sz + D[11];
            const double ex = x - Tg[3 * j], ey = y - Tg[3 * j + 1], ez = z - Tg[3 * j + 2];
            in += ((ex * ex + ey * ey) + ez * ez) < m2 ? 1u : 0u;
        }
    }
    if (it < iters) {
        for (int k = 0; k < 16; ++k) T[16 * size_t(it) + k] = ok ? D[k] : 0.0;
        valid[it] = ok ? 1 : 0;
        ratio[it] = ok ? double(in) / double(ncorr) : 0.0;
    }
}

}  // namespace

// splitmix64 stream: value k of seed s
static uint64_t splitmix(uint64_t s, uint64_t k) {
    uint64_t z = s + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void lsm_plane_samples(uint64_t seed, int64_t n, int64_t iters, int32_t *out) {
    for (int64_t it = 0; it < iters; ++it) {
        const uint64_t u0 = splitmix(seed, 3 * it), u1 = splitmix(seed, 3 * it + 1),
                       u2 = splitmix(seed, 3 * it + 2);
        int64_t i0 = int64_t(u0 % uint64_t(n));
        int64_t i1 = int64_t(u1 % uint64_t(n - 1));
        if (i1 >= i0) ++i1;
        int64_t i2 = int64_t(u2 % uint64_t(n - 2));
        const int64_t lo = i0 < i1 ? i0 : i1, hi = i0 < i1 ? i1 : i0;
        if (i2 >= lo) ++i2;
        if (i2 >= hi) ++i2;
        out[3 * it] = int32_t(i0);
        out[3 * it + 1] = int32_t(i1);
        out[3 * it + 2] = int32_t(i2);
    }
}

// reference-order f64 points of a processed cloud into scratch "pl_P"
static int ref_points(lsm_ctx *ctx, Cloud *c, double **out) {
    const int n = int(c->n);
    double *P = (double *)ctx->buf("pl_P", size_t(std::max(n, 1)) * 24);
    if (!P) return LSM_ENOMEM;
    if (n > 0) {
        if (c->voxelized) {
            LSM_HIP_TRY(ctx, hipMemcpyAsync(P, c->d_vox, size_t(n) * 24, hipMemcpyDeviceToDevice,
                                            ctx->stream));
        } else {
            ref_points_kernel<<<(n + 255) / 256, 256, 0, ctx->stream>>>(c->d_xyz, c->d_perm, n, P);
        }
    }
    *out = P;
    return LSM_OK;
}

int lsm_ground_plane_run(lsm_ctx *ctx, Cloud *c, double height, double thr, int64_t iters,
                         uint64_t seed, double probability, double plane[4], int64_t *n_inliers,
                         int64_t *n_subset) {
    hipStream_t st = ctx->stream;
    double *P;
    int rc;
    if ((rc = ref_points(ctx, c, &P))) return rc;
    const int n = int(c->n);
    double *sub = (double *)ctx->buf("pl_sub", size_t(std::max(n, 1)) * 24);
    uint32_t *d_cnt = (uint32_t *)ctx->buf("pl_cnt", 16);
    if (!sub || !d_cnt) return LSM_ENOMEM;
    subset_below_kernel<<<1, CT, 0, st>>>(P, n, height, sub, d_cnt);
    uint32_t n_sub = 0;
    LSM_HIP_TRY(ctx, hipMemcpyAsync(&n_sub, d_cnt, 4, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    if (n_subset) *n_subset = n_sub;
    if (n_sub < 3) {
        ctx->set_error("There must be at least 'ransac_n' points.");
        return LSM_EINVAL;
    }
    std::vector<int32_t> samples(size_t(iters) * 3);
    lsm_plane_samples(seed, int64_t(n_sub), iters, samples.data());
    int32_t *d_s = (int32_t *)ctx->buf("pl_samples", samples.size() * 4);
    double *d_models = (double *)ctx->buf("pl_models", size_t(iters) * 32);
    uint32_t *d_counts = (uint32_t *)ctx->buf("pl_counts", size_t(iters) * 4);
    double *d_errs = (double *)ctx->buf("pl_errs", size_t(iters) * 8);
    int32_t *d_valid = (int32_t *)ctx->buf("pl_valid", size_t(iters) * 4);
    double *d_out = (double *)ctx->buf("pl_out", 64);
    if (!d_s || !d_models || !d_counts || !d_errs || !d_valid || !d_out) return LSM_ENOMEM;
    LSM_HIP_TRY(ctx, hipMemcpyAsync(d_s, samples.data(), samples.size() * 4, hipMemcpyHostToDevice,
                                    st));
    hipEvent_t ev;
    ctx->tic("plane", &ev);
    ransac_eval_kernel<<<int((iters + LSM_WAVE - 1) / LSM_WAVE), LSM_WAVE, 0, st>>>(
        sub, int(n_sub), d_s, int(iters), thr, d_models, d_counts, d_errs, d_valid);
    ransac_finish_kernel<<<1, CT, 0, st>>>(sub, int(n_sub), d_models, d_counts, d_errs, d_valid,
                                           int(iters), thr, probability, d_out);
    ctx->toc("plane", ev);
    double h[6];
    LSM_HIP_TRY(ctx, hipMemcpyAsync(h, d_out, sizeof(h), hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    ctx->collect_timings();
    std::memcpy(plane, h, 4 * sizeof(double));
    if (n_inliers) *n_inliers = int64_t(h[4]);
    return LSM_OK;
}

// new raw clouds (f32, reference order) with the ground / non-ground points of c
int lsm_split_plane_run(lsm_ctx *ctx, Cloud *c, const double plane[4], double thr, Cloud *g,
                        Cloud *r) {
    hipStream_t st = ctx->stream;
    double *P;
    int rc;
    if ((rc = ref_points(ctx, c, &P))) return rc;
    const int n = int(c->n);
    double *d_pl = (double *)ctx->buf("pl_plane", 32);
    uint32_t *d_cnt = (uint32_t *)ctx->buf("pl_cnt", 16);
    if (!d_pl || !d_cnt) return LSM_ENOMEM;
    // the split parts keep the cloud's normals as their prior (select_by_index copies them;
    // EstimateNormals then orients the new normals to them)
    const bool carry = c->has_normals;
    for (Cloud *o : {g, r}) {
        if (hipMalloc(&o->d_raw, size_t(std::max(n, 1)) * 12) != hipSuccess ||
            (carry && hipMalloc(&o->d_prior_ref, size_t(std::max(n, 1)) * 16) != hipSuccess)) {
            ctx->set_error("hipMalloc failed for split cloud");
            return LSM_ENOMEM;
        }
    }
    float4 *N = nullptr;
    if (carry && n > 0) {
        N = (float4 *)ctx->buf("pl_nrm", size_t(n) * 16);
        if (!N) return LSM_ENOMEM;
        ref_normals_kernel<<<(n + 255) / 256, 256, 0, st>>>(c->d_nrm, c->d_perm, n, N);
    }
    LSM_HIP_TRY(ctx, hipMemcpyAsync(d_pl, plane, 32, hipMemcpyHostToDevice, st));
    split_kernel<<<1, CT, 0, st>>>(P, N, n, d_pl, thr, g->d_raw, r->d_raw, g->d_prior_ref,
                                   r->d_prior_ref, d_cnt);
    uint32_t h[2];
    LSM_HIP_TRY(ctx, hipMemcpyAsync(h, d_cnt, 8, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    g->n_raw = h[0];
    r->n_raw = h[1];
    g->prior_n = carry ? int64_t(h[0]) : 0;
    r->prior_n = carry ? int64_t(h[1]) : 0;
    return LSM_OK;
}

void lsm_ransac_samples(uint64_t seed, int64_t ncorr, int64_t iters, int32_t *out) {
    for (int64_t k = 0; k < iters * 3; ++k) out[k] = int32_t(splitmix(seed, k) % uint64_t(ncorr));
}

// RegistrationRANSACBasedOnCorrespondence, sequential form: iterations below the running
// estimate k are taken in order; a hypothesis that passes the checkers is evaluated by one
// correspondence pass of the ICP machinery (1-NN within max_corr: fitness, rmse); a better one
// (fitness, then rmse) lowers k to ceil(log(1 - confidence) / log(1 - ratio^3)).
int lsm_ransac_run(lsm_ctx *ctx, Cloud *src, Cloud *tgt, const int32_t *corr, int64_t ncorr,
                   double max_corr, double edge, int64_t iters, double confidence, uint64_t seed,
                   double T[16], double *fitness, double *rmse, int64_t *evaluated) {
    hipStream_t st = ctx->stream;
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    *fitness = *rmse = 0.0;
    *evaluated = 0;
    if (ncorr < 3 || iters <= 0) return LSM_OK;
    double *P;
    int rc;
    if ((rc = ref_points(ctx, src, &P))) return rc;
    double *dS = (double *)ctx->buf("rs_src", size_t(std::max<int64_t>(src->n, 1)) * 24);
    if (!dS) return LSM_ENOMEM;
    if (src->n > 0)
        LSM_HIP_TRY(ctx, hipMemcpyAsync(dS, P, size_t(src->n) * 24, hipMemcpyDeviceToDevice, st));
    if ((rc = ref_points(ctx, tgt, &P))) return rc;   // "pl_P" now holds the target
    std::vector<int32_t> samples(size_t(iters) * 3);
    lsm_ransac_samples(seed, ncorr, iters, samples.data());
    int32_t *d_corr = (int32_t *)ctx->buf("rs_corr", size_t(ncorr) * 8);
    int32_t *d_s = (int32_t *)ctx->buf("rs_samples", samples.size() * 4);
    double *d_T = (double *)ctx->buf("rs_T", size_t(iters) * 128);
    int32_t *d_valid = (int32_t *)ctx->buf("rs_valid", size_t(iters) * 4);
    double *d_ratio = (double *)ctx->buf("rs_ratio", size_t(iters) * 8);
    if (!d_corr || !d_s || !d_T || !d_valid || !d_ratio) return LSM_ENOMEM;
    LSM_HIP_TRY(ctx, hipMemcpyAsync(d_corr, corr, size_t(ncorr) * 8, hipMemcpyHostToDevice, st));
    LSM_HIP_TRY(ctx, hipMemcpyAsync(d_s, samples.data(), samples.size() * 4, hipMemcpyHostToDevice, st));
    hipEvent_t ev;
    ctx->tic("ransac", &ev);
    ransac_hyp_kernel<<<int((iters + LSM_WAVE - 1) / LSM_WAVE), LSM_WAVE, 0, st>>>(
        dS, P, d_corr, int(ncorr), d_s, int(iters), max_corr, edge, d_T, d_valid, d_ratio);
    ctx->toc("ransac", ev);
    std::vector<int32_t> valid(iters);
    std::vector<double> ratio(iters), hT(size_t(iters) * 16);
    LSM_HIP_TRY(ctx, hipMemcpyAsync(valid.data(), d_valid, size_t(iters) * 4, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipMemcpyAsync(ratio.data(), d_ratio, size_t(iters) * 8, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipMemcpyAsync(hT.data(), d_T, hT.size() * 8, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    ctx->collect_timings();
    lsm_icp_params ip;
    ip.max_correspondence_distance = max_corr;
    ip.method = LSM_P2P;
    ip.max_iteration = 0;
    ip.relative_fitness = 1e-6;
    ip.relative_rmse = 1e-6;
    int64_t est_k = iters;
    double bfit = 0.0, brmse = 0.0;
    constexpr int CHUNK = 64;
    std::vector<lsm_icp_result> res(CHUNK);
    std::vector<Cloud *> vs(CHUNK, src), vt(CHUNK, tgt);
    std::vector<double> init(size_t(CHUNK) * 16), efit(static_cast<size_t>(iters)),
        ermse(static_cast<size_t>(iters));
    std::vector<char> done(size_t(iters), 0);
    for (int64_t it = 0; it < iters && it < est_k; ++it) {
        if (!valid[size_t(it)]) continue;
        if (!done[size_t(it)]) {
            // evaluate this and the next valid iterations below the current estimate at once
            std::vector<int64_t> batch;
            for (int64_t q = it; q < iters && q < est_k && int(batch.size()) < CHUNK; ++q)
                if (valid[size_t(q)] && !done[size_t(q)]) batch.push_back(q);
            for (size_t e = 0; e < batch.size(); ++e)
                std::memcpy(&init[16 * e], &hT[16 * size_t(batch[e])], 128);
            if ((rc = lsm_icp_run(ctx, int64_t(batch.size()), vs.data(), vt.data(), init.data(),
                                  ip, res.data())))
                return rc;
            for (size_t e = 0; e < batch.size(); ++e) {
                done[size_t(batch[e])] = 1;
                efit[size_t(batch[e])] = res[e].fitness;
                ermse[size_t(batch[e])] = res[e].inlier_rmse;
            }
        }
        ++*evaluated;
        const double fit = efit[size_t(it)], rm = ermse[size_t(it)];
        if (fit > bfit || (fit == bfit && rm < brmse)) {
            bfit = fit;
            brmse = rm;
            std::memcpy(T, &hT[16 * size_t(it)], 128);
            const double r = ratio[size_t(it)];
            if (r > 0.0) {
                const double k = r < 1.0 ? log(1.0 - confidence) / log(1.0 - r * r * r) : 0.0;
                if (k < double(est_k)) est_k = int64_t(ceil(k));
            }
        }
    }
    *fitness = bfit;
    *rmse = brmse;
    return LSM_OK;
}
