// loop.hip -- loop-closure candidate matching on the device (graphslam/loopclosing.py).
//
//   find_index_backwards          :223-237  per-segment lengths in parallel, then the reference's
//                                           sequential backwards accumulation (one lane: the f64
//                                           running sum must round exactly as the reference's)
//   find_candidates_within_radius :239-253  one lane per past pose, order-preserving compaction
//   look_for_valid_indexes        :131-144  one lane per sorted candidate j1: first j2 in
//                                           candidates[k:] with 1 < |j2-j1| < 80, 1 < d < 2
//
// Distances are bit-exact with NumPy: np.linalg.norm of a 1-D float64 3-vector evaluates
// sqrt(x.dot(x)) whose BLAS ddot tail is fma(z, z, fma(y, y, x*x)); the row-wise
// np.linalg.norm(..., axis=1) evaluates sqrt((x*x + y*y) + z*z) with separate roundings
// (tests/golden pins both).
#include <hip/hip_runtime.h>

#include <vector>

#include "lsm_ctx.h"

namespace {

__device__ __forceinline__ double norm_dot(double x, double y, double z) {
    return sqrt(fma(z, z, fma(y, y, lsm_dmul(x, x))));
}

__device__ __forceinline__ double norm_rows(double x, double y, double z) {
    return sqrt(lsm_dadd(lsm_dadd(lsm_dmul(x, x), lsm_dmul(y, y)), lsm_dmul(z, z)));
}

__global__ void segment_lengths(const double *P, int64_t m, double *seg) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k + 1 >= m) return;
    seg[k] = norm_dot(lsm_dsub(P[3 * (k + 1)], P[3 * k]), lsm_dsub(P[3 * (k + 1) + 1], P[3 * k + 1]),
                      lsm_dsub(P[3 * (k + 1) + 2], P[3 * k + 2]));
}

__global__ void walk_back(const double *seg, int64_t m, double dback, int64_t *index) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double d = 0.0;
    int64_t out = -1;
    for (int64_t i = m - 2; i >= 0; --i) {
        d = lsm_dadd(d, seg[i]);
        if (d > dback) {
            out = i;
            break;
        }
    }
    *index = out;
}

// one workgroup; ballot compaction keeps ascending order
__global__ void __launch_bounds__(1024)
within_radius(const double *P, int64_t m, const int64_t *index, double radius, int64_t *cand,
              int64_t *ncand) {
    __shared__ uint32_t wtot[16];
    __shared__ int64_t base_sh;
    const int64_t idx = *index;
    if (threadIdx.x == 0) base_sh = 0;
    __syncthreads();
    if (idx < 0) {
        if (threadIdx.x == 0) *ncand = 0;
        return;
    }
    const double cx = P[3 * (m - 1)], cy = P[3 * (m - 1) + 1], cz = P[3 * (m - 1) + 2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t s = 0; s < idx; s += blockDim.x) {
        const int64_t k = s + threadIdx.x;
        bool keep = false;
        if (k < idx) {
            const double d = norm_rows(lsm_dsub(P[3 * k], cx), lsm_dsub(P[3 * k + 1], cy),
                                       lsm_dsub(P[3 * k + 2], cz));
            keep = d < radius;
        }
        const uint64_t mk = __ballot(keep);
        if (lane == 0) wtot[w] = __popcll(mk);
        __syncthreads();
        int64_t off = base_sh;
        uint32_t tot = 0;
        for (int q = 0; q < int(blockDim.x >> 6); ++q) {
            off += (q < w) ? wtot[q] : 0;
            tot += wtot[q];
        }
        if (keep) cand[off + __popcll(mk & ((uint64_t(1) << lane) - 1))] = k;
        __syncthreads();
        if (threadIdx.x == 0) base_sh += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *ncand = base_sh;
}

__global__ void partners_kernel(const double *P, const int64_t *cand, int64_t n, int64_t *partner) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int64_t j1 = cand[k];
    int64_t out = -1;
    for (int64_t q = k; q < n; ++q) {
        const int64_t u = cand[q];
        const int64_t di = u > j1 ? u - j1 : j1 - u;
        if (!(di > 1 && di < 80)) continue;
        const double de = norm_dot(lsm_dsub(P[3 * j1], P[3 * u]), lsm_dsub(P[3 * j1 + 1], P[3 * u + 1]),
                                   lsm_dsub(P[3 * j1 + 2], P[3 * u + 2]));
        if (de > 1.0 && de < 2.0) {
            out = u;
            break;
        }
    }
    partner[k] = out;
}

}  // namespace

int lsm_loop_candidates_run(lsm_ctx *ctx, const double *positions, int64_t m, double dback,
                            double radius, int64_t *index_backwards, int64_t *cand, int64_t cap,
                            int64_t *ncand) {
    hipStream_t st = ctx->stream;
    *ncand = 0;
    *index_backwards = -1;
    if (m < 2) return LSM_OK;
    double *dP = (double *)ctx->buf("l_pos", size_t(m) * 24);
    double *dseg = (double *)ctx->buf("l_seg", size_t(m) * 8);
    int64_t *dcand = (int64_t *)ctx->buf("l_cand", size_t(m) * 8);
    int64_t *dsc = (int64_t *)ctx->buf("l_scalars", 32);
    if (!dP || !dseg || !dcand || !dsc) return LSM_ENOMEM;
    LSM_HIP_TRY(ctx, hipMemcpyAsync(dP, positions, size_t(m) * 24, hipMemcpyHostToDevice, st));
    segment_lengths<<<int((m + 255) / 256), 256, 0, st>>>(dP, m, dseg);
    walk_back<<<1, 64, 0, st>>>(dseg, m, dback, dsc);
    within_radius<<<1, 1024, 0, st>>>(dP, m, dsc, radius, dcand, dsc + 1);
    int64_t h[2];
    LSM_HIP_TRY(ctx, hipMemcpyAsync(h, dsc, 16, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    *index_backwards = h[0];
    *ncand = h[1];
    if (h[1] > 0 && cand) {
        if (cap < h[1]) {
            ctx->set_error("candidate buffer too small");
            return LSM_EINVAL;
        }
        LSM_HIP_TRY(ctx, hipMemcpyAsync(cand, dcand, size_t(h[1]) * 8, hipMemcpyDeviceToHost, st));
        LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    }
    LSM_HIP_TRY(ctx, hipGetLastError());
    return LSM_OK;
}

int lsm_loop_partners_run(lsm_ctx *ctx, const double *positions, int64_t m, const int64_t *cand,
                          int64_t ncand, int64_t *partner) {
    hipStream_t st = ctx->stream;
    double *dP = (double *)ctx->buf("l_pos", size_t(m) * 24);
    int64_t *dcand = (int64_t *)ctx->buf("l_cand", size_t(ncand) * 8);
    int64_t *dpart = (int64_t *)ctx->buf("l_part", size_t(ncand) * 8);
    if (!dP || !dcand || !dpart) return LSM_ENOMEM;
    LSM_HIP_TRY(ctx, hipMemcpyAsync(dP, positions, size_t(m) * 24, hipMemcpyHostToDevice, st));
    LSM_HIP_TRY(ctx, hipMemcpyAsync(dcand, cand, size_t(ncand) * 8, hipMemcpyHostToDevice, st));
    partners_kernel<<<int((ncand + 255) / 256), 256, 0, st>>>(dP, dcand, ncand, dpart);
    LSM_HIP_TRY(ctx, hipMemcpyAsync(partner, dpart, size_t(ncand) * 8, hipMemcpyDeviceToHost, st));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(st));
    LSM_HIP_TRY(ctx, hipGetLastError());
    return LSM_OK;
}
