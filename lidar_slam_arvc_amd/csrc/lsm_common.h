// lsm_common.h -- shared device/host structures of liblidarsm (gfx950 / CDNA4 only).
//
// Data layout in HBM:
//   * every processed keyframe cloud is stored cell-sorted: points float4 (x, y, z, 0) ordered
//     by the linear index of a uniform grid cell (z-major, then y, then x), so the 3 cells of a
//     grid row are ONE contiguous point range, and a workgroup of consecutive points covers a
//     compact patch of space (coherent queries when the cloud is an ICP source);
//   * a dense CSR cell table cell_start[ncells + 1] (u32) over the cloud's own bounding box, with
//     cells linearised BLOCKED: LSM_BLKX x LSM_BLKY x 4-cell blocks (x, y, z; 64 x 8 x 4 by
//     default) in z-major order, cells z-major inside a block. Cells are ANISOTROPIC: `cell` in x
//     and z, cell / LSM_YSUB in y (0.42 x 0.21 x 0.42 m by default; voxelised clouds
//     max(0.75, 2.5 voxel) in x / z), so a layout block is 26.9 x 1.68 x 1.68 m. A row of cells
//     inside a block is one contiguous, x-sorted point range (what the walks scan; its y width
//     sets how much of a ball's disc a walk covers), and a block's x-chunk of 4 cells in its
//     LSM_BLKY * 4 rows is a virtual block, a cube of edge 4 cells (1.68 m; the
//     coarse level the far-field search walks, with an occupancy bit each);
//   * normals float4 in the same order; perm[] maps sorted position -> reference (filter) order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#define LSM_WAVE 64

// Device descriptor of one processed cloud (POD; an array of these lives in device memory).
struct CloudDev {
    const float4 *xyz;          // n, cell-sorted
    const float4 *nrm;          // n or nullptr
    const uint32_t *cell_start; // ncells + 1, offsets into xyz
    const uint32_t *bmask;      // occupancy bit per virtual block (4 x LSM_BLKY x 4 cells; id (bz*nby + by)*nvbx + vbx,
                                //   nvbx = nbx * LSM_BLKX / 4; grid_fill)
    float ox, oy, oz;           // grid origin
    float cell, inv_cell;       // cell edge in x and z and its reciprocal
    float cell_y, inv_cell_y;   // cell edge in y (cell / LSM_YSUB) and its reciprocal
    int nx, ny, nz;             // cells per axis
    int nbx, nby, nbz;          // layout blocks per axis (LSM_BLKX, LSM_BLKY, 4 cells)
    int n;
    const uint32_t *perm;       // sorted position -> reference order
    const float4 *prior_ref;    // prior normals in reference order (orientation), or nullptr
    const double *xyz64;        // f64 coordinates in reference order (a voxelised cloud's f64
                                // centroids: what Open3D's cloud holds), or nullptr
};

#define LSM_XYZ_PAD 16     // spare float4 points allocated past every processed cloud's end
#define LSM_BLK 4          // cells per block edge in z (in y: LSM_BLKY)
#define LSM_BLK_SHIFT 2
// y cells are 1 / LSM_YSUB of the x / z cell edge (a walk covers
// its ball's disc in rows as wide as a y cell; 0 = cubic cells)
#ifndef LSM_YSUB_SHIFT
#define LSM_YSUB_SHIFT 1
#endif
#define LSM_YSUB (1 << LSM_YSUB_SHIFT)
#define LSM_BLKY_SHIFT (LSM_BLK_SHIFT + LSM_YSUB_SHIFT)
#define LSM_BLKY (1 << LSM_BLKY_SHIFT)   // cells per block edge in y (the block stays 4 cells tall)
// cells per block edge in x: 1 << LSM_BLKX_SHIFT (>= 2). A row of cells inside a block is one
// contiguous, x-sorted run, so wider blocks cut the rows the walks visit into fewer runs
// (64: C3 7670 -> 8561 pairs/s, profiles/r05o; the correspondence fallback keeps its own
// 4x4x4-cell virtual blocks, whatever the width).
#ifndef LSM_BLKX_SHIFT
#define LSM_BLKX_SHIFT 6
#endif
static_assert(LSM_BLKX_SHIFT >= 2 && LSM_BLKX_SHIFT <= 8, "x block width 4 .. 256 cells");
#define LSM_BLKX (1 << LSM_BLKX_SHIFT)
#define LSM_BLK_CELLS (LSM_BLKX * LSM_BLKY * LSM_BLK)
// a virtual block: 4 x-cells of a layout block's LSM_VB_ROWS rows (a cube of edge 4 * cell)
#define LSM_VB_ROWS (LSM_BLKY * LSM_BLK)
#define LSM_VB_CELLS (4 * LSM_VB_ROWS)

// blocked linear cell index (see layout note above): blocks z-major, then cells z-major inside
// a block, x fastest
__host__ __device__ __forceinline__ int lsm_cell_lin(int nbx, int nby, int x, int y, int z) {
    const int bx = x >> LSM_BLKX_SHIFT, by = y >> LSM_BLKY_SHIFT, bz = z >> LSM_BLK_SHIFT;
    return (((bz * nby + by) * nbx + bx) << (LSM_BLKX_SHIFT + LSM_BLKY_SHIFT + LSM_BLK_SHIFT)) |
           ((z & (LSM_BLK - 1)) << (LSM_BLKX_SHIFT + LSM_BLKY_SHIFT)) |
           ((y & (LSM_BLKY - 1)) << LSM_BLKX_SHIFT) | (x & (LSM_BLKX - 1));
}

// Per-pair ICP state (device). Layout kept 8-byte aligned.
struct PairState {
    double T[16];        // current transformation (row-major), f64 as Open3D
    double Tp[16];       // transformation of the previous correspondence pass (stability check)
    double fitness, rmse;
    double prev_fitness, prev_rmse;
    int32_t iter;        // updates applied
    int32_t active;      // 1 while the pair still runs correspondence passes
    int32_t ncorr;       // correspondences of the latest pass
    int32_t nsrc;        // source points (fitness denominator)
    int32_t src, tgt;    // indices into the CloudDev table of this batch
    int32_t blk0, nblk;  // first logical partial slot and number of source blocks
    int64_t src_off;     // offset of this pair's source points in the batch corr arrays
};

// Logical block -> (pair, first source point) for pair-indexed grids.
struct BlockTask {
    int32_t pair;   // -1 = padding (XCD balancing)
    int32_t start;  // first source point of this block
    int32_t slot;   // partial-sum slot (pair's blk0 + k)
    int32_t pad;
};

// Accumulator layout of the ICP reduction (f64): see icp.hip.
#define LSM_ACC 32

// ----------------------------------------------------------------------------------------------
// Host-side helpers
// ----------------------------------------------------------------------------------------------
#define LSM_HIP_TRY(ctx, expr)                                                          \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            (ctx)->set_error(std::string(#expr) + ": " + hipGetErrorString(_e));        \
            return LSM_EHIP;                                                            \
        }                                                                               \
    } while (0)

// Correctly rounded f64 operations that the compiler may NOT fuse into an FMA (hipcc contracts
// a * b + c by default, and HIP's __dmul_rn / __dadd_rn are plain operators): the bit-exact
// paths (filter mask, distances that decide neighbourhood membership, loop-closure norms)
// must round every product and sum separately, as NumPy / nanoflann do.
__device__ __forceinline__ double lsm_dmul(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ double lsm_dadd(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ double lsm_dsub(double a, double b) {
#pragma clang fp contract(off)
    return a - b;
}
__device__ __forceinline__ double lsm_ddiv(double a, double b) {
#pragma clang fp contract(off)
    return a / b;
}

// Exact nanoflann-style squared distance in f64 without contraction:
// ((dx*dx + dy*dy) + dz*dz), dx = q - p (L2_Adaptor::evalMetric order).
__device__ __forceinline__ double lsm_sqdist64(double qx, double qy, double qz, double px,
                                               double py, double pz) {
    double dx = lsm_dsub(qx, px), dy = lsm_dsub(qy, py), dz = lsm_dsub(qz, pz);
    return lsm_dadd(lsm_dadd(lsm_dmul(dx, dx), lsm_dmul(dy, dy)), lsm_dmul(dz, dz));
}

// Loads through a global-address-space view of a device pointer that was read from a
// descriptor (CloudDev, PairState tables): the compiler then emits global_load (counted by
// vmcnt only) instead of flat_load, whose lgkmcnt share serialises it with LDS traffic.
// (The host pass of hipcc only type-checks device code; it has no address spaces.)
template <typename T>
__device__ __forceinline__ T lsm_ld(const T *p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(1))) T *)p)[i];
#else
    return p[i];
#endif
}

__device__ __forceinline__ float4 lsm_ld(const float4 *p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4 v = ((const __attribute__((address_space(1))) v4 *)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return p[i];
#endif
}

// Point readers of the grid walks: plain global loads (64-bit addresses), or buffer loads
// through a descriptor of a cloud's points (a 32-bit offset per load; constant offsets of a load
// group fold into the instructions). pt(k): point k; x(k): its x coordinate.
struct GlobalPts {
    const float4 *xyz;
    __device__ __forceinline__ float4 pt(uint32_t k) const { return lsm_ld(xyz, k); }
    __device__ __forceinline__ float x(uint32_t k) const {
        return lsm_ld(reinterpret_cast<const float *>(xyz), size_t(k) * 4);
    }
};
struct BufPts {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ float4 pt(uint32_t k) const {
        typedef float v4 __attribute__((ext_vector_type(4)));
        const v4 v = __builtin_bit_cast(v4, __builtin_amdgcn_raw_buffer_load_b128(r, int(k * 16u), 0, 0));
        return make_float4(v.x, v.y, v.z, v.w);
    }
    __device__ __forceinline__ float x(uint32_t k) const {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, int(k * 16u), 0, 0));
    }
};
// the descriptor of cloud C's points (C must be wave-uniform), its range covering the
// LSM_XYZ_PAD spare points that prefetching walks may read
__device__ __forceinline__ BufPts cloud_buf_pts(const CloudDev &C) {
    return BufPts{__builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(C.xyz), 0,
                                                    (C.n + LSM_XYZ_PAD) * 16, 0x00020000)};
}

__device__ __forceinline__ int lsm_clampi(int v, int lo, int hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

// Wave-wide sum of a double (64 lanes, fixed tree -> deterministic).
__device__ __forceinline__ double lsm_wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, LSM_WAVE);
    return v;
}

// Kernel launchers implemented in the .hip translation units (all on `s`).
struct PrepBatch;  // defined in prep.hip
