// lsm_ctx.h -- host-side context of liblidarsm: device buffers, clouds, instrumentation.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lidarsm.h"
#include "lsm_common.h"

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// One keyframe cloud resident on the device (the keyframe cache, SURVEY.md §8b "Ownership").
struct Cloud {
    int64_t n_raw = 0;
    float *d_raw = nullptr;       // n_raw x 3 float32 (as uploaded, reference order)
    std::shared_ptr<void> raw_slab;   // lsm_cloud_upload_batch: the batch's allocation d_raw
                                      // points into (freed with its last cloud), else null
    int64_t cap = 0;              // capacity of the processed arrays (points)
    int64_t n = 0;                // processed points
    float4 *d_xyz = nullptr;      // cell-sorted points
    float4 *d_nrm = nullptr;      // cell-sorted normals
    uint32_t *d_perm = nullptr;   // sorted position -> reference-order index
    uint32_t *d_cell = nullptr;   // cell_start table
    int64_t cell_cap = 0;
    uint32_t *d_bmask = nullptr;  // block occupancy bits (the fallback's empty-block test)
    int64_t bmask_cap = 0;        // words
    double *d_vox = nullptr;      // voxel centroids (f64, voxel-key order), voxelised clouds only
    int32_t *d_vkeys = nullptr;   // voxel keys (int32 x 3)
    int64_t vox_cap = 0;
    double *d_fpfh = nullptr;     // FPFH features, n x 33, reference order
    int64_t fpfh_cap = 0, fpfh_n = 0;
    float4 *d_prior_ref = nullptr; // prior normals (reference order) of a split cloud
    int64_t prior_n = 0;
    bool lazy = false;            // normals of some points still pending (computed on demand)
    double lazy_radius = 0.3;     // the KDTreeSearchParamHybrid of the pending normals
    int lazy_max_nn = 300;
    bool processed = false;
    bool has_normals = false;
    bool voxelized = false;
    int64_t nonempty_cells = 0;
    CloudDev dev{};               // host copy of the device descriptor
};

struct KStat {
    int64_t launches = 0;
    double ms = 0.0;
    double algo_bytes = 0.0;
};

struct lsm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // the normals' refine kernel (a handful of long single-lane scans) runs on `side`, so the
    // next ICP's first correspondence pass (which reads no normals) overlaps it; side_ev marks its
    // end. Every entry point but the ICP waits for it (join_side); the ICP waits on the device
    // before its first accumulation (join_side_device).
    // Invariant: the refine reads its launch's CloudDev / GridGeo tables and the normals' list
    // buffers; every writer of those (prep.hip's upload_vec, run_normals) joins first. A new entry
    // point that writes them without going through find_cloud (a host join) or upload_vec must
    // call join_side_device() before its first write.
    hipStream_t side = nullptr;
    hipEvent_t side_ev = nullptr;
    bool side_pending = false;
    void join_side();
    void join_side_device();
    std::string err;
    std::unordered_map<int64_t, Cloud *> clouds;
    int64_t next_id = 1;
    std::map<std::string, DevBuf> scratch;
    void *pinned = nullptr;       // small pinned staging area for counters
    size_t pinned_bytes = 0;
    int num_cus = 256;

    // instrumentation
    bool timing = false;
    bool statistics = false;      // lsm_set_timing(ctx, 2): also count the normals' neighbours
    std::map<std::string, KStat> stats;
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;

    // last correspondence set (reference order) of pair 0 of the last ICP call: the ICP leaves
    // a dense per-source-point array (target reference index or -1, indexed by the source's
    // reference index) in the scratch buffer "i_lastcorr_dense"; it is compacted into
    // last_corr only when asked for (lsm_icp_last_correspondences)
    std::vector<int64_t> last_corr;
    int64_t last_corr_dense_n = 0;
    bool last_corr_pending = false;

    void set_error(const std::string &e) { err = e; }
    // grow-only named scratch buffer
    void *buf(const std::string &name, size_t bytes);
    void *host_pinned(size_t bytes);
    void *host_pinned_extra(size_t bytes);   // a second, fixed 4 KiB pinned area
    void *pinned2 = nullptr;
    // grow-only host tables (the launches' workgroup -> (cloud, first point) lists), kept so a
    // call does not fault in a fresh multi-MB vector (≈ 10 ms of host time per C3 step)
    std::map<std::string, std::vector<uint64_t>> host_tables;
    hipEvent_t get_event();
    // bracket a launch with events when timing is on
    void tic(const char *name, hipEvent_t *a, hipStream_t on = nullptr);
    void toc(const char *name, hipEvent_t a, hipStream_t on = nullptr);
    void collect_timings();   // call after the stream is synchronised
};

// ------------------------------------------------------------------------------------------
// Internal entry points (implemented per translation unit)
// ------------------------------------------------------------------------------------------
int lsm_prep_batch(lsm_ctx *ctx, std::vector<Cloud *> &clouds, const lsm_prep_params &p,
                   int64_t *n_out);
int lsm_icp_run(lsm_ctx *ctx, int64_t npairs, Cloud **src, Cloud **tgt, const double *init,
                const lsm_icp_params &p, lsm_icp_result *out);
int lsm_loop_candidates_run(lsm_ctx *ctx, const double *positions, int64_t m, double dback,
                            double radius, int64_t *index_backwards, int64_t *cand, int64_t cap,
                            int64_t *ncand);
int lsm_loop_partners_run(lsm_ctx *ctx, const double *positions, int64_t m,
                          const int64_t *cand, int64_t ncand, int64_t *partner);
int lsm_download_run(lsm_ctx *ctx, Cloud *c, double *xyz, double *nrm, int64_t cap);
// test knob `name` (api.cpp's list; environment, read per call) or dflt
double lsm_knob(const char *name, double dflt);
// lazy normals: compute every pending normal of the clouds (any use other than the ICP's)
int lsm_normals_complete(lsm_ctx *ctx, std::vector<Cloud *> &clouds);
int lsm_ground_plane_run(lsm_ctx *ctx, Cloud *c, double height, double thr, int64_t iters,
                         uint64_t seed, double probability, double plane[4], int64_t *n_inliers,
                         int64_t *n_subset);
int lsm_split_plane_run(lsm_ctx *ctx, Cloud *c, const double plane[4], double thr, Cloud *g,
                        Cloud *r);
void lsm_plane_samples(uint64_t seed, int64_t n, int64_t iters, int32_t *out);
int lsm_fpfh_run(lsm_ctx *ctx, Cloud *c, double radius, int max_nn);
int lsm_voxel_normals_run(lsm_ctx *ctx, Cloud *c, double v, Cloud *o);
int lsm_feature_corr_run(lsm_ctx *ctx, Cloud *s, Cloud *t, int mutual, int ransac_n,
                         int32_t *out, int64_t cap, int64_t *n_out);
int lsm_ransac_run(lsm_ctx *ctx, Cloud *src, Cloud *tgt, const int32_t *corr, int64_t ncorr,
                   double max_corr, double edge, int64_t iters, double confidence, uint64_t seed,
                   double T[16], double *fitness, double *rmse, int64_t *evaluated);
