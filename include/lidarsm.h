/*
 * lidarsm.h -- C ABI of liblidarsm.so, the MI355X (gfx950) ICP scan-matching hot path.
 *
 * This is the drop-in boundary for the reference's Open3D calls on the scan-matching path
 * (JudithV/LIDAR_SLAM_ARVC). The reference is pure Python; its operators are pybind11 calls
 * into Open3D. Each entry point below names the reference call site it replaces (file:line,
 * paths relative to the reference repository root). The Python package
 * `lidar_slam_arvc_amd` binds these with ctypes and keeps the reference's KeyFrame /
 * KeyFrameManager / LoopClosing method names (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Plain C types only; host arrays are caller-owned and copied during the call.
 *  - Point clouds live on the device behind opaque int64 handles (the keyframe cache).
 *  - Every function returns LSM_OK (0) or a negative LSM_E* code; lsm_last_error() gives text.
 *    Argument errors mirror Open3D's LogError cases (which raise RuntimeError in Python).
 *  - Degenerate inputs are NOT errors, as in Open3D: an empty correspondence set or a failed
 *    solve yields an identity update, fitness = inlier_rmse = 0.
 *  - Transforms are 4x4 row-major float64 (numpy's default layout of HomogeneousMatrix.array).
 *  - One context per GPU, used from one host thread. Calls are synchronous at return.
 */
#ifndef LIDARSM_H
#define LIDARSM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSM_OK 0
#define LSM_EINVAL (-1)   /* invalid argument (Open3D LogError equivalents) */
#define LSM_ENOMEM (-2)   /* device allocation failed */
#define LSM_EHIP (-3)     /* HIP runtime error */
#define LSM_ESTATE (-4)   /* object in the wrong state (e.g. P2Plane target without normals) */
#define LSM_ENODEV (-5)   /* no usable gfx950 device */

#define LSM_MAX_ITERATION (1 << 20) /* bound on lsm_icp_params.max_iteration (LSM_EINVAL above) */

#define LSM_P2P 0     /* TransformationEstimationPointToPoint  (keyframe.py:246-248) */
#define LSM_P2PLANE 1 /* TransformationEstimationPointToPlane  (keyframe.py:249-252) */

/* want_normals = LSM_NORMALS_LAZY: the same normals as want_normals = 1, computed per keyframe
 * when they are first used. A P2Plane registration computes all pending normals of its batch's
 * targets before its first pass, in one launch over those clouds; clouds that are never a
 * P2Plane target (loop-closure or multi-scale sources) never compute theirs. Any other use of
 * the normals (download, FPFH, plane split, voxel_down_sample with normals) completes them
 * first. The values are bit-identical to the eager estimate_normals (keyframe.py:160-162). */
#define LSM_NORMALS_LAZY 2

typedef struct lsm_ctx lsm_ctx;
typedef int64_t lsm_cloud;

/* Pre-processing parameters: KeyFrame.pre_process (keyframe.py:113-124).
 * filter_radius_height keyframe.py:74-94 (defaults from ICP_PARAMETERS, config/config.py:28-51);
 * voxel_down_sample keyframe.py:150-151 / :158-159 (voxel_size None -> voxel_size <= 0 here);
 * estimate_normals(KDTreeSearchParamHybrid(0.3, 300)) keyframe.py:160-162, radius from :33. */
typedef struct {
    double min_radius;     /* 0.5  : keep x^2+y^2 > min_radius^2 (strict); -inf: no lower bound */
    double max_radius;     /* 35   : keep x^2+y^2 < max_radius^2 (strict)  */
    double min_height;     /* -1.0 : keep z > min_height (strict)          */
    double max_height;     /* 50.0 : keep z < max_height (strict)          */
    double voxel_size;     /* <= 0: no down-sample                          */
    double normal_radius;  /* 0.3                                          */
    int32_t max_nn;        /* 300                                          */
    int32_t want_normals;  /* 1 for 'icppointplane', 0 for 'icppointpoint';
                            * LSM_NORMALS_LAZY: normals on demand (below)                  */
    double grid_cell;      /* spatial-grid cell edge in x and z, metres (y cells: half of it);
                            * <= 0 -> library default (0.42; voxelised clouds:
                            * max(0.75, 2.5 voxel_size)) */
} lsm_prep_params;

/* registration_icp(source, target, max_correspondence_distance, init, estimation, criteria)
 * keyframe.py:246-252 with Open3D's default ICPConvergenceCriteria. */
typedef struct {
    double max_correspondence_distance; /* ICP_PARAMETERS.distance_threshold = 10.0 */
    int32_t method;                      /* LSM_P2P | LSM_P2PLANE */
    int32_t max_iteration;               /* 30   */
    double relative_fitness;             /* 1e-6 */
    double relative_rmse;                /* 1e-6 */
} lsm_icp_params;

/* RegistrationResult (transformation, fitness, inlier_rmse, |correspondence_set|) plus the
 * number of ICP updates performed and a per-pair status (0 ok, <0 error code). */
typedef struct {
    double transformation[16];
    double fitness;
    double inlier_rmse;
    int64_t correspondences;
    int32_t iterations;
    int32_t status;
} lsm_icp_result;

/* Context ------------------------------------------------------------------------------ */
int lsm_init(int device, lsm_ctx **out);
int lsm_free(lsm_ctx *ctx);
const char *lsm_last_error(lsm_ctx *ctx);
const char *lsm_version(void);
void lsm_default_prep_params(lsm_prep_params *p);
void lsm_default_icp_params(lsm_icp_params *p);

/* Clouds -------------------------------------------------------------------------------- */
/* Replaces o3d.io.read_point_cloud's in-memory result (keyframe.py:41-45): N x 3 float32
 * row-major, the on-disk PCD precision; the reference widens to float64 exactly. */
int lsm_cloud_upload(lsm_ctx *ctx, const float *xyz, int64_t n, lsm_cloud *out);
/* Same from float64 (rounded to float32 on the device hot path). */
int lsm_cloud_upload_f64(lsm_ctx *ctx, const double *xyz, int64_t n, lsm_cloud *out);
/* `count` lsm_cloud_upload calls in one (the keyframes of a sequence, keyframemanager.py's
 * load of every keyframe before pre_process): xyz[i] holds n[i] x 3 float32, out[i] receives its
 * handle. One device allocation and one synchronisation for the batch (each cloud's points start
 * 256-byte aligned in it; the allocation is freed with the batch's last handle). On an error no
 * handle is created. */
int lsm_cloud_upload_batch(lsm_ctx *ctx, const float *const *xyz, const int64_t *n, int64_t count,
                           lsm_cloud *out);
/* A second handle on a device copy of src's raw points (no host round trip), for processing one
 * scan at several settings at once: the multi-scale chain of config C5
 * keeps one voxelised cloud per scale, where the reference would call voxel_down_sample on
 * copies of pointcloud (keyframe.py:150-151). */
int lsm_cloud_clone(lsm_ctx *ctx, lsm_cloud src, lsm_cloud *out);
/* KeyFrame.unload_pointcloud (keyframe.py:61-72): frees the device buffers of the handle. */
int lsm_cloud_release(lsm_ctx *ctx, lsm_cloud cloud);
/* n_raw: uploaded points; n_proc: points after pre-processing (0 before); has_normals. */
int lsm_cloud_info(lsm_ctx *ctx, lsm_cloud cloud, int64_t *n_raw, int64_t *n_proc,
                   int32_t *has_normals);

/* Pre-processing (KeyFrame.pre_process, keyframe.py:113-124) -------------------------------
 * Filters the raw cloud, optionally voxel-down-samples it, builds the cloud's spatial index and
 * (want_normals) estimates normals. Raw points stay resident, so it can be re-run.
 * n_out (nullable) receives the processed point count per cloud. */
int lsm_preprocess(lsm_ctx *ctx, lsm_cloud cloud, const lsm_prep_params *p, int64_t *n_out);
int lsm_preprocess_batch(lsm_ctx *ctx, int64_t n, const lsm_cloud *clouds,
                         const lsm_prep_params *p, int64_t *n_out);

/* pointcloud_filtered.points / .normals in the reference's order (filter order; for a voxelised
 * cloud: voxel-key order, Open3D's own order being unspecified). Either pointer may be NULL.
 * cap = rows available in the outputs. */
int lsm_cloud_download(lsm_ctx *ctx, lsm_cloud cloud, double *xyz, double *normals, int64_t cap);
/* Voxel keys (int32 x 3 per output point, Open3D voxel_index) of a voxelised cloud. */
int lsm_cloud_voxel_keys(lsm_ctx *ctx, lsm_cloud cloud, int32_t *keys, int64_t cap);
/* Diagnostics (no reference counterpart): the device layout of a processed cloud -- perm[i] =
 * reference-order index of sorted point i (cap >= n rows), and the cell table (cell_start, the
 * first sorted position of every blocked cell, ncells + 1 entries; cells may be NULL). *ncells
 * receives the number of cells. The tests compare the grid builds with it. */
int lsm_cloud_layout(lsm_ctx *ctx, lsm_cloud cloud, int32_t *perm, int64_t cap, uint32_t *cells,
                     int64_t cell_cap, int64_t *ncells);

/* Registration (KeyFrame.local_registration_simple, keyframe.py:231-260) --------------------
 * src = `other` (keyframe j), tgt = `self` (keyframe i); the result maps src into tgt frame. */
int lsm_icp(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, const double init[16],
            const lsm_icp_params *p, lsm_icp_result *out);
/* Many independent pairs in one device pass (scan-matcher chain run_scanmatcher.py:196-213,
 * loop-closure candidates loopclosing.py:80-99). init: npairs x 16 (NULL -> identity). */
int lsm_icp_batch(lsm_ctx *ctx, int64_t npairs, const lsm_cloud *src, const lsm_cloud *tgt,
                  const double *init, const lsm_icp_params *p, lsm_icp_result *out);
/* Correspondence set of the final pass of the most recent lsm_icp / pair 0 of lsm_icp_batch,
 * as (source index, target index) pairs in reference order. Returns the count in *n. */
int lsm_icp_last_correspondences(lsm_ctx *ctx, int64_t *pairs, int64_t cap, int64_t *n);

/* 'icp2planes' pre-processing --------------------------------------
 * KeyFrame.calculate_plane (keyframe.py:417-437): RANSAC plane (Open3D PointCloud.segment_plane
 * restated: ransac_n = 3, inliers |plane . (p, 1)| <= distance_threshold, best by count then
 * error / sqrt(count), probability-based early stop, least-squares refit of the winner's
 * inliers) over the processed cloud's points with z < height. The candidate samples come from
 * splitmix64(seed) (lsm_plane_samples; the reference's Open3D RNG is unseeded). Fails with
 * LSM_EINVAL when fewer than 3 points lie below `height` (Open3D's LogError). */
int lsm_ground_plane(lsm_ctx *ctx, lsm_cloud cloud, double height, double distance_threshold,
                     int64_t num_iterations, uint64_t seed, double probability, double plane[4],
                     int64_t *n_inliers, int64_t *n_subset);
/* The three distinct subset indices of every RANSAC candidate: out = num_iterations x 3. */
int lsm_plane_samples_get(uint64_t seed, int64_t n, int64_t num_iterations, int32_t *out);
/* KeyFrame.segment_plane (keyframe.py:439-461): |a x + b y + c z + d| / |(a, b, c)| < threshold
 * -> *ground, else -> *rest: two NEW raw clouds (reference order, as select_by_index) to be
 * pre-processed (normals) like uploads. */
int lsm_split_plane(lsm_ctx *ctx, lsm_cloud cloud, const double plane[4], double threshold,
                    lsm_cloud *ground, lsm_cloud *rest);

/* 'fpfh' global registration ----------------------------------------
 * compute_fpfh_feature(cloud, KDTreeSearchParamHybrid(radius, max_nn)) (keyframe.py:226-229):
 * FPFH of a pre-processed cloud with normals, kept on the device; `features` (nullable) receives
 * them, n x 33 f64 in reference order. */
/* The second voxel_down_sample of preprocess_fpfh with a voxel_size (keyframe.py:202-203):
 * [O3D] PointCloud::VoxelDownSample of a pre-processed cloud WITH normals -- the same voxel keys
 * and per-voxel point means as lsm_preprocess's voxel pass, computed from the cloud's
 * reference-order points (the f64 centroids of a voxelised cloud), and per voxel the sum of the
 * members' non-NaN normals divided by the member count (AccumulatedPoint::GetAverageNormal, not
 * re-normalised). *out is a NEW pre-processed cloud (voxel-key order) whose normals are those
 * averages; lsm_cloud_download returns its f64 centroids. LSM_EINVAL: voxel_size <= 0 / too
 * small (Open3D's LogError cases); LSM_ESTATE: cloud not pre-processed with normals. */
int lsm_voxel_down_sample_normals(lsm_ctx *ctx, lsm_cloud cloud, double voxel_size,
                                  lsm_cloud *out);
int lsm_fpfh(lsm_ctx *ctx, lsm_cloud cloud, double radius, int32_t max_nn, double *features,
             int64_t cap);
/* Feature.data of the features lsm_fpfh computed last (o3d.pipelines.registration.Feature, read
 * by keyframe.py:318-321 through registration_ransac_based_on_feature_matching): a download only,
 * n x 33 f64 in reference order; never recomputes. LSM_ESTATE when the cloud has none. */
int lsm_fpfh_download(lsm_ctx *ctx, lsm_cloud cloud, double *features, int64_t cap);
/* The feature matches of registration_ransac_based_on_feature_matching (keyframe.py:318-327):
 * every source feature's exact nearest target feature; with `mutual`, only the mutual pairs
 * unless fewer than 3 * ransac_n remain. corres: (source, target) index pairs (reference order),
 * *n = count. */
int lsm_feature_correspondences(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, int32_t mutual,
                                int32_t ransac_n, int32_t *corres, int64_t cap, int64_t *n);
/* RANSAC over the matches (ransac_n = 3, P2P without scaling, edge-length and distance
 * checkers, RANSACConvergenceCriteria(max_iteration, confidence)), sequential form with
 * splitmix64(seed) samples: the best transformation by (fitness, inlier_rmse) of one
 * correspondence pass within max_correspondence_distance; *evaluated = hypotheses scored. */
int lsm_ransac_feature(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, const int32_t *corres,
                       int64_t n, double max_correspondence_distance, double edge_similarity,
                       int64_t max_iteration, double confidence, uint64_t seed, double T[16],
                       double *fitness, double *inlier_rmse, int64_t *evaluated);

/* Loop-closure candidate matching (graphslam/loopclosing.py:102-144, :202-268) -------------
 * positions: m x 3 float64 trajectory (store_positions :202-211, last row = current pose).
 * index_backwards: find_index_backwards :223-237 (-1 for None).
 * candidates: find_candidates_within_radius :239-253, ascending. */
int lsm_loop_candidates(lsm_ctx *ctx, const double *positions, int64_t m,
                        double distance_backwards, double radius_threshold,
                        int64_t *index_backwards, int64_t *candidates, int64_t cap,
                        int64_t *n_candidates);
/* find_feasible_triplets :102-117 + look_for_valid_indexes :131-144 over sorted candidates:
 * partner[k] = j2 for candidate k, or -1. */
int lsm_loop_triplet_partners(lsm_ctx *ctx, const double *positions, int64_t m,
                              const int64_t *candidates, int64_t n_candidates, int64_t *partner);

/* Chain composition (artelib/homogeneousmatrix.py:184-205 compute_global_transformations, the
 * serial product run_scanmatcher.py:214-234 applies to the relative transforms) -------------
 * Host only (no device, no context): out[0] = identity, out[k + 1] = out[k] * rel[k], row-major
 * 4 x 4 f64, k = 0 .. n - 1 (out holds n + 1 matrices). */
int lsm_se3_prefix(const double *rel, int64_t n, double *out);

/* Instrumentation ------------------------------------------------------------------------
 * With timing on, the library brackets every launch of the named kernel with HIP events on its
 * own stream and accumulates the durations. Kernel names:
 *   "filter", "voxel", "grid"          pre-processing (filter_radius_height, voxel_down_sample,
 *                                      the cell-sorted layout)
 *   "normals"                          estimate_normals in the pre-process (the split launch)
 *   "normals_lazy"                     LSM_NORMALS_LAZY clouds' normals, computed by a P2Plane
 *                                      registration or another first use
 *   "normals_refine"                   the normals' refine kernel (both of the above), timed on
 *                                      the side stream it runs on, overlapping the next ICP
 *   "nn", "nn_fallback"               the correspondence search and its fallback, per pass
 *   "accumulate", "solve"              the JtJ / moment sums and the per-pair solve, per pass
 *   "plane", "ransac", "fpfh", "feature_nn"   icp2planes and fpfh
 * Aggregates: "nn_pass" (launches = correspondence passes; ms = "nn" + "nn_fallback" of those
 * passes; algo_bytes = their SURVEY.md §8d bytes), and the counters "nn_queries",
 * "nn_queries_first_pass", "nn_uncertified", "nn_pending", "nn_pending_first_pass" (counts in
 * `launches`). algo_bytes: algorithmic bytes moved (SURVEY.md §8d model; "nn" and "nn_pass").
 * enable = 2 (statistics mode, slower): also count the neighbours of every normal computed
 * ("normals_neighbours", "normals_points" and "normals_truncated" in `launches`). */
int lsm_set_timing(lsm_ctx *ctx, int32_t enable);
int lsm_kernel_stats(lsm_ctx *ctx, const char *kernel, int64_t *launches, double *total_ms,
                     double *algo_bytes);
int lsm_reset_stats(lsm_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
