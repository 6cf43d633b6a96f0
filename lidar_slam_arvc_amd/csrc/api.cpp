// api.cpp -- the extern "C" boundary of liblidarsm (include/lidarsm.h).
//
// Thin validation + bookkeeping layer: argument errors are reported the way Open3D reports them
// (LogError -> RuntimeError in the reference's Python), device work lives in prep.hip / icp.hip
// / loop.hip. There is no CPU fallback: without a gfx950 device lsm_init fails.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lsm_ctx.h"

static const char *kVersion = "liblidarsm 0.1 (gfx950)";

// Test knobs: the search-path variants the GPU tests switch (through the environment, read per
// call) to prove every path exact; the defaults are the shipped values. DESIGN.md §7 lists them
// with the tests that cover each. No other environment variable changes the library's results
// (diagnostics builds, -DLSM_DIAG, add statistics printers).
static const char *const kKnobs[] = {
    "LSM_NN_SPLIT",  "LSM_NN_SPLIT_PLACE", "LSM_NN_NOCERT", "LSM_NN_CERT_FROM",  "LSM_NN_DIRECT",
    "LSM_NN_DIRECT_ITER", "LSM_NN_KCOLD", "LSM_NN_KMAX",   "LSM_NN_COLD_SEED",  "LSM_NORMALS_EXACT",
    "LSM_NORMALS_SPLIT", "LSM_NORMALS_SIDE", "LSM_NN_TILE", "LSM_NN_FULL_L", "LSM_FB_GL", "LSM_FB_WAVES", "LSM_FB_WIDE_FROM", "LSM_FB_FAR", "LSM_FB_WIDE_MAX", "LSM_FB_WIDE_MAXC"};

double lsm_knob(const char *name, double dflt) {
    bool known = false;
    for (const char *k : kKnobs) known = known || std::strcmp(k, name) == 0;
    if (!known) return dflt;
    const char *e = std::getenv(name);
    return e && *e ? std::atof(e) : dflt;
}

// ------------------------------------------------------------------------------------------
// lsm_ctx helpers
// ------------------------------------------------------------------------------------------
void *lsm_ctx::buf(const std::string &name, size_t bytes) {
    DevBuf &b = scratch[name];
    if (bytes == 0) bytes = 16;
    if (b.bytes < bytes) {
        if (b.p) {
            if (side) (void)hipStreamSynchronize(side);
            (void)hipStreamSynchronize(stream);
            (void)hipFree(b.p);
            b.p = nullptr;
            b.bytes = 0;
        }
        size_t want = bytes + bytes / 4;
        if (hipMalloc(&b.p, want) != hipSuccess) {
            b.p = nullptr;
            return nullptr;
        }
        b.bytes = want;
    }
    return b.p;
}

void *lsm_ctx::host_pinned(size_t bytes) {
    if (pinned_bytes < bytes) {
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
        pinned_bytes = 0;
        size_t want = bytes < 4096 ? 4096 : bytes * 2;
        if (hipHostMalloc(&pinned, want, hipHostMallocDefault) != hipSuccess) return nullptr;
        pinned_bytes = want;
    }
    return pinned;
}

void *lsm_ctx::host_pinned_extra(size_t bytes) {
    if (bytes > 4096) return nullptr;
    if (!pinned2 && hipHostMalloc(&pinned2, 4096, hipHostMallocDefault) != hipSuccess) {
        pinned2 = nullptr;
        return nullptr;
    }
    return pinned2;
}

hipEvent_t lsm_ctx::get_event() {
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void lsm_ctx::tic(const char *name, hipEvent_t *a, hipStream_t on) {
    (void)name;
    *a = nullptr;
    if (!timing) return;
    *a = get_event();
    (void)hipEventRecord(*a, on ? on : stream);
}

void lsm_ctx::toc(const char *name, hipEvent_t a, hipStream_t on) {
    if (!timing || !a) return;
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, on ? on : stream);
    pending.push_back({name, a, b});
}

void lsm_ctx::collect_timings() {
    std::vector<Pending> later;   // (side-stream brackets still running: the next collection)
    for (auto &pe : pending) {
        if (hipEventQuery(pe.b) == hipErrorNotReady) {
            later.push_back(pe);
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            KStat &s = stats[pe.name];
            s.launches += 1;
            s.ms += ms;
        }
        event_pool.push_back(pe.a);
        event_pool.push_back(pe.b);
    }
    pending.swap(later);
}

void lsm_ctx::join_side() {
    if (!side_pending) return;
    (void)hipStreamSynchronize(side);
    side_pending = false;
}

void lsm_ctx::join_side_device() {
    if (!side_pending) return;
    (void)hipStreamWaitEvent(stream, side_ev, 0);
    side_pending = false;
}

// the entry points' cloud lookup: first the normals' side-stream work completes (join_side)
static Cloud *find_cloud_nojoin(lsm_ctx *ctx, lsm_cloud id) {
    auto it = ctx->clouds.find(id);
    return it == ctx->clouds.end() ? nullptr : it->second;
}

static Cloud *find_cloud(lsm_ctx *ctx, lsm_cloud id) {
    ctx->join_side();
    return find_cloud_nojoin(ctx, id);
}

static void free_cloud(Cloud *c) {
    if (c->raw_slab)
        c->raw_slab.reset();   // a batch upload's slice: the batch's allocation goes with its last cloud
    else
        (void)hipFree(c->d_raw);
    (void)hipFree(c->d_xyz);
    (void)hipFree(c->d_nrm);
    (void)hipFree(c->d_perm);
    (void)hipFree(c->d_cell);
    (void)hipFree(c->d_bmask);
    (void)hipFree(c->d_vox);
    (void)hipFree(c->d_vkeys);
    (void)hipFree(c->d_prior_ref);
    (void)hipFree(c->d_fpfh);
    delete c;
}

// lazy normals (LSM_NORMALS_LAZY): every use of a cloud's normals other than a P2Plane
// registration completes the pending ones first
static int complete_normals(lsm_ctx *ctx, Cloud *c) {
    if (!c->lazy) return LSM_OK;
    std::vector<Cloud *> one{c};
    const int rc = lsm_normals_complete(ctx, one);
    ctx->join_side_device();   // the caller's next work on the stream reads the normals
    return rc;
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

const char *lsm_version(void) { return kVersion; }

void lsm_default_prep_params(lsm_prep_params *p) {
    if (!p) return;
    p->min_radius = 0.5;      // icp_parameters.yaml filter_by_radius.min_radius
    p->max_radius = 35.0;     // icp_parameters.yaml filter_by_radius.max_radius
    p->min_height = -1.0;     // icp_parameters.yaml filter_by_height.min_height
    p->max_height = 50.0;     // icp_parameters.yaml filter_by_height.max_height
    p->voxel_size = 0.0;      // down_sample.voxel_size: null
    p->normal_radius = 0.3;   // keyframe.py:33
    p->max_nn = 300;          // normals.maximum_neighbors
    p->want_normals = 1;      // method 'icppointplane' (keyframemanager.py:9)
    p->grid_cell = 0.0;
}

void lsm_default_icp_params(lsm_icp_params *p) {
    if (!p) return;
    p->max_correspondence_distance = 10.0;  // icp.distance_threshold
    p->method = LSM_P2PLANE;
    p->max_iteration = 30;                  // Open3D ICPConvergenceCriteria defaults
    p->relative_fitness = 1e-6;
    p->relative_rmse = 1e-6;
}

int lsm_init(int device, lsm_ctx **out) {
    if (!out) return LSM_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LSM_ENODEV;
    if (device < 0 || device >= ndev) return LSM_EINVAL;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return LSM_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LSM_ENODEV;
    if (hipSetDevice(device) != hipSuccess) return LSM_EHIP;
    lsm_ctx *ctx = new lsm_ctx();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return LSM_EHIP;
    }
    *out = ctx;
    return LSM_OK;
}

int lsm_free(lsm_ctx *ctx) {
    if (!ctx) return LSM_EINVAL;
    (void)hipSetDevice(ctx->device);
    ctx->join_side();
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &kv : ctx->clouds) free_cloud(kv.second);
    for (auto &kv : ctx->scratch) (void)hipFree(kv.second.p);
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    for (auto &pe : ctx->pending) {
        (void)hipEventDestroy(pe.a);
        (void)hipEventDestroy(pe.b);
    }
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->pinned2) (void)hipHostFree(ctx->pinned2);
    if (ctx->side_ev) (void)hipEventDestroy(ctx->side_ev);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return LSM_OK;
}

const char *lsm_last_error(lsm_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static int upload_common(lsm_ctx *ctx, const void *xyz, int64_t n, bool f64, lsm_cloud *out) {
    if (!ctx || !out || n < 0 || (n > 0 && !xyz)) return LSM_EINVAL;
    if (n >= (int64_t(1) << 31)) {
        ctx->set_error("cloud too large (>= 2^31 points)");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    Cloud *c = new Cloud();
    c->n_raw = n;
    size_t bytes = size_t(n > 0 ? n : 1) * 3 * sizeof(float);
    if (hipMalloc(&c->d_raw, bytes) != hipSuccess) {
        delete c;
        ctx->set_error("hipMalloc failed for raw cloud");
        return LSM_ENOMEM;
    }
    // every early return below frees the cloud (no leak of the handle-less allocation)
    auto fail = [&](hipError_t e, const char *what) {
        ctx->set_error(std::string(what) + ": " + hipGetErrorString(e));
        free_cloud(c);
        return LSM_EHIP;
    };
    hipError_t e = hipSuccess;
    if (n > 0) {
        if (!f64) {
            e = hipMemcpyAsync(c->d_raw, xyz, size_t(n) * 12, hipMemcpyHostToDevice, ctx->stream);
            if (e != hipSuccess) return fail(e, "hipMemcpyAsync (upload)");
        } else {
            std::vector<float> tmp(size_t(n) * 3);
            const double *d = static_cast<const double *>(xyz);
            for (size_t i = 0; i < tmp.size(); ++i) tmp[i] = float(d[i]);
            e = hipMemcpyAsync(c->d_raw, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice,
                               ctx->stream);
            if (e != hipSuccess) return fail(e, "hipMemcpyAsync (upload)");
            e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) return fail(e, "hipStreamSynchronize (upload)");
        }
    }
    e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return fail(e, "hipStreamSynchronize (upload)");
    int64_t id = ctx->next_id++;
    ctx->clouds[id] = c;
    *out = id;
    return LSM_OK;
}

int lsm_cloud_upload(lsm_ctx *ctx, const float *xyz, int64_t n, lsm_cloud *out) {
    return upload_common(ctx, xyz, n, false, out);
}

int lsm_cloud_upload_f64(lsm_ctx *ctx, const double *xyz, int64_t n, lsm_cloud *out) {
    return upload_common(ctx, xyz, n, true, out);
}

// Per-call costs dominate uploading many small scans one by one (an allocation, a copy and a
// synchronisation each: ≈ 39 us per HDL-64 scan on top of the copy), so a batch
// takes one allocation and one synchronisation, its copies queued back to back on the stream.
int lsm_cloud_upload_batch(lsm_ctx *ctx, const float *const *xyz, const int64_t *n, int64_t count,
                           lsm_cloud *out) {
    if (!ctx || count < 0 || (count > 0 && (!xyz || !n || !out))) return LSM_EINVAL;
    std::vector<size_t> off(static_cast<size_t>(count));
    size_t total = 0;
    for (int64_t i = 0; i < count; ++i) {
        if (n[i] < 0 || (n[i] > 0 && !xyz[i])) return LSM_EINVAL;
        if (n[i] >= (int64_t(1) << 31)) {
            ctx->set_error("cloud too large (>= 2^31 points)");
            return LSM_EINVAL;
        }
        off[size_t(i)] = total;
        total += (size_t(n[i] > 0 ? n[i] : 1) * 12 + 255) / 256 * 256;
    }
    if (count == 0) return LSM_OK;
    (void)hipSetDevice(ctx->device);
    void *slab = nullptr;
    if (hipMalloc(&slab, total) != hipSuccess) {
        ctx->set_error("hipMalloc failed for a batch of raw clouds");
        return LSM_ENOMEM;
    }
    std::shared_ptr<void> keep(slab, [](void *p) { (void)hipFree(p); });
    char *base = static_cast<char *>(slab);
    hipError_t e = hipSuccess;
    for (int64_t i = 0; i < count && e == hipSuccess; ++i)
        if (n[i] > 0)
            e = hipMemcpyAsync(base + off[size_t(i)], xyz[i], size_t(n[i]) * 12,
                               hipMemcpyHostToDevice, ctx->stream);
    const hipError_t es = hipStreamSynchronize(ctx->stream);   // (also before a failed batch's free)
    if (e == hipSuccess) e = es;
    if (e != hipSuccess) {
        ctx->set_error(std::string("lsm_cloud_upload_batch: ") + hipGetErrorString(e));
        return LSM_EHIP;
    }
    for (int64_t i = 0; i < count; ++i) {
        Cloud *c = new Cloud();
        c->n_raw = n[i];
        c->d_raw = reinterpret_cast<float *>(base + off[size_t(i)]);
        c->raw_slab = keep;
        const int64_t id = ctx->next_id++;
        ctx->clouds[id] = c;
        out[i] = id;
    }
    return LSM_OK;
}

int lsm_cloud_clone(lsm_ctx *ctx, lsm_cloud src, lsm_cloud *out) {
    if (!ctx || !out) return LSM_EINVAL;
    Cloud *s = find_cloud(ctx, src);
    if (!s) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    Cloud *c = new Cloud();
    c->n_raw = s->n_raw;
    const size_t bytes = size_t(s->n_raw > 0 ? s->n_raw : 1) * 3 * sizeof(float);
    if (hipMalloc(&c->d_raw, bytes) != hipSuccess) {
        delete c;
        ctx->set_error("hipMalloc failed for raw cloud");
        return LSM_ENOMEM;
    }
    hipError_t e = hipSuccess;
    if (s->n_raw > 0)
        e = hipMemcpyAsync(c->d_raw, s->d_raw, size_t(s->n_raw) * 12, hipMemcpyDeviceToDevice,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        ctx->set_error(std::string("lsm_cloud_clone: ") + hipGetErrorString(e));
        free_cloud(c);
        return LSM_EHIP;
    }
    const int64_t id = ctx->next_id++;
    ctx->clouds[id] = c;
    *out = id;
    return LSM_OK;
}

int lsm_ground_plane(lsm_ctx *ctx, lsm_cloud cloud, double height, double distance_threshold,
                     int64_t num_iterations, uint64_t seed, double probability, double plane[4],
                     int64_t *n_inliers, int64_t *n_subset) {
    if (!ctx || !plane) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed) {
        ctx->set_error("cloud not pre-processed");
        return LSM_ESTATE;
    }
    if (!(probability > 0.0 && probability <= 1.0)) {
        ctx->set_error("Probability must be > 0 or <= 1.0");
        return LSM_EINVAL;
    }
    if (num_iterations < 1 || num_iterations > (int64_t(1) << 24) || !(distance_threshold >= 0)) {
        ctx->set_error("invalid RANSAC parameters");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    return lsm_ground_plane_run(ctx, c, height, distance_threshold, num_iterations, seed,
                                probability, plane, n_inliers, n_subset);
}

int lsm_plane_samples_get(uint64_t seed, int64_t n, int64_t num_iterations, int32_t *out) {
    if (n < 3 || num_iterations < 0 || (num_iterations > 0 && !out)) return LSM_EINVAL;
    lsm_plane_samples(seed, n, num_iterations, out);
    return LSM_OK;
}

// lsm_se3_prefix: se3_host.cpp (host-only code, also built under ASan/UBSan by tests/asan)

int lsm_split_plane(lsm_ctx *ctx, lsm_cloud cloud, const double plane[4], double threshold,
                    lsm_cloud *ground, lsm_cloud *rest) {
    if (!ctx || !plane || !ground || !rest) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed) {
        ctx->set_error("cloud not pre-processed");
        return LSM_ESTATE;
    }
    (void)hipSetDevice(ctx->device);
    int rc0 = complete_normals(ctx, c);
    if (rc0) return rc0;
    Cloud *g = new Cloud(), *r = new Cloud();
    const int rc = lsm_split_plane_run(ctx, c, plane, threshold, g, r);
    if (rc != LSM_OK) {
        free_cloud(g);
        free_cloud(r);
        return rc;
    }
    const int64_t ig = ctx->next_id++, ir = ctx->next_id++;
    ctx->clouds[ig] = g;
    ctx->clouds[ir] = r;
    *ground = ig;
    *rest = ir;
    return LSM_OK;
}

int lsm_voxel_down_sample_normals(lsm_ctx *ctx, lsm_cloud cloud, double voxel_size,
                                  lsm_cloud *out) {
    if (!ctx || !out) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed || !c->has_normals) {
        ctx->set_error("voxel_down_sample with normals needs a pre-processed cloud with normals");
        return LSM_ESTATE;
    }
    (void)hipSetDevice(ctx->device);
    int rc0 = complete_normals(ctx, c);
    if (rc0) return rc0;
    Cloud *o = new Cloud();
    const int rc = lsm_voxel_normals_run(ctx, c, voxel_size, o);
    if (rc != LSM_OK) {
        free_cloud(o);
        return rc;
    }
    const int64_t id = ctx->next_id++;
    ctx->clouds[id] = o;
    *out = id;
    return LSM_OK;
}

int lsm_fpfh(lsm_ctx *ctx, lsm_cloud cloud, double radius, int32_t max_nn, double *features,
             int64_t cap) {
    if (!ctx) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed || !c->has_normals) {
        ctx->set_error("ComputeFPFHFeature needs a cloud with normals (pre-process with normals)");
        return LSM_ESTATE;
    }
    if (!(radius > 0) || max_nn < 1) {
        ctx->set_error("Invalid KDTreeSearchParamHybrid (radius <= 0 or max_nn < 1)");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    int rc = complete_normals(ctx, c);
    if (rc) return rc;
    rc = lsm_fpfh_run(ctx, c, radius, max_nn);
    if (rc) return rc;
    if (features && c->n > 0) {
        LSM_HIP_TRY(ctx, hipMemcpy(features, c->d_fpfh, size_t(std::min<int64_t>(cap, c->n)) * 33 * 8,
                                   hipMemcpyDeviceToHost));
    }
    return LSM_OK;
}

int lsm_fpfh_download(lsm_ctx *ctx, lsm_cloud cloud, double *features, int64_t cap) {
    if (!ctx || (cap > 0 && !features) || cap < 0) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->d_fpfh || c->fpfh_n != c->n) {
        ctx->set_error("the cloud has no FPFH features (lsm_fpfh first)");
        return LSM_ESTATE;
    }
    if (cap < c->n) {
        ctx->set_error("output capacity smaller than the feature count");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    if (c->n > 0)
        LSM_HIP_TRY(ctx, hipMemcpy(features, c->d_fpfh, size_t(c->n) * 33 * 8, hipMemcpyDeviceToHost));
    return LSM_OK;
}

int lsm_feature_correspondences(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, int32_t mutual,
                                int32_t ransac_n, int32_t *corres, int64_t cap, int64_t *n) {
    if (!ctx || !n) return LSM_EINVAL;
    Cloud *s = find_cloud(ctx, src), *t = find_cloud(ctx, tgt);
    if (!s || !t) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!s->d_fpfh || !t->d_fpfh || s->fpfh_n != s->n || t->fpfh_n != t->n) {
        ctx->set_error("compute the FPFH features of both clouds first (lsm_fpfh)");
        return LSM_ESTATE;
    }
    (void)hipSetDevice(ctx->device);
    return lsm_feature_corr_run(ctx, s, t, mutual, ransac_n, corres, cap, n);
}

int lsm_ransac_feature(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, const int32_t *corres,
                       int64_t n, double max_correspondence_distance, double edge_similarity,
                       int64_t max_iteration, double confidence, uint64_t seed, double T[16],
                       double *fitness, double *inlier_rmse, int64_t *evaluated) {
    if (!ctx || !T || !fitness || !inlier_rmse || !evaluated || (n > 0 && !corres)) return LSM_EINVAL;
    Cloud *s = find_cloud(ctx, src), *t = find_cloud(ctx, tgt);
    if (!s || !t) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!s->processed || !t->processed) {
        ctx->set_error("clouds not pre-processed");
        return LSM_ESTATE;
    }
    if (!(max_correspondence_distance > 0) || max_iteration < 0 || max_iteration > (int64_t(1) << 24) ||
        !(confidence > 0 && confidence < 1)) {
        ctx->set_error("invalid RANSAC parameters");
        return LSM_EINVAL;
    }
    for (int64_t k = 0; k < n; ++k)
        if (corres[2 * k] < 0 || corres[2 * k] >= s->n || corres[2 * k + 1] < 0 ||
            corres[2 * k + 1] >= t->n) {
            ctx->set_error("correspondence index out of range");
            return LSM_EINVAL;
        }
    (void)hipSetDevice(ctx->device);
    return lsm_ransac_run(ctx, s, t, corres, n, max_correspondence_distance, edge_similarity,
                          max_iteration, confidence, seed, T, fitness, inlier_rmse, evaluated);
}

int lsm_cloud_release(lsm_ctx *ctx, lsm_cloud cloud) {
    if (!ctx) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    free_cloud(c);
    ctx->clouds.erase(cloud);
    return LSM_OK;
}

int lsm_cloud_info(lsm_ctx *ctx, lsm_cloud cloud, int64_t *n_raw, int64_t *n_proc,
                   int32_t *has_normals) {
    if (!ctx) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (n_raw) *n_raw = c->n_raw;
    if (n_proc) *n_proc = c->processed ? c->n : 0;
    if (has_normals) *has_normals = c->has_normals ? 1 : 0;
    return LSM_OK;
}

static int check_prep(lsm_ctx *ctx, const lsm_prep_params *p) {
    if (!p) return LSM_EINVAL;
    if (!(p->max_radius > 0) || !std::isfinite(p->max_radius) || !std::isfinite(p->min_height) ||
        !std::isfinite(p->max_height)) {
        ctx->set_error("filter bounds must be finite (max_radius > 0)");
        return LSM_EINVAL;
    }
    if (p->want_normals < 0 || p->want_normals > LSM_NORMALS_LAZY) {
        ctx->set_error("want_normals must be 0, 1 or LSM_NORMALS_LAZY");
        return LSM_EINVAL;
    }
    if (p->want_normals && (!(p->normal_radius > 0) || p->max_nn < 0)) {
        ctx->set_error("Invalid KDTreeSearchParamHybrid (radius <= 0 or max_nn < 0)");
        return LSM_EINVAL;
    }
    return LSM_OK;
}

int lsm_preprocess_batch(lsm_ctx *ctx, int64_t n, const lsm_cloud *clouds,
                         const lsm_prep_params *p, int64_t *n_out) {
    if (!ctx || n < 0 || (n > 0 && !clouds)) return LSM_EINVAL;
    int rc = check_prep(ctx, p);
    if (rc) return rc;
    std::vector<Cloud *> cs;
    cs.reserve(size_t(n));
    for (int64_t i = 0; i < n; ++i) {
        Cloud *c = find_cloud(ctx, clouds[i]);
        if (!c) {
            ctx->set_error("unknown cloud handle");
            return LSM_EINVAL;
        }
        for (Cloud *o : cs)
            if (o == c) {
                ctx->set_error("duplicate cloud in preprocess batch");
                return LSM_EINVAL;
            }
        cs.push_back(c);
    }
    if (n == 0) return LSM_OK;
    (void)hipSetDevice(ctx->device);
    return lsm_prep_batch(ctx, cs, *p, n_out);
}

int lsm_preprocess(lsm_ctx *ctx, lsm_cloud cloud, const lsm_prep_params *p, int64_t *n_out) {
    return lsm_preprocess_batch(ctx, 1, &cloud, p, n_out);
}

int lsm_cloud_download(lsm_ctx *ctx, lsm_cloud cloud, double *xyz, double *normals,
                       int64_t cap) {
    if (!ctx) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed) {
        ctx->set_error("cloud has not been pre-processed");
        return LSM_ESTATE;
    }
    if (cap < c->n) {
        ctx->set_error("output capacity smaller than the processed cloud");
        return LSM_EINVAL;
    }
    if (normals && !c->has_normals) {
        ctx->set_error("cloud has no normals");
        return LSM_ESTATE;
    }
    (void)hipSetDevice(ctx->device);
    if (normals) {
        const int rc = complete_normals(ctx, c);
        if (rc) return rc;
    }
    return lsm_download_run(ctx, c, xyz, normals, cap);
}

int lsm_cloud_voxel_keys(lsm_ctx *ctx, lsm_cloud cloud, int32_t *keys, int64_t cap) {
    if (!ctx || !keys) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed || !c->voxelized) {
        ctx->set_error("cloud is not voxel-down-sampled");
        return LSM_ESTATE;
    }
    if (cap < c->n) return LSM_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (c->n > 0) {
        LSM_HIP_TRY(ctx, hipMemcpyAsync(keys, c->d_vkeys, size_t(c->n) * 12,
                                        hipMemcpyDeviceToHost, ctx->stream));
    }
    LSM_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return LSM_OK;
}

int lsm_cloud_layout(lsm_ctx *ctx, lsm_cloud cloud, int32_t *perm, int64_t cap, uint32_t *cells,
                     int64_t cell_cap, int64_t *ncells) {
    if (!ctx || !ncells) return LSM_EINVAL;
    Cloud *c = find_cloud(ctx, cloud);
    if (!c) {
        ctx->set_error("unknown cloud handle");
        return LSM_EINVAL;
    }
    if (!c->processed) {
        ctx->set_error("cloud is not processed");
        return LSM_ESTATE;
    }
    const int64_t nc = int64_t(c->dev.nbx) * c->dev.nby * c->dev.nbz * LSM_BLK_CELLS;
    *ncells = nc;
    if ((perm && cap < c->n) || (cells && cell_cap < nc + 1)) {
        ctx->set_error("perm / cells capacity too small");
        return LSM_EINVAL;
    }
    (void)hipSetDevice(ctx->device);
    if (perm && c->n > 0)
        LSM_HIP_TRY(ctx, hipMemcpyAsync(perm, c->d_perm, size_t(c->n) * 4, hipMemcpyDeviceToHost,
                                        ctx->stream));
    if (cells)
        LSM_HIP_TRY(ctx, hipMemcpyAsync(cells, c->d_cell, size_t(nc + 1) * 4,
                                        hipMemcpyDeviceToHost, ctx->stream));
    LSM_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return LSM_OK;
}

static int check_icp(lsm_ctx *ctx, const lsm_icp_params *p) {
    if (!p) return LSM_EINVAL;
    if (!(p->max_correspondence_distance > 0.0)) {
        ctx->set_error("Invalid max_correspondence_distance.");
        return LSM_EINVAL;
    }
    if (p->method != LSM_P2P && p->method != LSM_P2PLANE) {
        ctx->set_error("unknown transformation estimation method");
        return LSM_EINVAL;
    }
    if (p->max_iteration < 0 || p->max_iteration > LSM_MAX_ITERATION) {
        ctx->set_error("max_iteration must be in [0, 2^20]");
        return LSM_EINVAL;
    }
    return LSM_OK;
}

int lsm_icp_batch(lsm_ctx *ctx, int64_t npairs, const lsm_cloud *src, const lsm_cloud *tgt,
                  const double *init, const lsm_icp_params *p, lsm_icp_result *out) {
    if (!ctx || npairs < 0 || (npairs > 0 && (!src || !tgt || !out))) return LSM_EINVAL;
    int rc = check_icp(ctx, p);
    if (rc) return rc;
    std::vector<Cloud *> s(static_cast<size_t>(npairs)), t(static_cast<size_t>(npairs));
    for (int64_t i = 0; i < npairs; ++i) {
        s[i] = find_cloud_nojoin(ctx, src[i]);   // (the ICP joins the side stream on the
        t[i] = find_cloud_nojoin(ctx, tgt[i]);   //  device, before its first accumulation)
        if (!s[i] || !t[i]) {
            ctx->set_error("unknown cloud handle");
            return LSM_EINVAL;
        }
        if (!s[i]->processed || !t[i]->processed) {
            ctx->set_error("registration needs pre-processed clouds (KeyFrame.pre_process)");
            return LSM_ESTATE;
        }
        if (p->method == LSM_P2PLANE && !t[i]->has_normals) {
            ctx->set_error("TransformationEstimationPointToPlane and "
                           "TransformationEstimationColoredICP require pre-computed normal "
                           "vectors for target PointCloud.");
            return LSM_ESTATE;
        }
    }
    if (npairs == 0) return LSM_OK;
    (void)hipSetDevice(ctx->device);
    return lsm_icp_run(ctx, npairs, s.data(), t.data(), init, *p, out);
}

int lsm_icp(lsm_ctx *ctx, lsm_cloud src, lsm_cloud tgt, const double init[16],
            const lsm_icp_params *p, lsm_icp_result *out) {
    return lsm_icp_batch(ctx, 1, &src, &tgt, init, p, out);
}

int lsm_icp_last_correspondences(lsm_ctx *ctx, int64_t *pairs, int64_t cap, int64_t *n) {
    if (!ctx || !n) return LSM_EINVAL;
    if (ctx->last_corr_pending) {   // compact the dense device array (source reference order)
        const int64_t n0 = ctx->last_corr_dense_n;
        std::vector<int32_t> dense(size_t(std::max<int64_t>(n0, 0)));
        if (n0 > 0) {
            void *d = ctx->buf("i_lastcorr_dense", size_t(n0) * 4);
            LSM_HIP_TRY(ctx, hipMemcpyAsync(dense.data(), d, size_t(n0) * 4, hipMemcpyDeviceToHost,
                                            ctx->stream));
            LSM_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        ctx->last_corr.clear();
        for (int64_t i = 0; i < n0; ++i)
            if (dense[size_t(i)] >= 0) {
                ctx->last_corr.push_back(i);
                ctx->last_corr.push_back(dense[size_t(i)]);
            }
        ctx->last_corr_pending = false;
    }
    int64_t m = int64_t(ctx->last_corr.size() / 2);
    *n = m;
    if (pairs) {
        if (cap < m) return LSM_EINVAL;
        std::memcpy(pairs, ctx->last_corr.data(), ctx->last_corr.size() * sizeof(int64_t));
    }
    return LSM_OK;
}

int lsm_loop_candidates(lsm_ctx *ctx, const double *positions, int64_t m,
                        double distance_backwards, double radius_threshold,
                        int64_t *index_backwards, int64_t *candidates, int64_t cap,
                        int64_t *n_candidates) {
    if (!ctx || m < 0 || (m > 0 && !positions) || !index_backwards || !n_candidates)
        return LSM_EINVAL;
    (void)hipSetDevice(ctx->device);
    return lsm_loop_candidates_run(ctx, positions, m, distance_backwards, radius_threshold,
                                   index_backwards, candidates, cap, n_candidates);
}

int lsm_loop_triplet_partners(lsm_ctx *ctx, const double *positions, int64_t m,
                              const int64_t *candidates, int64_t n_candidates, int64_t *partner) {
    if (!ctx || m < 0 || n_candidates < 0 || (n_candidates > 0 && (!candidates || !partner)))
        return LSM_EINVAL;
    for (int64_t k = 0; k < n_candidates; ++k)
        if (candidates[k] < 0 || candidates[k] >= m) {
            ctx->set_error("candidate index out of range");
            return LSM_EINVAL;
        }
    if (n_candidates == 0) return LSM_OK;
    (void)hipSetDevice(ctx->device);
    return lsm_loop_partners_run(ctx, positions, m, candidates, n_candidates, partner);
}

int lsm_set_timing(lsm_ctx *ctx, int32_t enable) {
    if (!ctx) return LSM_EINVAL;
    ctx->timing = enable != 0;
    ctx->statistics = enable >= 2;
    return LSM_OK;
}

int lsm_kernel_stats(lsm_ctx *ctx, const char *kernel, int64_t *launches, double *total_ms,
                     double *algo_bytes) {
    if (!ctx || !kernel) return LSM_EINVAL;
    auto it = ctx->stats.find(kernel);
    KStat s;
    if (it != ctx->stats.end()) s = it->second;
    if (launches) *launches = s.launches;
    if (total_ms) *total_ms = s.ms;
    if (algo_bytes) *algo_bytes = s.algo_bytes;
    return LSM_OK;
}

int lsm_reset_stats(lsm_ctx *ctx) {
    if (!ctx) return LSM_EINVAL;
    ctx->stats.clear();
    return LSM_OK;
}

}  // extern "C"
