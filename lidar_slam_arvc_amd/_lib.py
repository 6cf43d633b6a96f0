"""ctypes binding of liblidarsm.so (include/lidarsm.h).

The shared library is built in-tree (``lidar_slam_arvc_amd/_lib/liblidarsm.so``) by
``__graft_entry__.build()`` / ``make -C lidar_slam_arvc_amd/csrc``. There is no CPU fallback: if
the library or a gfx950 device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

LIB_PATH = os.environ.get("LIDARSM_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "_lib", "liblidarsm.so")   # env: A/B builds

LSM_OK = 0
LSM_P2P = 0
LSM_P2PLANE = 1
LSM_NORMALS_LAZY = 2     # lsm_prep_params.want_normals: normals on demand

EXPORTED = [
    "lsm_init", "lsm_free", "lsm_last_error", "lsm_version", "lsm_default_prep_params",
    "lsm_default_icp_params", "lsm_cloud_upload", "lsm_cloud_upload_f64", "lsm_cloud_upload_batch", "lsm_cloud_clone", "lsm_cloud_release",
    "lsm_cloud_info", "lsm_preprocess", "lsm_preprocess_batch", "lsm_cloud_download",
    "lsm_cloud_voxel_keys", "lsm_cloud_layout", "lsm_icp", "lsm_icp_batch", "lsm_icp_last_correspondences",
    "lsm_loop_candidates", "lsm_loop_triplet_partners", "lsm_set_timing", "lsm_kernel_stats",
    "lsm_reset_stats", "lsm_ground_plane", "lsm_plane_samples_get", "lsm_split_plane",
    "lsm_fpfh", "lsm_fpfh_download", "lsm_feature_correspondences", "lsm_ransac_feature",
    "lsm_se3_prefix", "lsm_voxel_down_sample_normals",
]


class PrepParams(C.Structure):
    _fields_ = [("min_radius", C.c_double), ("max_radius", C.c_double),
                ("min_height", C.c_double), ("max_height", C.c_double),
                ("voxel_size", C.c_double), ("normal_radius", C.c_double),
                ("max_nn", C.c_int32), ("want_normals", C.c_int32),
                ("grid_cell", C.c_double)]


class IcpParams(C.Structure):
    _fields_ = [("max_correspondence_distance", C.c_double), ("method", C.c_int32),
                ("max_iteration", C.c_int32), ("relative_fitness", C.c_double),
                ("relative_rmse", C.c_double)]


class IcpResult(C.Structure):
    _fields_ = [("transformation", C.c_double * 16), ("fitness", C.c_double),
                ("inlier_rmse", C.c_double), ("correspondences", C.c_int64),
                ("iterations", C.c_int32), ("status", C.c_int32)]


_P = C.c_void_p
_i64p = C.POINTER(C.c_int64)
_f64p = C.POINTER(C.c_double)
_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)


def load_library(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"liblidarsm.so not found at {path}; build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    sig = {
        "lsm_init": (C.c_int, [C.c_int, C.POINTER(_P)]),
        "lsm_free": (C.c_int, [_P]),
        "lsm_last_error": (C.c_char_p, [_P]),
        "lsm_version": (C.c_char_p, []),
        "lsm_default_prep_params": (None, [C.POINTER(PrepParams)]),
        "lsm_default_icp_params": (None, [C.POINTER(IcpParams)]),
        "lsm_cloud_upload": (C.c_int, [_P, _f32p, C.c_int64, _i64p]),
        "lsm_cloud_upload_f64": (C.c_int, [_P, _f64p, C.c_int64, _i64p]),
        "lsm_cloud_upload_batch": (C.c_int, [_P, C.POINTER(_f32p), _i64p, C.c_int64, _i64p]),
        "lsm_cloud_clone": (C.c_int, [_P, C.c_int64, _i64p]),
        "lsm_cloud_release": (C.c_int, [_P, C.c_int64]),
        "lsm_cloud_info": (C.c_int, [_P, C.c_int64, _i64p, _i64p, _i32p]),
        "lsm_preprocess": (C.c_int, [_P, C.c_int64, C.POINTER(PrepParams), _i64p]),
        "lsm_preprocess_batch": (C.c_int, [_P, C.c_int64, _i64p, C.POINTER(PrepParams), _i64p]),
        "lsm_cloud_download": (C.c_int, [_P, C.c_int64, _f64p, _f64p, C.c_int64]),
        "lsm_cloud_voxel_keys": (C.c_int, [_P, C.c_int64, _i32p, C.c_int64]),
        "lsm_cloud_layout": (C.c_int, [_P, C.c_int64, _i32p, C.c_int64, C.POINTER(C.c_uint32),
                                       C.c_int64, _i64p]),
        "lsm_icp": (C.c_int, [_P, C.c_int64, C.c_int64, _f64p, C.POINTER(IcpParams),
                              C.POINTER(IcpResult)]),
        "lsm_icp_batch": (C.c_int, [_P, C.c_int64, _i64p, _i64p, _f64p, C.POINTER(IcpParams),
                                    C.POINTER(IcpResult)]),
        "lsm_icp_last_correspondences": (C.c_int, [_P, _i64p, C.c_int64, _i64p]),
        "lsm_loop_candidates": (C.c_int, [_P, _f64p, C.c_int64, C.c_double, C.c_double, _i64p,
                                          _i64p, C.c_int64, _i64p]),
        "lsm_loop_triplet_partners": (C.c_int, [_P, _f64p, C.c_int64, _i64p, C.c_int64, _i64p]),
        "lsm_set_timing": (C.c_int, [_P, C.c_int32]),
        "lsm_kernel_stats": (C.c_int, [_P, C.c_char_p, _i64p, _f64p, _f64p]),
        "lsm_reset_stats": (C.c_int, [_P]),
        "lsm_ground_plane": (C.c_int, [_P, C.c_int64, C.c_double, C.c_double, C.c_int64,
                                       C.c_uint64, C.c_double, _f64p, _i64p, _i64p]),
        "lsm_plane_samples_get": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, _i32p]),
        "lsm_se3_prefix": (C.c_int, [_f64p, C.c_int64, _f64p]),
        "lsm_split_plane": (C.c_int, [_P, C.c_int64, _f64p, C.c_double, _i64p, _i64p]),
        "lsm_voxel_down_sample_normals": (C.c_int, [_P, C.c_int64, C.c_double, _i64p]),
        "lsm_fpfh": (C.c_int, [_P, C.c_int64, C.c_double, C.c_int32, _f64p, C.c_int64]),
        "lsm_fpfh_download": (C.c_int, [_P, C.c_int64, _f64p, C.c_int64]),
        "lsm_feature_correspondences": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int32, C.c_int32,
                                                  _i32p, C.c_int64, _i64p]),
        "lsm_ransac_feature": (C.c_int, [_P, C.c_int64, C.c_int64, _i32p, C.c_int64, C.c_double,
                                         C.c_double, C.c_int64, C.c_double, C.c_uint64, _f64p,
                                         _f64p, _f64p, _i64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None
_lib_lock = threading.Lock()


def lib() -> C.CDLL:
    global _lib
    with _lib_lock:
        if _lib is None:
            _lib = load_library()
        return _lib


def plane_samples(seed: int, n: int, num_iterations: int) -> np.ndarray:
    """The RANSAC candidate samples lsm_ground_plane draws (num_iterations x 3 indices)."""
    out = np.zeros((int(num_iterations), 3), dtype=np.int32)
    rc = lib().lsm_plane_samples_get(int(seed) & 0xFFFFFFFFFFFFFFFF, int(n), int(num_iterations),
                                     _ptr(out, C.c_int32))
    if rc != LSM_OK:
        raise ValueError("plane_samples needs n >= 3")
    return out


def se3_prefix(relative) -> np.ndarray:
    """Serial products of a chain of 4 x 4 transforms (lsm_se3_prefix): out[0] = I,
    out[k + 1] = out[k] @ relative[k] -- the global poses of compute_global_transformations
    (artelib/homogeneousmatrix.py:184-205) relative to the first keyframe."""
    rel = np.ascontiguousarray(np.asarray(relative, dtype=np.float64).reshape(-1, 16))
    out = np.empty((len(rel) + 1, 4, 4))
    rc = lib().lsm_se3_prefix(_ptr(rel, C.c_double), len(rel), _ptr(out, C.c_double))
    if rc != LSM_OK:
        raise ValueError("lsm_se3_prefix failed")
    return out


def _ptr(a: np.ndarray, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class Device:
    """One liblidarsm context (one GPU). Use :func:`device` for the per-process default."""

    def __init__(self, index: int = 0):
        self.lib = lib()
        h = _P()
        rc = self.lib.lsm_init(int(index), C.byref(h))
        if rc != LSM_OK:
            raise RuntimeError(f"lsm_init({index}) failed with code {rc}: no usable gfx950 device "
                               "(the registration path has no CPU fallback)")
        self.handle = h
        self.index = index

    # -- errors ------------------------------------------------------------------------------
    def check(self, rc: int, what: str):
        if rc != LSM_OK:
            msg = self.lib.lsm_last_error(self.handle).decode()
            raise RuntimeError(f"{what}: {msg} (code {rc})")

    def close(self):
        if getattr(self, "handle", None):
            self.lib.lsm_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- clouds ------------------------------------------------------------------------------
    def upload(self, points) -> int:
        p = np.asarray(points)
        if p.ndim != 2 or p.shape[1] != 3:
            raise ValueError("points must be N x 3")
        out = C.c_int64()
        if p.dtype == np.float32:
            p = np.ascontiguousarray(p)
            self.check(self.lib.lsm_cloud_upload(self.handle, _ptr(p, C.c_float), len(p),
                                                 C.byref(out)), "lsm_cloud_upload")
        else:
            p = np.ascontiguousarray(p, dtype=np.float64)
            self.check(self.lib.lsm_cloud_upload_f64(self.handle, _ptr(p, C.c_double), len(p),
                                                     C.byref(out)), "lsm_cloud_upload_f64")
        return out.value

    def upload_many(self, clouds) -> list:
        """lsm_cloud_upload_batch: every cloud (N x 3; float64 rounded to float32 on the host, as
        lsm_cloud_upload_f64 does) in one device allocation and one synchronisation."""
        arrs = []
        for points in clouds:
            p = np.asarray(points)
            if p.ndim != 2 or p.shape[1] != 3:
                raise ValueError("points must be N x 3")
            arrs.append(np.ascontiguousarray(p, dtype=np.float32))
        k = len(arrs)
        ptrs = (_f32p * max(k, 1))(*[_ptr(a, C.c_float) for a in arrs])
        ns = np.array([len(a) for a in arrs] or [0], dtype=np.int64)
        out = np.zeros(max(k, 1), dtype=np.int64)
        self.check(self.lib.lsm_cloud_upload_batch(self.handle, ptrs, _ptr(ns, C.c_int64), k,
                                                   _ptr(out, C.c_int64)), "lsm_cloud_upload_batch")
        return [int(x) for x in out[:k]]

    def clone(self, cloud: int) -> int:
        out = C.c_int64()
        self.check(self.lib.lsm_cloud_clone(self.handle, int(cloud), C.byref(out)),
                   "lsm_cloud_clone")
        return out.value

    def ground_plane(self, cloud: int, height=-0.5, distance_threshold=0.01,
                     num_iterations=1000, seed=0, probability=0.99999999):
        """KeyFrame.calculate_plane on the device: (plane[4], n_inliers, n_subset)."""
        plane = np.zeros(4)
        ni, ns = C.c_int64(), C.c_int64()
        self.check(self.lib.lsm_ground_plane(self.handle, int(cloud), float(height),
                                             float(distance_threshold), int(num_iterations),
                                             int(seed) & 0xFFFFFFFFFFFFFFFF, float(probability),
                                             _ptr(plane, C.c_double), C.byref(ni), C.byref(ns)),
                   "segment_plane")
        return plane, ni.value, ns.value

    def split_plane(self, cloud: int, plane, threshold=0.4):
        """KeyFrame.segment_plane on the device: two new raw cloud handles (ground, rest)."""
        pl = np.ascontiguousarray(plane, dtype=np.float64)
        g, r = C.c_int64(), C.c_int64()
        self.check(self.lib.lsm_split_plane(self.handle, int(cloud), _ptr(pl, C.c_double),
                                            float(threshold), C.byref(g), C.byref(r)),
                   "lsm_split_plane")
        return g.value, r.value

    def voxel_normals(self, cloud: int, voxel_size: float) -> int:
        """voxel_down_sample of a pre-processed cloud with normals (points averaged, normals
        averaged and not re-normalised): a new pre-processed cloud handle with those normals."""
        out = C.c_int64()
        self.check(self.lib.lsm_voxel_down_sample_normals(self.handle, int(cloud), float(voxel_size),
                                                          C.byref(out)),
                   "voxel_down_sample")
        return out.value

    def fpfh(self, cloud: int, radius=0.3, max_nn=100, download=True):
        """compute_fpfh_feature on the device; returns the n x 33 features (reference order)."""
        n = self.info(cloud)[1]
        out = np.zeros((n, 33)) if download else None
        self.check(self.lib.lsm_fpfh(self.handle, int(cloud), float(radius), int(max_nn),
                                     _ptr(out, C.c_double) if download else None, n),
                   "compute_fpfh_feature")
        return out

    def fpfh_download(self, cloud: int):
        """The features the last fpfh() call computed (n x 33, reference order); no recompute."""
        n = self.info(cloud)[1]
        out = np.zeros((n, 33))
        self.check(self.lib.lsm_fpfh_download(self.handle, int(cloud), _ptr(out, C.c_double), n),
                   "lsm_fpfh_download")
        return out

    def feature_correspondences(self, src: int, tgt: int, mutual=True, ransac_n=3):
        n_src = self.info(src)[1]
        out = np.zeros((max(n_src, 1), 2), dtype=np.int32)
        n = C.c_int64()
        self.check(self.lib.lsm_feature_correspondences(self.handle, int(src), int(tgt),
                                                        1 if mutual else 0, int(ransac_n),
                                                        _ptr(out, C.c_int32), len(out),
                                                        C.byref(n)), "feature matching")
        return out[:n.value].copy()

    def ransac_feature(self, src: int, tgt: int, corres, max_correspondence_distance=5.0,
                       edge=0.9, max_iteration=100000, confidence=0.999, seed=0):
        c = np.ascontiguousarray(corres, dtype=np.int32).reshape(-1, 2)
        T = np.zeros(16)
        fit, rmse = C.c_double(), C.c_double()
        ev = C.c_int64()
        self.check(self.lib.lsm_ransac_feature(self.handle, int(src), int(tgt),
                                               _ptr(c, C.c_int32), len(c),
                                               float(max_correspondence_distance), float(edge),
                                               int(max_iteration), float(confidence),
                                               int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(T, C.c_double),
                                               C.byref(fit), C.byref(rmse), C.byref(ev)),
                   "registration_ransac_based_on_feature_matching")
        return dict(transformation=T.reshape(4, 4), fitness=fit.value, inlier_rmse=rmse.value,
                    evaluated=ev.value)

    def release(self, cloud: int):
        self.check(self.lib.lsm_cloud_release(self.handle, int(cloud)), "lsm_cloud_release")

    def info(self, cloud: int):
        nr, npr, hn = C.c_int64(), C.c_int64(), C.c_int32()
        self.check(self.lib.lsm_cloud_info(self.handle, int(cloud), C.byref(nr), C.byref(npr),
                                           C.byref(hn)), "lsm_cloud_info")
        return nr.value, npr.value, bool(hn.value)

    def preprocess(self, clouds, params: PrepParams) -> np.ndarray:
        ids = np.ascontiguousarray(np.atleast_1d(np.asarray(clouds, dtype=np.int64)))
        n_out = np.zeros(len(ids), dtype=np.int64)
        self.check(self.lib.lsm_preprocess_batch(self.handle, len(ids), _ptr(ids, C.c_int64),
                                                 C.byref(params), _ptr(n_out, C.c_int64)),
                   "lsm_preprocess_batch")
        return n_out

    def download(self, cloud: int, normals: bool = False):
        _, n, hn = self.info(cloud)
        xyz = np.empty((n, 3), dtype=np.float64)
        nrm = np.empty((n, 3), dtype=np.float64) if normals else None
        self.check(self.lib.lsm_cloud_download(
            self.handle, int(cloud), _ptr(xyz, C.c_double),
            _ptr(nrm, C.c_double) if nrm is not None else None, n), "lsm_cloud_download")
        return (xyz, nrm) if normals else xyz

    def voxel_keys(self, cloud: int) -> np.ndarray:
        _, n, _ = self.info(cloud)
        k = np.empty((n, 3), dtype=np.int32)
        self.check(self.lib.lsm_cloud_voxel_keys(self.handle, int(cloud), _ptr(k, C.c_int32), n),
                   "lsm_cloud_voxel_keys")
        return k

    def layout(self, cloud: int):
        """(perm, cell_start) of a processed cloud's device layout (diagnostics: lsm_cloud_layout)."""
        _, n, _ = self.info(cloud)
        nc = np.zeros(1, dtype=np.int64)
        self.check(self.lib.lsm_cloud_layout(self.handle, int(cloud), None, 0, None, 0,
                                             _ptr(nc, C.c_int64)), "lsm_cloud_layout")
        perm = np.empty(n, dtype=np.int32)
        cells = np.empty(int(nc[0]) + 1, dtype=np.uint32)
        self.check(self.lib.lsm_cloud_layout(self.handle, int(cloud), _ptr(perm, C.c_int32), n,
                                             _ptr(cells, C.c_uint32), cells.size,
                                             _ptr(nc, C.c_int64)), "lsm_cloud_layout")
        return perm, cells

    # -- registration ------------------------------------------------------------------------
    def icp_batch(self, src, tgt, init, params: IcpParams):
        """registration_icp of every (src[k], tgt[k]) pair: a list of result dicts."""
        a = self.icp_batch_arrays(src, tgt, init, params)
        T = a["transformation"]
        fit, rmse = a["fitness"].tolist(), a["inlier_rmse"].tolist()
        nc, it, stt = a["n_corr"].tolist(), a["iterations"].tolist(), a["status"].tolist()
        return [dict(transformation=T[k], fitness=fit[k], inlier_rmse=rmse[k], n_corr=nc[k],
                     iterations=it[k], status=stt[k]) for k in range(len(T))]

    def icp_batch_arrays(self, src, tgt, init, params: IcpParams):
        """icp_batch with the results as arrays (transformation n x 4 x 4, fitness, inlier_rmse,
        n_corr, iterations, status): no per-pair Python objects for large batches."""
        s = np.ascontiguousarray(np.atleast_1d(np.asarray(src, dtype=np.int64)))
        t = np.ascontiguousarray(np.atleast_1d(np.asarray(tgt, dtype=np.int64)))
        if len(s) != len(t):
            raise ValueError("src and tgt must have the same length")
        n = len(s)
        ip = None
        if init is not None:
            ini = np.ascontiguousarray(np.asarray(init, dtype=np.float64).reshape(n, 16))
            ip = _ptr(ini, C.c_double)
        res = (IcpResult * max(n, 1))()
        self.check(self.lib.lsm_icp_batch(self.handle, n, _ptr(s, C.c_int64), _ptr(t, C.c_int64),
                                          ip, C.byref(params), res), "registration_icp")
        # one structured view of the result array (a per-field ctypes walk costs ~4 us a pair)
        a = np.frombuffer(res, dtype=np.dtype(IcpResult), count=n)
        return dict(transformation=a["transformation"].reshape(n, 4, 4).copy(),
                    fitness=a["fitness"].copy(), inlier_rmse=a["inlier_rmse"].copy(),
                    n_corr=a["correspondences"].copy(), iterations=a["iterations"].copy(),
                    status=a["status"].copy())

    def last_correspondences(self) -> np.ndarray:
        n = C.c_int64()
        self.check(self.lib.lsm_icp_last_correspondences(self.handle, None, 0, C.byref(n)),
                   "lsm_icp_last_correspondences")
        out = np.empty((n.value, 2), dtype=np.int64)
        self.check(self.lib.lsm_icp_last_correspondences(self.handle, _ptr(out, C.c_int64),
                                                         n.value, C.byref(n)),
                   "lsm_icp_last_correspondences")
        return out

    # -- loop closure ------------------------------------------------------------------------
    def loop_candidates(self, positions, distance_backwards, radius_threshold):
        P = np.ascontiguousarray(np.asarray(positions, dtype=np.float64).reshape(-1, 3))
        m = len(P)
        cand = np.empty(max(m, 1), dtype=np.int64)
        idx, nc = C.c_int64(), C.c_int64()
        self.check(self.lib.lsm_loop_candidates(self.handle, _ptr(P, C.c_double), m,
                                                float(distance_backwards),
                                                float(radius_threshold), C.byref(idx),
                                                _ptr(cand, C.c_int64), len(cand), C.byref(nc)),
                   "lsm_loop_candidates")
        return (None if idx.value < 0 else int(idx.value)), cand[:nc.value].copy()

    def loop_partners(self, positions, candidates):
        P = np.ascontiguousarray(np.asarray(positions, dtype=np.float64).reshape(-1, 3))
        c = np.ascontiguousarray(np.asarray(candidates, dtype=np.int64))
        part = np.empty(max(len(c), 1), dtype=np.int64)
        self.check(self.lib.lsm_loop_triplet_partners(self.handle, _ptr(P, C.c_double), len(P),
                                                      _ptr(c, C.c_int64), len(c),
                                                      _ptr(part, C.c_int64)),
                   "lsm_loop_triplet_partners")
        return part[:len(c)].copy()

    # -- instrumentation ---------------------------------------------------------------------
    def set_timing(self, on: bool, statistics: bool = False):
        """Per-kernel event timing; statistics=True also counts the neighbours of every normal
        computed (slower: statistics runs only)."""
        level = 2 if statistics else (1 if on else 0)
        self.check(self.lib.lsm_set_timing(self.handle, level), "lsm_set_timing")

    def kernel_stats(self, name: str):
        n, ms, b = C.c_int64(), C.c_double(), C.c_double()
        self.check(self.lib.lsm_kernel_stats(self.handle, name.encode(), C.byref(n), C.byref(ms),
                                             C.byref(b)), "lsm_kernel_stats")
        return dict(launches=n.value, ms=ms.value, algo_bytes=b.value)

    def reset_stats(self):
        self.check(self.lib.lsm_reset_stats(self.handle), "lsm_reset_stats")


_devices: dict = {}
_dev_lock = threading.Lock()


def device(index: int | None = None) -> Device:
    """Per-process default context (LOCAL_RANK or 0 unless given)."""
    if index is None:
        index = int(os.environ.get("LSM_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    with _dev_lock:
        d = _devices.get(index)
        if d is None:
            d = Device(index)
            _devices[index] = d
        return d


def prep_params(min_radius=0.5, max_radius=35.0, min_height=-1.0, max_height=50.0,
                voxel_size=None, normal_radius=0.3, max_nn=300, want_normals=True,
                grid_cell=0.0) -> PrepParams:
    """want_normals: True / False, or "lazy" (LSM_NORMALS_LAZY: the same normals, each computed
    when first used -- a P2Plane registration computes only those its correspondences reach)."""
    wn = LSM_NORMALS_LAZY if want_normals == "lazy" else (1 if want_normals else 0)
    return PrepParams(float(min_radius), float(max_radius), float(min_height), float(max_height),
                      float(voxel_size) if voxel_size is not None else 0.0, float(normal_radius),
                      int(max_nn), wn, float(grid_cell))


def icp_params(max_correspondence_distance=10.0, method="p2plane", max_iteration=30,
               relative_fitness=1e-6, relative_rmse=1e-6) -> IcpParams:
    m = {"p2p": LSM_P2P, "pointpoint": LSM_P2P, "p2plane": LSM_P2PLANE,
         "pointplane": LSM_P2PLANE}.get(method, method)
    if m not in (LSM_P2P, LSM_P2PLANE):
        raise ValueError(f"unknown estimation method {method!r}")
    return IcpParams(float(max_correspondence_distance), int(m), int(max_iteration),
                     float(relative_fitness), float(relative_rmse))
