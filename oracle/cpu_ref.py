"""ctypes binding of oracle/cpu/lsm_cpu.cpp -- TEST INFRASTRUCTURE ONLY.

The C++/OpenMP f64 CPU implementation of the path (SURVEY.md §8d's CPU baseline): bench.py's
``cpu_baseline`` leg times it, and tests check it against ``open3d_restated`` (the NumPy/SciPy
oracle). Same function names, arguments and results as the NumPy oracle, so either can be the
checker. The product never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import open3d_restated as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liblsmcpu.so")

_lib = None


def build() -> str:
    """Compile the library with g++ (oracle/cpu/Makefile) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpu")], check=True)
    return LIB


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    dp = ctypes.POINTER(ctypes.c_double)
    lib.lsmcpu_set_threads.argtypes = [ctypes.c_int]
    lib.lsmcpu_set_threads.restype = None
    lib.lsmcpu_filter.argtypes = [dp, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_double, dp]
    lib.lsmcpu_filter.restype = ctypes.c_int64
    lib.lsmcpu_voxel.argtypes = [dp, ctypes.c_int64, ctypes.c_double, dp]
    lib.lsmcpu_voxel.restype = ctypes.c_int64
    lib.lsmcpu_normals.argtypes = [dp, ctypes.c_int64, ctypes.c_double, ctypes.c_int, dp,
                                   ctypes.POINTER(ctypes.c_int64)]
    lib.lsmcpu_normals.restype = ctypes.c_int
    lib.lsmcpu_icp.argtypes = [dp, ctypes.c_int64, dp, ctypes.c_int64, dp, ctypes.c_double,
                               ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp,
                               dp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int32)]
    lib.lsmcpu_icp.restype = ctypes.c_int
    _lib = lib
    return lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _pts(points):
    return np.ascontiguousarray(np.asarray(points, dtype=np.float64).reshape(-1, 3))


def set_threads(n: int) -> None:
    load().lsmcpu_set_threads(int(n))


def filter_radius_height(points, min_radius=O.MIN_RADIUS, max_radius=O.MAX_RADIUS,
                         min_height=O.MIN_HEIGHT, max_height=O.MAX_HEIGHT):
    """keyframe.py:74-94 (strict radius/height mask, order kept)."""
    p = _pts(points)
    out = np.empty_like(p)
    m = load().lsmcpu_filter(_dp(p), len(p), float(min_radius), float(max_radius),
                             float(min_height), float(max_height), _dp(out))
    return out[:m].copy()


def voxel_down_sample(points, voxel_size):
    """VoxelDownSample: centroids in lexicographic key order (the NumPy oracle's [1])."""
    p = _pts(points)
    out = np.empty_like(p)
    m = load().lsmcpu_voxel(_dp(p), len(p), float(voxel_size), _dp(out))
    if m == -1:
        raise RuntimeError("voxel_size <= 0.")
    if m == -2:
        raise RuntimeError("voxel_size is too small.")
    return out[:m].copy()


def registration_multiscale(source_raw, target_raw, init=None, scales=(0.4, 0.2, 0.1),
                            max_corr=(2.0, 1.0, 0.5), method="p2plane"):
    """The multi-scale chain of the NumPy oracle (filter, then per scale voxel + normals + ICP)."""
    src_f = filter_radius_height(source_raw)
    tgt_f = filter_radius_height(target_raw)
    T = np.eye(4) if init is None else np.array(init, dtype=np.float64)
    out = []
    for v, d in zip(scales, max_corr):
        src = voxel_down_sample(src_f, v)
        tgt = voxel_down_sample(tgt_f, v)
        nrm = estimate_normals(tgt) if method == "p2plane" else None
        r = registration_icp(src, tgt, d, T, method, nrm)
        T = r["transformation"]
        out.append(r)
    return out


def estimate_normals(points, radius=O.NORMAL_RADIUS, max_nn=O.MAX_NN, return_counts=False):
    """EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) on a cloud without normals."""
    p = _pts(points)
    n = np.empty_like(p)
    c = np.empty(len(p), dtype=np.int64)
    load().lsmcpu_normals(_dp(p), len(p), float(radius), int(max_nn), _dp(n),
                          c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return (n, c) if return_counts else n


def registration_icp(source, target, max_corr=O.DISTANCE_THRESHOLD, init=None, method="p2plane",
                     target_normals=None, max_iteration=30, relative_fitness=1e-6,
                     relative_rmse=1e-6):
    """RegistrationICP (keyframe.py:246-252); the same dict as the NumPy oracle's."""
    if max_corr <= 0.0:
        raise RuntimeError("Invalid max_correspondence_distance.")
    if method == "p2plane" and target_normals is None:
        raise RuntimeError("TransformationEstimationPointToPlane requires pre-computed normal "
                           "vectors for target PointCloud.")
    if method not in ("p2plane", "p2p"):
        raise ValueError(f"unknown method {method!r}")
    s, t = _pts(source), _pts(target)
    tn = _pts(target_normals) if method == "p2plane" else None
    T = np.ascontiguousarray(np.eye(4) if init is None else np.array(init, dtype=np.float64))
    info = np.zeros(3)
    it = ctypes.c_int(0)
    corr = np.empty(len(s), dtype=np.int32)
    rc = load().lsmcpu_icp(_dp(s), len(s), _dp(t), len(t), _dp(tn) if tn is not None else None,
                           float(max_corr), 1 if method == "p2plane" else 0, int(max_iteration),
                           float(relative_fitness), float(relative_rmse), _dp(T), _dp(info),
                           ctypes.byref(it), corr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    if rc != 0:
        raise RuntimeError("lsmcpu_icp failed")
    si = np.flatnonzero(corr >= 0)
    return dict(transformation=T, fitness=float(info[0]), inlier_rmse=float(info[1]),
                n_corr=int(info[2]), iterations=int(it.value),
                correspondences=np.stack([si, corr[si].astype(np.int64)], axis=1))
