"""Seeded synthetic LiDAR scenes for tests and the benchmark.

The reference ships no data (its datasets live under absolute paths, run_scanmatcher.py:146-157),
so every workload here is synthetic, as SURVEY.md §8d specifies:

* a ground plane at world z = 0 seen from a sensor mounted 0.69 m above it (the reference's
  ground-plane model ``[0, 0, 1, 0.69]``, keyframe.py:436);
* axis-aligned boxes (buildings, parked objects), thin wall segments and vertical poles placed
  in a band around a closed trajectory;
* a spinning multi-ring LiDAR (HDL-64 / Ouster-128 / 16-ring) ray-cast against that scene,
  range noise N(0, 0.02 m), returns beyond 60 m dropped.

Scans come out as float32 N x 3 arrays in the sensor frame, ring-major (all azimuths of ring 0,
then ring 1, ...), misses removed -- the same shape ``o3d.io.read_point_cloud`` hands the
reference (keyframe.py:45). Poses are 4x4 float64 world<-sensor transforms.

This module is data generation only; it is not part of the registration path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

SENSOR_HEIGHT = 0.69


@dataclass(frozen=True)
class LidarModel:
    rings: int
    azimuths: int
    el_min_deg: float
    el_max_deg: float
    max_range: float = 60.0
    noise: float = 0.02

    def directions(self) -> np.ndarray:
        el = np.deg2rad(np.linspace(self.el_min_deg, self.el_max_deg, self.rings))
        az = np.arange(self.azimuths) * (2.0 * np.pi / self.azimuths)
        ce, se = np.cos(el)[:, None], np.sin(el)[:, None]
        d = np.stack([ce * np.cos(az)[None, :], ce * np.sin(az)[None, :],
                      np.broadcast_to(se, (self.rings, self.azimuths))], axis=-1)
        return d.reshape(-1, 3)


VLP16_8K = LidarModel(16, 512, -15.0, 15.0)          # C1: 8,192 rays
HDL64 = LidarModel(64, 1024, -24.9, 2.0)             # C2/C3/C4: 65,536 rays
OUSTER128 = LidarModel(128, 2048, -22.5, 22.5)       # C5: 262,144 rays


@dataclass
class Scene:
    boxes: np.ndarray                 # K x 6 (xmin, ymin, zmin, xmax, ymax, zmax)
    poles: np.ndarray                 # P x 4 (cx, cy, radius, height)
    path: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))


def loop_path(length_m: float = 1000.0, n: int = 4000) -> np.ndarray:
    """Closed, gently wavy loop of the given length (x, y samples, uniform in arc length)."""
    th = np.linspace(0.0, 2.0 * np.pi, 8 * n, endpoint=False)
    r = 1.0 + 0.12 * np.sin(3 * th) + 0.05 * np.cos(5 * th)
    xy = np.stack([r * np.cos(th), r * np.sin(th)], axis=1)
    seg = np.linalg.norm(np.diff(np.vstack([xy, xy[:1]]), axis=0), axis=1)
    xy *= length_m / seg.sum()
    s = np.concatenate([[0.0], np.cumsum(seg * length_m / seg.sum())])[:-1]
    su = np.linspace(0.0, length_m, n, endpoint=False)
    return np.stack([np.interp(su, s, xy[:, 0]), np.interp(su, s, xy[:, 1])], axis=1)


def make_scene(seed: int, path: np.ndarray) -> Scene:
    """Objects in a band around ``path``: boxes, wall segments and poles, never on the path."""
    rng = np.random.default_rng(seed)
    seg = np.diff(np.vstack([path, path[:1]]), axis=0)
    s = np.concatenate([[0.0], np.cumsum(np.linalg.norm(seg, axis=1))])
    total = s[-1]

    def frame_at(u):
        x = np.interp(u % total, s[:-1], path[:, 0])
        y = np.interp(u % total, s[:-1], path[:, 1])
        x2 = np.interp((u + 1.0) % total, s[:-1], path[:, 0])
        y2 = np.interp((u + 1.0) % total, s[:-1], path[:, 1])
        t = np.array([x2 - x, y2 - y])
        t /= max(np.linalg.norm(t), 1e-9)
        return np.array([x, y]), t, np.array([-t[1], t[0]])

    boxes, poles = [], []
    for u in np.arange(0.0, total, 4.0):
        p, t, nrm = frame_at(u + rng.uniform(0, 5))
        for side in (-1.0, 1.0):
            if rng.random() < 0.8:       # building / object box
                off = side * rng.uniform(4.0, 22.0)
                c = p + off * nrm
                hx, hy = rng.uniform(0.25, 1.5, size=2)
                h = rng.uniform(0.5, 8.0)
                boxes.append([c[0] - hx, c[1] - hy, 0.0, c[0] + hx, c[1] + hy, h])
            if rng.random() < 0.45:      # pole
                off = side * rng.uniform(3.0, 12.0)
                c = p + off * nrm
                poles.append([c[0], c[1], rng.uniform(0.1, 0.3), rng.uniform(2.0, 7.0)])
            if rng.random() < 0.5:       # wall segment, axis aligned, 15-25 m out
                off = side * rng.uniform(15.0, 25.0)
                c = p + off * nrm
                ln = rng.uniform(4.0, 10.0)
                if abs(t[0]) > abs(t[1]):
                    boxes.append([c[0] - ln / 2, c[1] - 0.15, 0.0, c[0] + ln / 2, c[1] + 0.15,
                                  rng.uniform(2.0, 4.0)])
                else:
                    boxes.append([c[0] - 0.15, c[1] - ln / 2, 0.0, c[0] + 0.15, c[1] + ln / 2,
                                  rng.uniform(2.0, 4.0)])
    return Scene(np.asarray(boxes, dtype=np.float64).reshape(-1, 6),
                 np.asarray(poles, dtype=np.float64).reshape(-1, 4), path)


def path_pose(path: np.ndarray, u: float, rng: np.random.Generator | None = None,
              tilt_deg: float = 0.5) -> np.ndarray:
    """World<-sensor pose at arc length ``u`` along ``path`` (yaw along the tangent)."""
    seg = np.diff(np.vstack([path, path[:1]]), axis=0)
    s = np.concatenate([[0.0], np.cumsum(np.linalg.norm(seg, axis=1))])
    total = s[-1]
    x = np.interp(u % total, s[:-1], path[:, 0])
    y = np.interp(u % total, s[:-1], path[:, 1])
    x2 = np.interp((u + 0.5) % total, s[:-1], path[:, 0])
    y2 = np.interp((u + 0.5) % total, s[:-1], path[:, 1])
    yaw = math.atan2(y2 - y, x2 - x)
    roll = pitch = 0.0
    if rng is not None:
        roll, pitch = np.deg2rad(rng.normal(0.0, tilt_deg, size=2))
    return pose_from(x, y, SENSOR_HEIGHT, roll, pitch, yaw)


def rot_xyz(roll: float, pitch: float, yaw: float) -> np.ndarray:
    cr, sr, cp, sp, cy, sy = (math.cos(roll), math.sin(roll), math.cos(pitch), math.sin(pitch),
                              math.cos(yaw), math.sin(yaw))
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1.0]])
    ry = np.array([[cp, 0, sp], [0, 1.0, 0], [-sp, 0, cp]])
    rx = np.array([[1.0, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return rz @ ry @ rx


def pose_from(x, y, z, roll, pitch, yaw) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = rot_xyz(roll, pitch, yaw)
    T[:3, 3] = (x, y, z)
    return T


def perturb(T: np.ndarray, rng: np.random.Generator, sigma_t: float, sigma_rot_deg: float,
            yaw_only: bool = False) -> np.ndarray:
    """T composed with a small random motion (odometry-like prior)."""
    r = np.deg2rad(rng.normal(0.0, sigma_rot_deg, size=3))
    if yaw_only:
        r[:2] = 0.0
    D = pose_from(*rng.normal(0.0, sigma_t, size=3), *r)
    return T @ D


def _box_hits(d: np.ndarray, o: np.ndarray, bx: np.ndarray) -> np.ndarray:
    """Nearest slab-test hit of each ray (rows of d) over the boxes bx (inf: none)."""
    if not len(bx) or not len(d):
        return np.full(len(d), np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1 = (bx[None, :, 0:3] - o[None, None, :]) * inv[:, None, :]
        t2 = (bx[None, :, 3:6] - o[None, None, :]) * inv[:, None, :]
    tmin = np.nanmax(np.minimum(t1, t2), axis=2)
    tmax = np.nanmin(np.maximum(t1, t2), axis=2)
    ok = (tmax >= np.maximum(tmin, 1e-6))
    tb = np.where(ok, np.where(tmin > 1e-6, tmin, np.inf), np.inf)
    return tb.min(axis=1)


def _pole_hits(d: np.ndarray, o: np.ndarray, pl: np.ndarray) -> np.ndarray:
    """Nearest hit of each ray on the vertical cylinders pl (inf: none)."""
    if not len(pl) or not len(d):
        return np.full(len(d), np.inf)
    ox = o[0] - pl[None, :, 0]
    oy = o[1] - pl[None, :, 1]
    a2 = (d[:, 0:1] ** 2 + d[:, 1:2] ** 2)
    b2 = 2.0 * (ox * d[:, 0:1] + oy * d[:, 1:2])
    c2 = ox * ox + oy * oy - pl[None, :, 2] ** 2
    disc = b2 * b2 - 4.0 * a2 * c2
    with np.errstate(divide="ignore", invalid="ignore"):
        tc = (-b2 - np.sqrt(np.maximum(disc, 0.0))) / (2.0 * a2)
    z = o[2] + tc * d[:, 2:3]
    okc = (disc > 0) & (tc > 1e-6) & (z >= 0.0) & (z <= pl[None, :, 3])
    return np.where(okc, tc, np.inf).min(axis=1)


N_SECTORS = 64          # azimuth sectors of the culled ray cast
_ANG_MARGIN = 1e-3      # rad: angular intervals are widened by this much (conservative)


def _sector_sets(o: np.ndarray, lo: np.ndarray, hi: np.ndarray, everywhere: np.ndarray) -> list:
    """Object indices per azimuth sector: object j covers the world azimuths [lo_j, hi_j] (as
    seen from o, span < pi, possibly wrapping), or every azimuth when everywhere_j."""
    w = 2.0 * np.pi / N_SECTORS
    sets = [[] for _ in range(N_SECTORS)]
    for j in range(len(lo)):
        if everywhere[j]:
            for s in range(N_SECTORS):
                sets[s].append(j)
            continue
        s0 = int(math.floor((lo[j] - _ANG_MARGIN + np.pi) / w))
        s1 = int(math.floor((hi[j] + _ANG_MARGIN + np.pi) / w))
        for s in range(s0, s1 + 1):
            sets[s % N_SECTORS].append(j)
    return [np.asarray(v, dtype=np.int64) for v in sets]


def raycast(scene: Scene, pose: np.ndarray, model: LidarModel, rng: np.random.Generator,
            chunk: int = 16384) -> np.ndarray:
    """Ray-cast one spinning scan; returns float32 M x 3 sensor-frame points (misses removed).

    Rays are grouped by world azimuth sector and tested only against the boxes / poles whose
    angular extent (seen from the sensor) overlaps the sector. A ray's xy direction must lie
    inside an object's angular extent to reach its vertical prism, so the culled set always
    holds the object it hits, and every (ray, object) test is the same arithmetic as the brute
    force over all objects (``raycast_bruteforce``): the scans are bit-identical to it.
    """
    d_s = model.directions()
    R, o = pose[:3, :3], pose[:3, 3]
    # d_s R^T without BLAS: this runs in worker threads, and concurrent OpenBLAS calls gave
    # run-to-run different scans on many-core hosts
    d_w = d_s[:, 0:1] * R[:, 0] + d_s[:, 1:2] * R[:, 1] + d_s[:, 2:3] * R[:, 2]
    bx, pl = _near_objects(scene, o, model)
    dz = d_w[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        t_hit = np.where(dz < -1e-9, -o[2] / dz, np.inf)
    # angular extents of the boxes' xy footprints and of the poles
    if len(bx):
        inside = ((o[0] >= bx[:, 0] - 1e-6) & (o[0] <= bx[:, 3] + 1e-6) &
                  (o[1] >= bx[:, 1] - 1e-6) & (o[1] <= bx[:, 4] + 1e-6))
        cxs = np.stack([bx[:, 0], bx[:, 3], bx[:, 3], bx[:, 0]], axis=1) - o[0]
        cys = np.stack([bx[:, 1], bx[:, 1], bx[:, 4], bx[:, 4]], axis=1) - o[1]
        ref = np.arctan2(cys.mean(axis=1), cxs.mean(axis=1))
        rel = np.arctan2(cys, cxs) - ref[:, None]
        rel = (rel + np.pi) % (2.0 * np.pi) - np.pi
        blo, bhi = ref + rel.min(axis=1), ref + rel.max(axis=1)
        box_sets = _sector_sets(o, blo, bhi, inside)
    if len(pl):
        dist = np.hypot(pl[:, 0] - o[0], pl[:, 1] - o[1])
        near_pole = dist <= pl[:, 2] * 1.001 + 1e-3
        half = np.arcsin(np.minimum(1.0, (pl[:, 2] * 1.001 + 1e-3) / np.maximum(dist, 1e-9)))
        pc = np.arctan2(pl[:, 1] - o[1], pl[:, 0] - o[0])
        pole_sets = _sector_sets(o, pc - half, pc + half, near_pole)
    w = 2.0 * np.pi / N_SECTORS
    sec = np.floor((np.arctan2(d_w[:, 1], d_w[:, 0]) + np.pi) / w).astype(np.int64) % N_SECTORS
    order = np.argsort(sec, kind="stable")
    bounds = np.searchsorted(sec[order], np.arange(N_SECTORS + 1))
    for s in range(N_SECTORS):
        idx = order[bounds[s]:bounds[s + 1]]
        if not len(idx):
            continue
        d = d_w[idx]
        best = t_hit[idx]
        if len(bx):
            best = np.minimum(best, _box_hits(d, o, bx[box_sets[s]]))
        if len(pl):
            best = np.minimum(best, _pole_hits(d, o, pl[pole_sets[s]]))
        t_hit[idx] = best
    return _finish_scan(d_s, t_hit, model, rng)


def _near_objects(scene: Scene, o: np.ndarray, model: LidarModel):
    near = model.max_range + 3.0
    bx = scene.boxes
    if len(bx):
        cx = np.clip(o[0], bx[:, 0], bx[:, 3]) - o[0]
        cy = np.clip(o[1], bx[:, 1], bx[:, 4]) - o[1]
        bx = bx[cx * cx + cy * cy < near * near]
    pl = scene.poles
    if len(pl):
        pl = pl[(pl[:, 0] - o[0]) ** 2 + (pl[:, 1] - o[1]) ** 2 < near * near]
    return bx, pl


def raycast_bruteforce(scene: Scene, pose: np.ndarray, model: LidarModel,
                       rng: np.random.Generator, chunk: int = 16384) -> np.ndarray:
    """``raycast`` without the sector culling (every ray against every near object); kept as
    the check that the culled ray cast returns the same scans."""
    d_s = model.directions()
    R, o = pose[:3, :3], pose[:3, 3]
    d_w = d_s[:, 0:1] * R[:, 0] + d_s[:, 1:2] * R[:, 1] + d_s[:, 2:3] * R[:, 2]
    bx, pl = _near_objects(scene, o, model)
    t_hit = np.full(len(d_w), np.inf)
    for a in range(0, len(d_w), chunk):
        d = d_w[a:a + chunk]
        dz = d[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            best = np.where(dz < -1e-9, -o[2] / dz, np.inf)
        best = np.minimum(best, _box_hits(d, o, bx))
        best = np.minimum(best, _pole_hits(d, o, pl))
        t_hit[a:a + chunk] = best
    return _finish_scan(d_s, t_hit, model, rng)


def _finish_scan(d_s, t_hit, model, rng):
    hit = np.isfinite(t_hit) & (t_hit <= model.max_range)
    rng_noise = rng.normal(0.0, model.noise, size=len(d_s))
    t = t_hit + rng_noise
    pts = d_s[hit] * t[hit, None]
    return pts.astype(np.float32)


@dataclass
class Sequence:
    """Keyframes along a path: scans, ground-truth poses, odometry-like relative priors."""
    scans: list
    poses: np.ndarray          # K x 4 x 4 world<-sensor (ground truth)
    priors: np.ndarray         # (K-1) x 4 x 4 noisy relative transforms T_i^-1 T_{i+1}


def make_sequence(n_keyframes: int, seed: int = 3, model: LidarModel = HDL64,
                  spacing: float = 0.5, start: float = 0.0, path_length: float = 1000.0,
                  sigma_t: float = 0.05, sigma_rot_deg: float = 1.0,
                  first_index: int = 0, processes: int = 0) -> Sequence:
    """C3-style sequence: keyframes every ``spacing`` metres along a closed loop.

    ``first_index`` lets ranks generate disjoint chunks of one global sequence: keyframe ``k``
    always gets the same pose, scan noise and prior no matter which chunk generates it.
    ``processes`` > 0 ray-casts in that many forked worker processes (only before the GPU is
    initialised in this process: bench.py); otherwise threads.
    """
    path = loop_path(path_length)
    scene = make_scene(seed, path)

    def one(k):
        rng = np.random.default_rng([seed, k])
        T = path_pose(path, start + k * spacing, rng)
        return T, raycast(scene, T, model, rng)

    out = _parallel_map(one, range(first_index, first_index + n_keyframes), processes)
    poses = np.asarray([o[0] for o in out])
    scans = [o[1] for o in out]
    priors = []
    for k in range(first_index, first_index + n_keyframes - 1):
        rng = np.random.default_rng([seed, k, 7])
        j = k - first_index
        rel = np.linalg.inv(poses[j]) @ poses[j + 1]
        priors.append(perturb(rel, rng, sigma_t, sigma_rot_deg))
    return Sequence(scans, poses, np.asarray(priors).reshape(-1, 4, 4))


@dataclass
class PairSet:
    """Independent revisit pairs (C4 loop-closure batch)."""
    targets: list
    sources: list
    gt: np.ndarray             # P x 4 x 4, T_target^-1 T_source
    init: np.ndarray           # P x 4 x 4 noisy initial guesses


def make_revisit_pairs(n_pairs: int, seed: int = 4, model: LidarModel = HDL64,
                       path_length: float = 1000.0, sigma_t: float = 0.3,
                       sigma_yaw_deg: float = 3.0, first_index: int = 0,
                       processes: int = 0) -> PairSet:
    """C4-style pairs: a pose on the loop and a revisit 0.5-2 m / <=10 deg away."""
    path = loop_path(path_length)
    scene = make_scene(seed, path)

    def one(k):
        rng = np.random.default_rng([seed, k])
        u = rng.uniform(0.0, path_length)
        Ti = path_pose(path, u, rng)
        off = rng.uniform(0.5, 2.0)
        ang = rng.uniform(0, 2 * np.pi)
        D = pose_from(off * math.cos(ang), off * math.sin(ang), 0.0, 0.0, 0.0,
                      np.deg2rad(rng.uniform(-10.0, 10.0)))
        Tj = Ti @ D
        a = raycast(scene, Ti, model, rng)
        b = raycast(scene, Tj, model, rng)
        rel = np.linalg.inv(Ti) @ Tj
        return a, b, rel, perturb(rel, rng, sigma_t, sigma_yaw_deg, yaw_only=True)

    out = _parallel_map(one, range(first_index, first_index + n_pairs), processes)
    return PairSet([o[0] for o in out], [o[1] for o in out], np.asarray([o[2] for o in out]),
                   np.asarray([o[3] for o in out]))


_FORK_FN = None


def _fork_call(i):
    return _FORK_FN(i)


def _gpu_initialised() -> bool:
    """True when this process may already hold a GPU context (so it must not fork): torch or
    liblidarsm initialised it, or a profiler (rocprofv3 preloads a library that does)."""
    import os
    import sys
    if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(
            k.startswith("ROCPROF") for k in os.environ):
        return True
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        return True
    lib = sys.modules.get("lidar_slam_arvc_amd._lib")
    return bool(lib is not None and getattr(lib, "_devices", None))


def _parallel_map(fn, items, processes: int = 0):
    """Order-preserving map: forked processes when asked for and safe (no GPU context in this
    process yet), else a thread pool (the per-sector NumPy calls are small and mostly hold the
    GIL, so threads gain little)."""
    from concurrent.futures import ThreadPoolExecutor
    import os
    from threadpoolctl import threadpool_limits
    items = list(items)
    if processes > 1 and len(items) > 1 and not _gpu_initialised():
        import multiprocessing as mp
        global _FORK_FN
        _FORK_FN = fn
        try:
            with threadpool_limits(limits=1, user_api="blas"):
                with mp.get_context("fork").Pool(min(processes, len(items))) as pool:
                    return pool.map(_fork_call, items, chunksize=4)
        finally:
            _FORK_FN = None
    workers = max(1, min(8, os.cpu_count() or 1, len(items)))
    # single-threaded BLAS inside the workers: the small matrix products of the pose math must
    # not race on OpenBLAS's shared buffers (that made scans differ between runs)
    with threadpool_limits(limits=1, user_api="blas"):
        if workers == 1:
            return [fn(i) for i in items]
        with ThreadPoolExecutor(workers) as ex:
            return list(ex.map(fn, items))
