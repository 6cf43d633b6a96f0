"""KeyFrame drop-in (reference: keyframemanager/keyframe.py) on the MI355X registration path.

Same constructor, attributes and method names as the reference's KeyFrame; the Open3D calls
behind them are replaced by liblidarsm (include/lidarsm.h) through ctypes:

    load_pointcloud            keyframe.py:41-45    PCD -> device raw cloud (kept resident)
    filter_radius_height       keyframe.py:74-94    lsm_preprocess (filter only)
    down_sample                keyframe.py:108-111  lsm_preprocess (filter + voxel)
    pre_process                keyframe.py:113-124  lsm_preprocess (filter + voxel + normals)
    local_registration_simple  keyframe.py:231-260  lsm_icp (P2P / P2Plane, Open3D criteria)
    preprocess_icp2planes      keyframe.py:164-189  lsm_ground_plane (RANSAC) + lsm_split_plane +
                                                    normals of both parts
    local_registration_two_planes keyframe.py:262-295  two P2Plane ICPs in one batch, composed
    preprocess_fpfh            keyframe.py:191-229  icp2planes pre-processing + lsm_fpfh (§8f row 4)
    global_registration        keyframe.py:296-345  lsm_feature_correspondences + lsm_ransac_feature
                                                    + P2Plane refinement

``pointcloud`` / ``pointcloud_filtered`` expose ``.points`` (N x 3 float64) and ``.normals`` like
the o3d.geometry.PointCloud the reference kept, downloaded lazily from the device cache.

Deliberate divergences: an unknown ``option`` raises ValueError (the
reference hits UnboundLocalError, keyframe.py:253-255); ``transform`` returns a transformed host
copy instead of mutating the device-resident filtered cloud; both RANSACs ('icp2planes' plane,
'fpfh' feature matching) sample from splitmix64(``ransac_seed``) where Open3D uses its unseeded
RNG, and ``segment_plane`` returns the two parts with their final normals (r = 0.5 ground / 0.3
rest) already estimated. 'fpfh' with a voxel_size voxelises twice like the reference
(keyframe.py:193-203): the second pass (lsm_voxel_down_sample_normals) yields a new device cloud,
which becomes ``pointcloud_filtered``.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .config import ICP_PARAMETERS
from .pcd import read_pcd
from .se3 import HomogeneousMatrix


class HostPointCloud:
    """Plain host point cloud (what o3d.geometry.PointCloud offered to the reference's callers)."""

    def __init__(self, points, normals=None):
        self.points = np.asarray(points, dtype=np.float64)
        self.normals = None if normals is None else np.asarray(normals, dtype=np.float64)

    def has_normals(self):
        return self.normals is not None and len(self.normals) == len(self.points)

    def __len__(self):
        return len(self.points)

    def __add__(self, other):
        n = None
        if self.has_normals() and other.has_normals():
            n = np.vstack([self.normals, other.normals])
        return HostPointCloud(np.vstack([self.points, other.points]), n)

    def transform(self, T):
        T = np.asarray(getattr(T, "array", T), dtype=np.float64)
        self.points = self.points @ T[:3, :3].T + T[:3, 3]
        if self.has_normals():
            self.normals = self.normals @ T[:3, :3].T
        return self


class FeatureHandle:
    """The FPFH features of a device cloud (o3d Feature: ``.data`` 33 x N), fetched lazily.

    ``radius`` / ``max_nn`` record the KDTreeSearchParamHybrid the features were computed with;
    reading ``.data`` only downloads them (lsm_fpfh_download) and never recomputes."""

    def __init__(self, dev, handle, radius, max_nn):
        self._dev = dev
        self._handle = handle
        self.radius = radius
        self.max_nn = max_nn
        self._data = None

    @property
    def data(self):
        if self._data is None:
            self._data = self._dev.fpfh_download(self._handle).T
        return self._data


class DevicePointCloud:
    """A pre-processed cloud resident in HBM; host arrays are fetched on first access."""

    def __init__(self, dev, handle, has_normals):
        self._dev = dev
        self._handle = handle
        self._has_normals = has_normals
        self._points = None
        self._normals = None

    def _fetch(self):
        if self._has_normals:
            self._points, self._normals = self._dev.download(self._handle, normals=True)
        else:
            self._points = self._dev.download(self._handle)

    @property
    def points(self):
        if self._points is None:
            self._fetch()
        return self._points

    @property
    def normals(self):
        if not self._has_normals:
            return np.zeros((0, 3))
        if self._normals is None:
            self._fetch()
        return self._normals

    def has_normals(self):
        return self._has_normals

    def __len__(self):
        return self._dev.info(self._handle)[1]

    def to_host(self):
        return HostPointCloud(self.points.copy(), self.normals.copy() if self._has_normals else None)


class KeyFrame:
    def __init__(self, directory, scan_time, voxel_size, device=None):
        self.directory = directory
        self.scan_time = scan_time
        self.voxel_size = voxel_size
        self.voxel_size_normals = 0.1
        self.fpfh_threshold = 5
        self.pointcloud = None
        self.pointcloud_filtered = None
        self.pointcloud_ground_plane = None
        self.pointcloud_non_ground_plane = None
        self.pointcloud_fpfh = None
        self.voxel_size_normals_ground_plane = 0.5
        self.voxel_size_normals = 0.3            # keyframe.py:33 overrides :16
        self.max_radius = ICP_PARAMETERS.max_radius
        self.min_radius = ICP_PARAMETERS.min_radius
        self.max_height = ICP_PARAMETERS.max_height
        self.min_height = ICP_PARAMETERS.min_height
        self.plane_model = None
        self.pre_processed = False
        self.last_registration = None
        self._dev = device if device is not None else _lib.device()
        self._handle = None
        self._source = None           # path or "memory" of the resident raw cloud
        self._filter = None           # (radii, heights) of the current filtered cloud
        self._prep_key = None         # parameters of the current processed cloud
        self._planes = None           # (ground, rest) device handles of 'icp2planes'
        self._vn = None               # 'fpfh' + voxel_size: handle of the twice-voxelised cloud
        self.ransac_seed = 0          # RANSAC sampler seed (calculate_plane)

    # ------------------------------------------------------------------ raw cloud
    def pcd_path(self):
        return self.directory + "/robot0/lidar/data/" + str(self.scan_time) + ".pcd"

    def load_pointcloud(self):
        path = self.pcd_path()
        if self.resident(path):
            return          # device keyframe cache: same file already resident
        self.set_points(read_pcd(path), source=path)

    def set_points(self, xyz, source="memory"):
        """Attach an in-memory N x 3 scan (float32 = PCD precision) instead of reading a file."""
        self._release()
        xyz = np.asarray(xyz)
        self._attach(self._dev.upload(xyz if xyz.dtype == np.float32 else
                                      np.asarray(xyz, dtype=np.float64)), xyz, source)

    def resident(self, source) -> bool:
        """the raw cloud of `source` (a path) is already on the device (keyframe cache)"""
        return self._handle is not None and self._source == source

    def _attach(self, handle, xyz, source):
        """take over an uploaded raw cloud (set_points, KeyFrameManager.load_pointclouds)"""
        self._release()
        xyz = np.asarray(xyz)
        self._handle = handle
        self._source = source
        self.pointcloud = HostPointCloud(np.asarray(xyz, dtype=np.float64))
        self.pointcloud_filtered = None
        self._prep_key = None

    def _release(self):
        if self._handle is not None:
            try:
                self._dev.release(self._handle)
            finally:
                self._handle = None
                self._source = None

    def _release_planes(self):
        if self._planes is not None:
            try:
                for h in self._planes:
                    self._dev.release(h)
            finally:
                self._planes = None
        self._release_vn()

    def _release_vn(self):
        if self._vn is not None:
            try:
                self._dev.release(self._vn)
            finally:
                self._vn = None

    def _filtered_handle(self):
        """Device handle behind pointcloud_filtered (the twice-voxelised cloud after 'fpfh' with
        a voxel_size, else the keyframe's own cloud)."""
        return self._vn if self._vn is not None else self._handle

    def unload_pointcloud(self):
        self._release_planes()
        self._release()
        self.pointcloud = None
        self.pointcloud_filtered = None
        self.pointcloud_ground_plane = None
        self.pointcloud_non_ground_plane = None
        self.pointcloud_fpfh = None
        self._prep_key = None

    def __del__(self):
        try:
            self._release_planes()
            self._release()
        except Exception:
            pass

    # ------------------------------------------------------------------ pre-processing
    def _params(self, radii, heights, voxel, normals):
        r = radii if radii is not None else (self.min_radius, self.max_radius)
        h = heights if heights is not None else (self.min_height, self.max_height)
        return _lib.prep_params(min_radius=r[0], max_radius=r[1], min_height=h[0],
                                max_height=h[1], voxel_size=voxel,
                                normal_radius=self.voxel_size_normals,
                                max_nn=ICP_PARAMETERS.max_nn, want_normals=normals)

    def _key(self, radii, heights, voxel, normals):
        """Cache key of a processed cloud: every parameter the device pass depends on."""
        r = radii if radii is not None else (self.min_radius, self.max_radius)
        h = heights if heights is not None else (self.min_height, self.max_height)
        nk = (self.voxel_size_normals, ICP_PARAMETERS.max_nn) if normals else None
        return (tuple(r), tuple(h), voxel, normals, nk)

    def _run(self, radii, heights, voxel, normals):
        if self._handle is None:
            raise RuntimeError("KeyFrame has no point cloud loaded (call load_pointcloud)")
        key = self._key(radii, heights, voxel, normals)
        self._release_vn()              # pointcloud_filtered goes back to the keyframe's cloud
        if key != self._prep_key:
            self._dev.preprocess([self._handle], self._params(radii, heights, voxel, normals))
            self._prep_key = key
        self._filter = (radii, heights)
        self.pointcloud_filtered = DevicePointCloud(self._dev, self._handle, normals)
        return self.pointcloud_filtered

    def filter_radius_height(self, radii=None, heights=None):
        return self._run(radii, heights, None, False)

    def down_sample(self):
        if self.voxel_size is None:
            return
        radii, heights = self._filter if self._filter is not None else (None, None)
        self._run(radii, heights, self.voxel_size, False)

    def preprocess_icp_point_point(self):
        self._run(None, None, self.voxel_size, False)

    def preprocess_icp_point_plane(self):
        self._run(None, None, self.voxel_size, True)

    def pre_process(self, method=False):
        if self.pre_processed:
            return
        if method == "icppointpoint":
            self.preprocess_icp_point_point()
        elif method == "icppointplane":
            self.preprocess_icp_point_plane()
        elif method == "icp2planes":
            self.preprocess_icp2planes()
        elif method == "fpfh":
            self.preprocess_fpfh()

    # ------------------------------------------------------------------ FPFH (§8f row 4)
    def preprocess_fpfh(self):
        self._run(None, None, self.voxel_size, True)         # filter (+ voxel), normals
        if self.voxel_size is not None:                      # keyframe.py:202-203
            self._vn = self._dev.voxel_normals(self._handle, self.voxel_size)
            self.pointcloud_filtered = DevicePointCloud(self._dev, self._vn, True)
        self.plane_model = self.calculate_plane(pcd=self.pointcloud_filtered)
        g, ng = self.segment_plane(self.plane_model, pcd=self.pointcloud_filtered)
        self.pointcloud_ground_plane = g
        self.pointcloud_non_ground_plane = ng
        self._dev.fpfh(self._planes[1], self.voxel_size_normals, 100, download=False)
        self.pointcloud_fpfh = FeatureHandle(self._dev, self._planes[1], self.voxel_size_normals,
                                             100)

    def global_registration(self, other):
        """RANSAC on the non-ground parts' FPFH matches, then P2Plane ICP of the filtered clouds
        from its result (keyframe.py:296-345)."""
        for kf in (self, other):
            if kf.pointcloud_fpfh is None:
                raise RuntimeError("global_registration needs pre_process('fpfh') on both keyframes")
        src, tgt = other._planes[1], self._planes[1]
        corres = self._dev.feature_correspondences(src, tgt, mutual=True, ransac_n=3)
        r = self._dev.ransac_feature(src, tgt, corres, self.fpfh_threshold, 0.9, 100000, 0.999,
                                     seed=self.ransac_seed)
        self.last_ransac = r
        res = self._dev.icp_batch([other._filtered_handle()], [self._filtered_handle()],
                                  r["transformation"].reshape(1, 16),
                                  self.registration_params("pointplane"))[0]
        self.last_registration = res
        return HomogeneousMatrix(res["transformation"])

    # ------------------------------------------------------------------ two planes (§8f row 2)
    def preprocess_icp2planes(self):
        self._run(None, None, self.voxel_size, True)
        self.plane_model = self.calculate_plane(pcd=self.pointcloud_filtered)
        g, ng = self.segment_plane(self.plane_model, pcd=self.pointcloud_filtered)
        self.pointcloud_ground_plane = g
        self.pointcloud_non_ground_plane = ng

    def calculate_plane(self, pcd=None, height=-0.5, thresholdA=0.01):
        """RANSAC ground plane [a, b, c, d] of the points below `height` (keyframe.py:417-437)."""
        h = self._filtered_handle()
        if pcd is not None and getattr(pcd, "_handle", h) != h:
            raise ValueError("calculate_plane works on this keyframe's device cloud")
        if h is None or self._prep_key is None:
            raise RuntimeError("calculate_plane needs a pre-processed keyframe")
        plane, _, _ = self._dev.ground_plane(h, height, thresholdA, 1000,
                                             seed=self.ransac_seed)
        return plane.tolist()

    def segment_plane(self, plane_model, pcd=None, thresholdB=0.4):
        """(ground, non-ground) clouds within / beyond thresholdB of the plane
        (keyframe.py:439-461), resident on the device with their normals."""
        h = self._filtered_handle()
        if pcd is not None and getattr(pcd, "_handle", h) != h:
            raise ValueError("segment_plane works on this keyframe's device cloud")
        if self._planes is not None:
            for p in self._planes:
                self._dev.release(p)
            self._planes = None
        g, ng = self._dev.split_plane(h, np.asarray(plane_model, dtype=np.float64), thresholdB)
        self._planes = (g, ng)
        keep_all = dict(min_radius=-np.inf, max_radius=1e15, min_height=-1e15, max_height=1e15,
                        max_nn=ICP_PARAMETERS.max_nn_gd, want_normals=True)
        self._dev.preprocess([g], _lib.prep_params(normal_radius=self.voxel_size_normals_ground_plane,
                                                   **keep_all))
        keep_all["max_nn"] = ICP_PARAMETERS.max_nn
        self._dev.preprocess([ng], _lib.prep_params(normal_radius=self.voxel_size_normals,
                                                    **keep_all))
        return DevicePointCloud(self._dev, g, True), DevicePointCloud(self._dev, ng, True)

    def local_registration_two_planes(self, other, initial_transform):
        """Ground parts and non-ground parts registered from the same guess (one ICP batch);
        x, y, yaw from the non-ground result, z, roll, pitch from the ground result."""
        T, _ = two_planes_batch(self._dev, [(self, other)],
                                [np.eye(4) if initial_transform is None else initial_transform])
        return T[0]

    # ------------------------------------------------------------------ registration
    def registration_params(self, option):
        m = {"pointpoint": "p2p", "pointplane": "p2plane"}.get(option)
        if m is None:
            raise ValueError("UNKNOWN OPTION. Should be pointpoint or pointplane")
        return _lib.icp_params(max_correspondence_distance=ICP_PARAMETERS.distance_threshold,
                               method=m)

    def local_registration_simple(self, other, initial_transform, option="pointpoint"):
        """ICP of `other` (source) onto `self` (target); returns T mapping other -> self."""
        if initial_transform is None:
            initial_transform = np.eye(4)
        prm = self.registration_params(option)
        for kf in (self, other):
            if kf._handle is None or kf._prep_key is None:
                raise RuntimeError("registration needs pre-processed keyframes (pre_process)")
        init = np.asarray(initial_transform, dtype=np.float64).reshape(1, 16)
        # the reference registers pointcloud_filtered (keyframe.py:246-252): after 'fpfh' with a
        # voxel_size that is the twice-voxelised cloud, not the keyframe's own processed cloud
        res = self._dev.icp_batch([other._filtered_handle()], [self._filtered_handle()], init,
                                  prm)[0]
        self.last_registration = res
        return HomogeneousMatrix(res["transformation"])

    def transform(self, T):
        if self.pointcloud_filtered is None:
            raise RuntimeError("no filtered cloud")
        pc = self.pointcloud_filtered
        host = pc.to_host() if isinstance(pc, DevicePointCloud) else pc
        return host.transform(T)


def two_planes_batch(dev, pairs, inits):
    """local_registration_two_planes for many (target, source) keyframe pairs: all 2P ICPs in one
    device batch. Returns (HomogeneousMatrix list, raw per-pair (ground, rest) results)."""
    from .se3 import Euler
    src, tgt, init = [], [], []
    for (kt, ks), T0 in zip(pairs, inits):
        for kf in (kt, ks):
            if kf._planes is None:
                raise RuntimeError("local_registration_two_planes needs "
                                   "pre_process('icp2planes') on both keyframes")
        T0 = np.asarray(getattr(T0, "array", T0), dtype=np.float64).reshape(16)
        src += [ks._planes[0], ks._planes[1]]
        tgt += [kt._planes[0], kt._planes[1]]
        init += [T0, T0]
    if not src:
        return [], []
    res = dev.icp_batch(src, tgt, np.stack(init),
                        _lib.icp_params(method="p2plane",
                                        max_correspondence_distance=ICP_PARAMETERS.distance_threshold))
    out, raw = [], []
    for k in range(len(pairs)):
        ra, rb = res[2 * k], res[2 * k + 1]
        t1 = HomogeneousMatrix(ra["transformation"]).t2v(n=3)
        t2 = HomogeneousMatrix(rb["transformation"]).t2v(n=3)
        out.append(HomogeneousMatrix(np.array([t2[0], t2[1], t1[2]]),
                                     Euler([t1[3], t1[4], t2[5]])))
        raw.append((ra, rb))
    return out, raw
