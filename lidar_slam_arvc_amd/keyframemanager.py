"""KeyFrameManager drop-in (reference: keyframemanager/keyframemanager.py).

Same constructor and methods (add_keyframes :20-24, add_keyframe :26-30, load_pointcloud(s)
:32-38, unload_pointcloud :40-41, pre_process :49-50, compute_transformation :52-75, build_map
:154-184), plus the batched forms the MI355X path is built for:

* ``pre_process_batch(indices)`` -- one device pass over many keyframes;
* ``compute_transformations(pairs, Tijs)`` -- many independent registrations in one ICP batch
  (scan-matcher chain, loop-closure candidates).

``compute_transformation`` dispatches on ``method`` exactly like the reference: 'icppointpoint'
-> P2P, 'icppointplane' -> P2Plane, 'icp2planes' -> local_registration_two_planes (:66-67),
'fpfh' -> global_registration (:68-69); an unknown method prints and returns None, as in the
reference (:70-72).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .keyframe import HostPointCloud, KeyFrame
from .pcd import read_pcd
from .se3 import HomogeneousMatrix

_OPTION = {"icppointpoint": "pointpoint", "icppointplane": "pointplane"}


class KeyFrameManager:
    def __init__(self, directory, scan_times, voxel_size, method="icppointplane", device=None):
        self.directory = directory
        self.scan_times = scan_times
        self.keyframes = []
        self.voxel_size = voxel_size
        self.method = method
        self.show_registration_result = False
        self._dev = device if device is not None else _lib.device()

    # ------------------------------------------------------------------ keyframes
    def add_keyframes(self, keyframe_sampling):
        for i in range(0, len(self.scan_times), keyframe_sampling):
            self.add_keyframe(i)

    def add_keyframe(self, index):
        self.keyframes.append(KeyFrame(directory=self.directory, scan_time=self.scan_times[index],
                                       voxel_size=self.voxel_size, device=self._dev))

    def load_pointclouds(self):
        """keyframemanager.py:32-35. The scans not already resident are read, then uploaded as
        one batch (lsm_cloud_upload_batch: one device allocation and one synchronisation; the
        allocation is freed with the last of the batch's clouds, so unloading single keyframes
        of a batch returns their memory only when the whole batch is unloaded)."""
        todo = [kf for kf in self.keyframes
                if kf._dev is self._dev and not kf.resident(kf.pcd_path())]
        if todo:
            xyzs = [read_pcd(kf.pcd_path()) for kf in todo]
            for kf in todo:
                kf._release()
            for kf, xyz, h in zip(todo, xyzs, self._dev.upload_many(xyzs)):
                kf._attach(h, xyz, kf.pcd_path())
        for kf in self.keyframes:
            kf.load_pointcloud()     # keyframes on another device; no-op for the resident ones

    def load_pointcloud(self, i):
        self.keyframes[i].load_pointcloud()

    def unload_pointcloud(self, i):
        self.keyframes[i].unload_pointcloud()

    def pre_process(self, index):
        self.keyframes[index].pre_process(method=self.method)

    def pre_process_batch(self, indices):
        """pre_process for many keyframes in one device pass (identical results)."""
        kfs = [self.keyframes[i] for i in indices]
        if self.method not in _OPTION:
            for kf in kfs:
                kf.pre_process(method=self.method)
            return
        from .keyframe import DevicePointCloud
        normals = self.method == "icppointplane"
        # one device pass per distinct parameter set (each keyframe keeps its own voxel size,
        # normal radius and filter bounds, exactly as KeyFrame.pre_process would use them)
        groups = {}
        for kf in kfs:
            if kf._handle is None:
                raise RuntimeError("KeyFrame has no point cloud loaded (call load_pointcloud)")
            key = kf._key(None, None, kf.voxel_size, normals)
            if kf._prep_key != key:
                groups.setdefault(key, []).append(kf)
        for key, group in groups.items():
            prm = group[0]._params(None, None, group[0].voxel_size, normals)
            self._dev.preprocess([kf._handle for kf in group], prm)
            for kf in group:
                kf._prep_key = key
        for kf in kfs:
            kf._release_vn()   # as KeyFrame._run: pointcloud_filtered is the keyframe's cloud
            kf._filter = (None, None)
            kf.pointcloud_filtered = DevicePointCloud(self._dev, kf._handle, normals)

    # ------------------------------------------------------------------ registration
    def compute_transformation(self, i, j, Tij):
        if self.method in _OPTION:
            transform = self.keyframes[i].local_registration_simple(
                self.keyframes[j], initial_transform=Tij.array, option=_OPTION[self.method])
        elif self.method == "icp2planes":
            transform = self.keyframes[i].local_registration_two_planes(
                self.keyframes[j], initial_transform=Tij.array)
        elif self.method == "fpfh":
            transform = self.keyframes[i].global_registration(self.keyframes[j])
        else:
            print("Unknown registration method")
            transform = None
        return transform

    def compute_transformations(self, pairs, Tijs):
        """Batched compute_transformation over independent (i, j) pairs."""
        if self.method == "icp2planes":
            from .keyframe import two_planes_batch
            T, _ = two_planes_batch(self._dev, [(self.keyframes[i], self.keyframes[j])
                                                for i, j in pairs], Tijs)
            return T
        if self.method not in _OPTION:
            return [self.compute_transformation(i, j, T) for (i, j), T in zip(pairs, Tijs)]
        if len(pairs) == 0:
            return []
        prm = self.keyframes[pairs[0][0]].registration_params(_OPTION[self.method])
        # pointcloud_filtered of each keyframe, as local_registration_simple registers
        src = [self.keyframes[j]._filtered_handle() for i, j in pairs]
        tgt = [self.keyframes[i]._filtered_handle() for i, j in pairs]
        if any(h is None for h in src + tgt) or any(
                self.keyframes[k]._prep_key is None for ij in pairs for k in ij):
            raise RuntimeError("registration needs loaded, pre-processed keyframes")
        init = np.stack([np.asarray(getattr(T, "array", T), dtype=np.float64) for T in Tijs])
        res = self._dev.icp_batch(src, tgt, init.reshape(-1, 16), prm)
        for (i, j), r in zip(pairs, res):
            self.keyframes[i].last_registration = r
        return [HomogeneousMatrix(r["transformation"]) for r in res]

    # ------------------------------------------------------------------ maps (§8f row 3)
    def build_map(self, global_transforms, keyframe_sampling=10, radii=None, heights=None):
        """Map of every keyframe, filtered (radii 0.5-35 m, heights +-120 m by default), voxelised
        when the keyframe has a voxel_size, moved to the global frame and concatenated
        (keyframemanager.py:154-184); no rendering.

        As the reference, keyframe i is placed with ``global_transforms[i * keyframe_sampling]``
        (the i-th sampled transform), for every keyframe of the manager: fewer sampled transforms
        than keyframes raises IndexError there (keyframemanager.py:176) and here. The device
        filter and voxel passes are the registration path's own (bit-exact to the oracle); the
        transform and the concatenation run on the host in f64, as Open3D's PointCloud.transform
        and operator+ do."""
        if radii is None:
            radii = [0.5, 35.0]
        if heights is None:
            heights = [-120.0, 120.0]
        sampled_transforms = [global_transforms[i]
                              for i in range(0, len(global_transforms), keyframe_sampling)]
        out = HostPointCloud(np.zeros((0, 3)))
        for i in range(len(self.keyframes)):
            kf = self.keyframes[i]
            kf.filter_radius_height(radii=radii, heights=heights)
            kf.down_sample()
            Ti = sampled_transforms[i]
            out = out + kf.transform(getattr(Ti, "array", Ti))
        return out
