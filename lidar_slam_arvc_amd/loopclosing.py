"""LoopClosing drop-in (reference: graphslam/loopclosing.py) with device candidate matching and
batched ICP.

Same constructor and methods as the reference class. What moves to the GPU:

* ``find_candidates`` (:213-221) = store_positions (:202-211) + find_index_backwards (:223-237) +
  find_candidates_within_radius (:239-253): one liblidarsm call (lsm_loop_candidates), bit-exact
  with the reference's NumPy arithmetic;
* ``find_feasible_triplets`` (:102-117) + ``look_for_valid_indexes`` (:131-144): one call
  (lsm_loop_triplet_partners);
* the <= 2 * number_of_triplets ICP registrations of ``loop_closing_triangle`` (:80-99): gathered
  into ONE batch (pairs de-duplicated; results are deterministic, so a repeated pair would give
  the same transform) instead of sequential calls that re-read and re-pre-process both clouds
  each time (:163-178).

The triplet sampling keeps the reference's ``np.random.choice`` on NumPy's global RNG, so a
seeded run picks the same triplets. The pose-graph back end (GTSAM) stays on the CPU; this
class only reads ``current_estimate`` / ``T0_gps`` and calls ``add_edge`` like the reference.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .se3 import HomogeneousMatrix


class LoopClosing:
    def __init__(self, graphslam, distance_backwards=7, radius_threshold=5.0, device=None):
        self.graphslam = graphslam
        self.distance_backwards = distance_backwards
        self.radius_threshold = radius_threshold
        self.positions = None
        self._dev = device

    @property
    def dev(self):
        if self._dev is None:
            self._dev = _lib.device()
        return self._dev

    # ------------------------------------------------------------------ candidates (GPU)
    def store_positions(self):
        poses = []
        i = 0
        est = self.graphslam.current_estimate
        while est.exists(i):
            poses.append(np.asarray(est.atPose3(i).matrix(), dtype=np.float64)[0:3, 3])
            i += 1
        self.positions = np.array(poses).reshape(-1, 3)

    def _candidates(self):
        idx, cand = self.dev.loop_candidates(self.positions, self.distance_backwards,
                                             self.radius_threshold)
        return idx, cand

    def find_candidates(self):
        self.store_positions()
        return self._candidates()[1]

    def find_index_backwards(self):
        return self._candidates()[0]

    def find_candidates_within_radius(self, index):
        if index is None:
            return []
        return self._candidates()[1]

    def find_feasible_triplets(self, current_index):
        candidates = np.sort(self.find_candidates())
        if len(candidates) == 0:
            return []
        partners = self.dev.loop_partners(self.positions, candidates)
        return [[current_index, int(j1), int(j2)] for j1, j2 in zip(candidates, partners)
                if j2 >= 0]

    def distance(self, i, j):
        est = self.graphslam.current_estimate
        pi = HomogeneousMatrix(est.atPose3(i).matrix()).pos()
        pj = HomogeneousMatrix(est.atPose3(j).matrix()).pos()
        return np.linalg.norm(pi - pj)

    def look_for_valid_indexes(self, i, rest_of_candidates):
        for u in rest_of_candidates:
            if 1 < abs(u - i) < 80 and 1.0 < self.distance(i, u) < 2.0:
                return u
        return None

    # ------------------------------------------------------------------ host SE(3) logic
    def check_distances(self, I):
        dp = np.linalg.norm(I.pos())
        e1, e2 = I.euler()
        da = min([np.linalg.norm(e1.abg), np.linalg.norm(e2.abg)])
        return bool(dp < 0.1 and da < 0.05)

    def add_loop_closing_observation(self, i, j, Tij):
        self.graphslam.add_edge(Tij, i, j, "SM")

    def _lidar_relative(self, i, j):
        T0_gps = self.graphslam.T0_gps
        est = self.graphslam.current_estimate
        Ti = HomogeneousMatrix(est.atPose3(i).matrix()) * T0_gps.inv()
        Tj = HomogeneousMatrix(est.atPose3(j).matrix()) * T0_gps.inv()
        return Ti.inv() * Tj

    def compute_consecutive_transformations(self, i, j):
        return self._lidar_relative(i, j)

    def compute_transformations_between_candidates(self, i, j, keyframe_manager):
        return self.compute_transformations_batch([(i, j)], keyframe_manager)[(i, j)]

    def compute_transformations_batch(self, pairs, keyframe_manager):
        """ICP for many (i, j) candidate pairs in one batch; returns {(i, j): T (robot frame)}."""
        T0_gps = self.graphslam.T0_gps
        uniq = list(dict.fromkeys((int(i), int(j)) for i, j in pairs))
        for k in sorted({x for p in uniq for x in p}):
            keyframe_manager.load_pointcloud(k)
        if hasattr(keyframe_manager, "pre_process_batch"):
            keyframe_manager.pre_process_batch(sorted({x for p in uniq for x in p}))
        else:
            for k in sorted({x for p in uniq for x in p}):
                keyframe_manager.pre_process(k)
        inits = [self._lidar_relative(i, j) for i, j in uniq]
        if hasattr(keyframe_manager, "compute_transformations"):
            res = keyframe_manager.compute_transformations(uniq, inits)
        else:
            res = [keyframe_manager.compute_transformation(i, j, Tij=T)
                   for (i, j), T in zip(uniq, inits)]
        return {p: T0_gps.inv() * T * T0_gps for p, T in zip(uniq, res)}

    # ------------------------------------------------------------------ drivers
    def loop_closing_simple(self, current_index, number_of_candidates_DA, keyframe_manager):
        candidates = self.find_candidates()
        i = current_index
        n = np.min([len(candidates), number_of_candidates_DA])
        candidates = np.random.choice(candidates, size=n, replace=False)
        res = self.compute_transformations_batch([(i, j) for j in candidates], keyframe_manager)
        for j in candidates:
            self.add_loop_closing_observation(i=i, j=j, Tij=res[(int(i), int(j))])

    def loop_closing_triangle(self, current_index, number_of_triplets_loop_closing,
                              keyframe_manager):
        triplets = self.find_feasible_triplets(current_index=current_index)
        if len(triplets) == 0:
            return
        n = np.min([len(triplets), number_of_triplets_loop_closing])
        sampled = np.random.choice(range(len(triplets)), size=n, replace=False)
        pairs = []
        for k in sampled:
            i, j1, j2 = triplets[k]
            pairs += [(i, j1), (i, j2)]
        res = self.compute_transformations_batch(pairs, keyframe_manager)
        added = []
        for k in sampled:
            i, j1, j2 = triplets[k]
            Tij1, Tij2 = res[(int(i), int(j1))], res[(int(i), int(j2))]
            Tj1j2 = self.compute_consecutive_transformations(i=j1, j=j2)
            I = Tij1 * Tj1j2 * Tij2.inv()
            if self.check_distances(I):
                self.add_loop_closing_observation(i=i, j=j1, Tij=Tij1)
                self.add_loop_closing_observation(i=i, j=j2, Tij=Tij2)
                added.append([i, j1])
                added.append([i, j2])
        return added
