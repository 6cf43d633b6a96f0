"""Coarse-to-fine (multi-scale) registration: config C5 of BASELINE.json.

The reference registers at one scale only: ``KeyFrame.pre_process`` filters, optionally
voxel-downsamples (``voxel_down_sample(voxel_size)``, keyframe.py:150-151 / :158-159) and
estimates normals (:160-162), then ``local_registration_simple`` runs one
``registration_icp`` (keyframe.py:231-260). A multi-scale chain is that same single-scale
registration repeated on voxel grids of decreasing size, each stage starting from the previous
stage's transform -- so every stage is exactly the reference's operator, and every stage is
parity-checked against the oracle's own chain (``oracle.open3d_restated.registration_multiscale``).

Device flow: each raw scan stays resident once; per scale, a device clone of it
(``lsm_cloud_clone``) is filtered + voxelised + normal-estimated in one batched pre-process, and
all pairs of a stage run as one ICP batch.
"""
from __future__ import annotations

import numpy as np

from . import _lib

DEFAULT_SCALES = (0.4, 0.2, 0.1)          # voxel sizes, metres
DEFAULT_MAX_CORR = (2.0, 1.0, 0.5)        # max_correspondence_distance per stage


class MultiScaleSet:
    """Per-scale device clones of a list of resident raw scans (``Device.upload`` handles)."""

    def __init__(self, dev, raw_handles, scales=DEFAULT_SCALES):
        self.dev = dev
        self.scales = tuple(float(v) for v in scales)
        if not self.scales or any(not v > 0 for v in self.scales):
            raise ValueError("scales must be positive voxel sizes")
        self.raw = [int(h) for h in raw_handles]
        self.handles = []
        try:
            for _ in self.scales:
                self.handles.append([dev.clone(h) for h in self.raw])
        except Exception:
            self.release()
            raise

    def preprocess(self, want_normals=True, grid_cells=None, **prep_kwargs):
        """KeyFrame.pre_process at every scale: filter -> voxel_down_sample(v) -> normals.
        grid_cells: the spatial grid's cell per scale (None: ``grid_cell`` of prep_kwargs, or the
        library's choice); the grid only indexes the points, results do not depend on it."""
        if grid_cells is not None:
            grid_cells = tuple(float(c) for c in grid_cells)
            if len(grid_cells) != len(self.scales):
                raise ValueError("one grid cell per scale")
            prep_kwargs.pop("grid_cell", None)
        for k, (v, hs) in enumerate(zip(self.scales, self.handles)):
            kw = dict(prep_kwargs)
            if grid_cells is not None:
                kw["grid_cell"] = grid_cells[k]
            self.dev.preprocess(hs, _lib.prep_params(voxel_size=v, want_normals=want_normals, **kw))

    def register(self, src_idx, tgt_idx, inits=None, max_corr=DEFAULT_MAX_CORR,
                 method="p2plane", max_iteration=30, arrays=False):
        """Pairs (src_idx[k] onto tgt_idx[k], indices into raw_handles) through every scale.
        Returns the per-stage lists of :meth:`Device.icp_batch` result dicts (``arrays``: the
        per-stage dicts of arrays of :meth:`Device.icp_batch_arrays`, no per-pair objects)."""
        max_corr = tuple(float(d) for d in max_corr)
        if len(max_corr) != len(self.scales):
            raise ValueError("one max_correspondence_distance per scale")
        P = len(src_idx)
        if P != len(tgt_idx):
            raise ValueError("src_idx and tgt_idx must have the same length")
        if P == 0:
            return [[] for _ in self.scales]
        T = (np.broadcast_to(np.eye(4), (P, 4, 4)).copy() if inits is None
             else np.asarray(inits, dtype=np.float64).reshape(P, 4, 4).copy())
        stages = []
        for hs, dmax in zip(self.handles, max_corr):
            prm = _lib.icp_params(method=method, max_correspondence_distance=dmax,
                                  max_iteration=max_iteration)
            src = [hs[i] for i in src_idx]
            tgt = [hs[i] for i in tgt_idx]
            if arrays:
                res = self.dev.icp_batch_arrays(src, tgt, T.reshape(P, 16), prm)
                T = res["transformation"]
            else:
                res = self.dev.icp_batch(src, tgt, T.reshape(P, 16), prm)
                T = np.stack([r["transformation"] for r in res])
            stages.append(res)
        return stages

    def release(self):
        for hs in self.handles:
            for h in hs:
                self.dev.release(h)
        self.handles = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()


def register_multiscale(dev, sources, targets, inits=None, scales=DEFAULT_SCALES,
                        max_corr=DEFAULT_MAX_CORR, method="p2plane", max_iteration=30,
                        return_stages=False):
    """Register ``sources[k]`` onto ``targets[k]`` (raw device handles from ``Device.upload``)
    through the voxel ``scales`` (coarse to fine). ``inits``: P x 4 x 4 (None -> identity).

    Returns the P final result dicts (the last stage's); with ``return_stages`` also the
    per-stage lists.
    """
    sources = [int(h) for h in sources]
    targets = [int(h) for h in targets]
    raw = list(dict.fromkeys(sources + targets))          # unique, order-preserving
    pos = {h: k for k, h in enumerate(raw)}
    with MultiScaleSet(dev, raw, scales) as ms:
        ms.preprocess(want_normals=(method == "p2plane"))
        stages = ms.register([pos[h] for h in sources], [pos[h] for h in targets], inits,
                             max_corr, method, max_iteration)
    final = stages[-1] if stages else []
    return (final, stages) if return_stages else final
