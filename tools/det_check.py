"""Determinism check: synthetic data hash + device filter counts across repeated pre-processes."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402
from oracle import open3d_restated as O  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 65
seq = synthetic.make_sequence(K, seed=3, model=synthetic.HDL64)
h = hashlib.sha256()
for s in seq.scans:
    h.update(s.tobytes())
print("data sha", h.hexdigest()[:16], "rows", sum(len(s) for s in seq.scans))
ref = np.array([len(O.filter_radius_height(s)) for s in seq.scans])
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
for rep in range(3):
    n = dev.preprocess(ids, _lib.prep_params(want_normals=False))
    print("rep", rep, "device total", int(n.sum()), "oracle total", int(ref.sum()),
          "mismatching clouds", int((n != ref).sum()))
