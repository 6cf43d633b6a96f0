"""Per-pass counters of one timed bench-sized ICP batch (LSM_DEBUG_PASSES=1 prints them)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LSM_DEBUG_PASSES"] = "1"
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 64
method = sys.argv[2] if len(sys.argv) > 2 else "p2plane"
seq = synthetic.make_sequence(P + 1, seed=3, model=synthetic.HDL64)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.preprocess(ids, _lib.prep_params(want_normals=(method == "p2plane")))
dev.set_timing(True)
res = dev.icp_batch(ids[1:], ids[:-1], seq.priors, _lib.icp_params(method=method))
it = np.array([r["iterations"] for r in res])
print("iterations:", np.bincount(it).tolist(), "mean", it.mean())
print("slow pairs:", np.nonzero(it >= 20)[0].tolist())
