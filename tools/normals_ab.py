"""Normals time of one bench chunk (250 HDL-64 keyframes pre-processed as one batch), per library
variant: python tools/normals_ab.py [reps]  (LIDARSM_LIB selects the library; the scans come from
bench.py's --seq-cache file when it exists)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

K = 250
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cache = "/tmp/lsm_seq.npz"
if os.path.exists(cache):
    z = np.load(cache)
    scans = [z[f"s{k}"] for k in range(K)]
else:
    scans = synthetic.make_sequence(K, seed=3, model=synthetic.HDL64, processes=16).scans
dev = _lib.device(0)
ids = [dev.upload(s) for s in scans]
dev.preprocess(ids, _lib.prep_params())   # warm-up
dev.set_timing(True)
for _ in range(reps):
    dev.preprocess(ids, _lib.prep_params())
out = {k: dev.kernel_stats(k)["ms"] / reps for k in ("normals", "grid", "filter")}
print(os.environ.get("LIDARSM_LIB", "in-tree"), {k: round(v, 3) for k, v in out.items()})
