"""Exactness probe of the NN search variants (env knobs read at library load): register the
bench's HDL-64 sequence pairs and save every result, so runs under different LSM_NN_* settings
can be compared bit for bit. usage: python tools/split_check.py OUT.npz [pairs]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

out = sys.argv[1]
P = int(sys.argv[2]) if len(sys.argv) > 2 else 64
seq = synthetic.make_sequence(P + 1, seed=3)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.preprocess(ids, _lib.prep_params(want_normals=True))
res = dev.icp_batch(ids[1:], ids[:-1], seq.priors, _lib.icp_params(method="p2plane"))
T = np.stack([r["transformation"] for r in res])
it = np.array([r["iterations"] for r in res])
fit = np.array([r["fitness"] for r in res])
rm = np.array([r["inlier_rmse"] for r in res])
np.savez(out, T=T, it=it, fit=fit, rmse=rm, corr=dev.last_correspondences())
print(out, "mean iterations", it.mean(), "max", it.max())
