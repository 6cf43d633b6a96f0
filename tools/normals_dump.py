"""Pre-process K HDL-64 scans (normals r=0.3/max_nn=300 and FPFH r=0.3/max_nn=100 lists) and save
the downloaded normals / FPFH features: python tools/normals_dump.py OUT.npz [K]. Comparing two
library builds' dumps (tools/npz_same.py) checks that a normals-kernel change is bit-identical."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
seq = synthetic.make_sequence(K, seed=3, model=synthetic.HDL64)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.preprocess(ids, _lib.prep_params())
out = {}
for k, h in enumerate(ids):
    pts, nrm = dev.download(h, normals=True)
    out[f"n{k}"] = nrm
    out[f"f{k}"] = dev.fpfh(h, 0.3, 100)
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], K, "scans")
