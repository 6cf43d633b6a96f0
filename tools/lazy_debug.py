"""Per-pass lazy-normals waves and kernel time on the bench's sequence (diagnostics)."""
import os, sys, time
os.environ["LSM_DEBUG_LAZY"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from lidar_slam_arvc_amd import _lib, synthetic
P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
seq = synthetic.make_sequence(P + 1, seed=3, model=synthetic.HDL64, processes=16)
dev = _lib.device(0)
for mode in ("lazy", True):
    ids = [dev.upload(s) for s in seq.scans]
    dev.preprocess(ids, _lib.prep_params(want_normals=mode))
    dev.reset_stats(); dev.set_timing(True)
    dev.preprocess(ids, _lib.prep_params(want_normals=mode))
    r = dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, _lib.icp_params())
    dev.set_timing(False)
    print(mode, {k: round(dev.kernel_stats(k)["ms"], 3) for k in ("normals", "normals_lazy", "normals_mark", "nn")}, flush=True)
    for h in ids: dev.release(h)
