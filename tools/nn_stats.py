"""Per-pass NN search statistics (LSM_NN_STATS, LSM_DEBUG_PASSES) on the first pairs of the
bench's seed-3 sequence (diagnostics): python tools/nn_stats.py [P]
(needs a diagnostics build: bash tools/build_ab.sh diag -DLSM_DIAG=1, run with LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/diag.so)
"""
import os
import sys

os.environ["LSM_NN_STATS"] = "1"
os.environ["LSM_DEBUG_PASSES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
seq = synthetic.make_sequence(P + 1, seed=3, model=synthetic.HDL64, processes=16)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.preprocess(ids, _lib.prep_params())
dev.set_timing(True)
r = dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, _lib.icp_params())
print({k: round(dev.kernel_stats(k)["ms"], 3) for k in ("nn", "nn_fallback", "accumulate")})
