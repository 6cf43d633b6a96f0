"""Normals phase statistics (LSM_NORMALS_PHASES): walk steps and members per phase of
hybrid_lane on the first keyframes of the bench's seed-3 HDL-64 sequence (diagnostics).
(needs a diagnostics build: bash tools/build_ab.sh diag -DLSM_DIAG=1, run with LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/diag.so)
"""
import os
import sys

os.environ["LSM_NORMALS_PHASES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seq = synthetic.make_sequence(K, seed=3, model=synthetic.HDL64, processes=16)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.preprocess(ids, _lib.prep_params())
