"""Is the synthetic data generation deterministic on this machine? (hash of repeated runs)"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_arvc_amd import synthetic  # noqa: E402

for rep in range(4):
    seq = synthetic.make_sequence(65, seed=3, model=synthetic.HDL64)
    h = hashlib.sha256()
    for s in seq.scans:
        h.update(s.tobytes())
    print(rep, h.hexdigest()[:16], sum(len(s) for s in seq.scans), flush=True)
