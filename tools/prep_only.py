"""Pre-process a bench-sized keyframe batch a few times (profiling target for the normals)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LSM_NORMALS_STATS", "1")
from lidar_slam_arvc_amd import _lib, synthetic  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 65
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
seq = synthetic.make_sequence(K, seed=3, model=synthetic.HDL64)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
dev.set_timing(True)
for _ in range(reps):
    n = dev.preprocess(ids, _lib.prep_params())
st = dev.kernel_stats("normals")
tr = dev.kernel_stats("normals_truncated")
print(f"points {sum(n) / len(n):.0f}/scan, normals {st['ms'] / reps:.3f} ms per batch of {K}, "
      f"truncated {tr['launches'] / reps / sum(n):.4f} of points")
