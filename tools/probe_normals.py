"""Time the grid + normals stages on the bench workload (65 HDL-64 scans) under different
(radius, max_nn) settings: python tools/probe_normals.py [r:max_nn ...]"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from lidar_slam_arvc_amd import _lib, synthetic

seq = synthetic.make_sequence(65, seed=int(os.environ.get("SEED", "3")), model=synthetic.HDL64)
dev = _lib.device(0)
ids = [dev.upload(s) for s in seq.scans]
CASES = [(0.3, 300), (0.3, 100000)]
if len(sys.argv) > 1:
    CASES = [tuple(t(v) for t, v in zip((float, int), a.split(':'))) for a in sys.argv[1:]]
for r, mnn in CASES:
    prep = _lib.prep_params(normal_radius=r, max_nn=mnn)
    dev.preprocess(ids, prep)
    dev.reset_stats(); dev.set_timing(True)
    for _ in range(5):
        dev.preprocess(ids, prep)
    dev.set_timing(False)
    st = {k: dev.kernel_stats(k)["ms"] / 5 for k in ("grid", "normals")}
    print(f"r={r} max_nn={mnn}: " + " ".join(f"{k}={v:.3f}ms" for k, v in st.items()), flush=True)
if os.environ.get("LSM_NORMALS_STATS"):
    dev.reset_stats()
    dev.preprocess(ids, _lib.prep_params())
    names = ["ns_points", "ns_scan1_iters", "ns_selecting", "ns_refines", "ns_refine_iters",
             "ns_final_iters", "ns_box"]
    v = {k: dev.kernel_stats(k)["launches"] for k in names}
    n = v["ns_points"]
    print({k: round(x / n, 3) for k, x in v.items()}, "per point; selecting:",
          v["ns_selecting"], "final iters per selecting", v["ns_final_iters"] / max(v["ns_selecting"], 1))
