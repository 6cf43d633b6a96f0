"""Normals agreement by neighbourhood size: the GPU against both f64 oracles (diagnostics).

For a few scans (the 8k / 64k parity scans and the target keyframes of chosen headline pairs)
prints, per neighbourhood-size bucket, how often the GPU's f32 normal equals the C++ oracle's
(rounded to f32, up to sign) bit for bit, and how often |n . n_ref| > 1 - 1e-6 against the C++
and the NumPy oracle. Small neighbourhoods (n <= 8) take Open3D's own covariance arithmetic on
the device (small_normal / small_normal_from_list), the same arithmetic as the C++ oracle, so they should agree
bit for bit except where the device's and the host's acos / cos round differently.

    python tools/normals_small_check.py [--pairs 333,734,...] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(nrm, c_n, c_cnt, p_n, covs):
    f32 = c_n.astype(np.float32)
    g = nrm.astype(np.float32)
    bit = np.all(g == f32, axis=1) | np.all(g == -f32, axis=1)
    dc = np.abs((nrm * c_n).sum(1))
    dp = np.abs((nrm * p_n).sum(1))
    ev = np.linalg.eigvalsh(covs)
    sep = (ev[:, 1] - ev[:, 0]) > 1e-4 * np.maximum(np.abs(ev[:, 2]), 1e-300)
    out = {}
    for name, m in [("n<3", c_cnt < 3), ("n=3", c_cnt == 3), ("n=4..8", (c_cnt >= 4) & (c_cnt <= 8)),
                    ("n=9..16", (c_cnt >= 9) & (c_cnt <= 16)), ("n>16", c_cnt > 16)]:
        k = int(m.sum())
        if k == 0:
            continue
        out[name] = {"points": k, "bit_equal_cpp": float(bit[m].mean()),
                     "dot_cpp_1e-6": float((dc[m] > 1 - 1e-6).mean()),
                     "dot_numpy_1e-6": float((dp[m] > 1 - 1e-6).mean()),
                     "separated": int(sep[m].sum()),
                     "separated_dot_numpy_min": float(dp[m & sep].min()) if (m & sep).any() else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="333,734,784,825,1136,1608,1620,1707,1901")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import _lib, synthetic
    from oracle import cpu_ref as C
    from oracle import open3d_restated as O
    scans = {"8k seed 21": synthetic.make_sequence(1, seed=21, model=synthetic.VLP16_8K).scans[0],
             "64k seed 2": synthetic.make_sequence(1, seed=2, model=synthetic.HDL64).scans[0]}
    for k in [int(v) for v in args.pairs.split(",") if v]:
        scans[f"seed 3 keyframe {k}"] = synthetic.make_sequence(1, seed=3, model=synthetic.HDL64,
                                                               first_index=k).scans[0]
    dev = _lib.device(0)
    report = {}
    for name, scan in scans.items():
        h = dev.upload(scan)
        dev.preprocess([h], _lib.prep_params())
        xyz, nrm = dev.download(h, normals=True)
        dev.release(h)
        pts = O.filter_radius_height(scan)
        assert np.array_equal(xyz, pts)
        c_n, c_cnt = C.estimate_normals(pts, return_counts=True)
        p_n, _, covs = O.estimate_normals(pts, return_counts=True, return_covs=True)
        report[name] = stats(nrm, c_n, c_cnt, p_n, covs)
        print(name, json.dumps(report[name]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
