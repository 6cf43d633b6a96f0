"""Fixture generator (test infrastructure): the NumPy/SciPy oracle (oracle/open3d_restated.py,
a restatement of Open3D's registration_icp / EstimateNormals) on 32 pairs of bench.py's headline
workload, the seed-3 HDL-64 sequence (keyframe.py:246-252 via run_scanmatcher.py:196-213).

The pairs: 8 of the 53 pairs on which the C++ oracle (tests/golden/seed3_seq_cpu_oracle.npz,
tools/bench_parity.py --make-cpu) hits max_iteration = 30 without converging, and 24 of the
converging ones drawn with a fixed seed. Each pair's two scans are regenerated alone
(synthetic.make_sequence(2, first_index=k): the same data as inside the 2000-keyframe sequence)
and their SHA-256 is stored, so tests/test_gpu_headline.py proves it registers the same clouds.

    python tests/golden/make_seed3_oracle.py     (about 2 minutes on 8 cores)
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from lidar_slam_arvc_amd import synthetic  # noqa: E402
from oracle import open3d_restated as O  # noqa: E402


def pair_sha(seq) -> str:
    h = hashlib.sha256()
    for s in seq.scans:
        h.update(np.ascontiguousarray(s, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(seq.priors, dtype=np.float64).tobytes())
    return h.hexdigest()


def main():
    cpu = np.load(os.path.join(HERE, "seed3_seq_cpu_oracle.npz"))
    it = cpu["iterations"]
    nonconv = np.flatnonzero(it >= 30)
    conv = np.flatnonzero(it < 30)
    rng = np.random.default_rng(0)
    pairs = np.sort(np.r_[nonconv[:8], rng.choice(conv, 24, replace=False)])
    out = {k: [] for k in ("transformation", "fitness", "inlier_rmse", "iterations", "n_corr")}
    shas = []
    t0 = time.time()
    for k in pairs:
        seq = synthetic.make_sequence(2, seed=3, model=synthetic.HDL64, first_index=int(k))
        shas.append(pair_sha(seq))
        tgt = O.filter_radius_height(seq.scans[0])
        src = O.filter_radius_height(seq.scans[1])
        r = O.registration_icp(src, tgt, 10.0, seq.priors[0], "p2plane", O.estimate_normals(tgt))
        for key in out:
            out[key].append(r[key])
        dR = np.abs(r["transformation"][:3, :3] - cpu["transformation"][k][:3, :3]).max()
        dt = np.abs(r["transformation"][:3, 3] - cpu["transformation"][k][:3, 3]).max()
        print(f"pair {k:4d}: iters {r['iterations']:2d} (C++ {it[k]:2d})  vs C++ oracle "
              f"|dR| {dR:.2e} |dt| {dt:.2e}  ({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, "seed3_pairs_o3d_oracle.npz"), pairs=pairs,
                        sha256=np.asarray(shas),
                        **{k: np.asarray(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
