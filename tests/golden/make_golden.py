"""Capture golden vectors from the reference's importable modules (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference

Imports, read-only, the NumPy-only reference modules that sit on or beside the hot path:
artelib.homogeneousmatrix / artelib.tools (SE(3) host math), graphslam.loopclosing (candidate
matching, triplets, triangle check), tools.sampling.sample_times and
eurocreader.eurocreader.EurocReader (CSV schema). Open3D-backed modules (keyframemanager.*) cannot
be imported here (no open3d) and are not used. The fixtures written next to this
script are data only (inputs and the reference's outputs); no reference source is copied.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref_root):
    sys.path.insert(0, ref_root)
    from artelib.euler import Euler
    from artelib.homogeneousmatrix import (HomogeneousMatrix, compute_global_transformations,
                                           compute_relative_transformations)
    from eurocreader.eurocreader import EurocReader
    from graphslam.loopclosing import LoopClosing
    from tools.sampling import sample_times

    rng = np.random.default_rng(1234)
    out = {}

    # ---------------- SE(3): inv, mul, t2v(3), Q, euler, global/relative ----------------
    n = 40
    abg = rng.uniform(-np.pi, np.pi, size=(n, 3))
    abg[:4, 1] = [np.pi / 2, -np.pi / 2, np.pi / 2 - 1e-6, -np.pi / 2 + 2e-5]  # gimbal cases
    pos = rng.normal(scale=10.0, size=(n, 3))
    Ts = [HomogeneousMatrix(pos[i].tolist(), Euler(abg[i].tolist())) for i in range(n)]
    out["se3_abg"] = abg
    out["se3_pos"] = pos
    out["se3_T"] = np.stack([T.array for T in Ts])
    out["se3_inv"] = np.stack([T.inv().array for T in Ts])
    out["se3_mul"] = np.stack([(Ts[i] * Ts[(i + 1) % n]).array for i in range(n)])
    out["se3_t2v"] = np.stack([T.t2v(n=3) for T in Ts])
    out["se3_Q"] = np.stack([np.asarray(T.Q().array, dtype=np.float64) for T in Ts])
    eul = [T.euler() for T in [HomogeneousMatrix(T.array.copy()) for T in Ts]]
    out["se3_euler"] = np.stack([np.stack([e[0].abg, e[1].abg]) for e in eul])
    rel = compute_relative_transformations(Ts)
    out["se3_relative"] = np.stack([T.array for T in rel])
    glob = compute_global_transformations(rel, T0=HomogeneousMatrix(), Trobot_gps=None)
    out["se3_global"] = np.stack([T.array for T in glob])

    # ---------------- sample_times ----------------
    t = np.cumsum(rng.integers(40_000_000, 160_000_000, size=300)).astype(np.int64) + 10 ** 18
    out["st_times"] = t
    for si, dt in [(0, 0.5e9), (10, 1.0e9), (20, 0.3e9)]:
        out[f"st_out_{si}_{int(dt)}"] = sample_times(t, start_index=si, delta_time=dt)

    # ---------------- loop closing ----------------
    class Pose:
        def __init__(self, T):
            self.T = T

        def matrix(self):
            return self.T

    class Estimate:
        def __init__(self, poses):
            self.poses = poses

        def exists(self, i):
            return 0 <= i < len(self.poses)

        def atPose3(self, i):
            return Pose(self.poses[i])

    class FakeGraph:
        def __init__(self, poses, T0_gps):
            self.current_estimate = Estimate(poses)
            self.T0_gps = T0_gps
            self.edges = []

        def add_edge(self, Tij, i, j, kind):
            self.edges.append((int(i), int(j), kind, np.asarray(Tij.array).copy()))

    m = 700
    s = np.linspace(0, 3.2 * np.pi, m)
    traj = np.stack([15 * np.cos(s) + 0.2 * rng.normal(size=m),
                     15 * np.sin(s) + 0.2 * rng.normal(size=m), 0.05 * rng.normal(size=m)], 1)
    yaw = s + np.pi / 2
    poses = []
    for k in range(m):
        T = np.eye(4)
        c, sn = np.cos(yaw[k]), np.sin(yaw[k])
        T[:2, :2] = [[c, -sn], [sn, c]]
        T[:3, 3] = traj[k]
        poses.append(T)
    poses = np.stack(poses)
    out["lc_poses"] = poses
    T0_gps = HomogeneousMatrix([0.36, 0.0, 0.0], Euler([0, 0, 0.01]))
    out["lc_T0_gps"] = T0_gps.array
    cases = []
    for cur in [50, 200, 350, 420, 560, 699]:
        g = FakeGraph(list(poses[:cur + 1]), T0_gps)
        lc = LoopClosing(g, distance_backwards=9.0, radius_threshold=2.0)
        cand = lc.find_candidates()
        trip = lc.find_feasible_triplets(current_index=cur)
        cases.append({"current": cur, "index_backwards": lc.find_index_backwards(),
                      "candidates": [int(c) for c in cand],
                      "triplets": [[int(a), int(b), int(c)] for a, b, c in trip]})
    out_json = {"loop_cases": cases}

    # loop_closing_triangle with canned ICP results: the fake manager returns the estimate's own
    # relative transform perturbed deterministically, so some triplets pass and some fail
    class FakeKFM:
        def __init__(self, poses, T0_gps):
            self.poses = poses
            self.T0_gps = T0_gps
            self.calls = []

        def load_pointcloud(self, i):
            pass

        def pre_process(self, i):
            pass

        def compute_transformation(self, i, j, Tij):
            self.calls.append((int(i), int(j)))
            bump = HomogeneousMatrix([0.002 * ((i + j) % 7), 0.0, 0.0],
                                     Euler([0, 0, 0.004 * ((i * j) % 5)]))
            return Tij * bump

    tri_cases = []
    for cur, seed in [(420, 7), (560, 11), (699, 3)]:
        g = FakeGraph(list(poses[:cur + 1]), T0_gps)
        lc = LoopClosing(g, distance_backwards=9.0, radius_threshold=2.0)
        kfm = FakeKFM(poses, T0_gps)
        np.random.seed(seed)
        added = lc.loop_closing_triangle(cur, 20, kfm)
        tri_cases.append({"current": cur, "seed": seed,
                          "added": [[int(a), int(b)] for a, b in (added or [])],
                          "icp_calls": kfm.calls,
                          "edges": [[e[0], e[1], e[2], e[3].tolist()] for e in g.edges]})
    out_json["triangle_cases"] = tri_cases

    # loop_closing_simple (loopclosing.py:33-56): candidates sampled with np.random.choice under
    # np.random.seed, one canned registration per sampled candidate, one 'SM' edge each
    simple_cases = []
    for cur, seed, ncand in [(420, 5, 6), (560, 9, 4), (699, 2, 30), (50, 1, 6)]:
        g = FakeGraph(list(poses[:cur + 1]), T0_gps)
        lc = LoopClosing(g, distance_backwards=9.0, radius_threshold=2.0)
        kfm = FakeKFM(poses, T0_gps)
        np.random.seed(seed)
        try:
            lc.loop_closing_simple(cur, ncand, kfm)
            err = None
        except Exception as e:   # (no candidates: np.random.choice of an empty list works)
            err = type(e).__name__
        simple_cases.append({"current": cur, "seed": seed, "number_of_candidates": ncand,
                             "error": err, "icp_calls": kfm.calls,
                             "edges": [[e[0], e[1], e[2], e[3].tolist()] for e in g.edges]})
    out_json["simple_cases"] = simple_cases

    # ---------------- EuRoC CSV schema ----------------
    with tempfile.TemporaryDirectory() as d:
        er = EurocReader(d)
        times = t[:5]
        er.save_transforms_as_csv(times, Ts[:5], filename="/robot0/sm/rel.csv")
        er.save_sensor_times_as_csv(times, filename="/robot0/sm/times.csv")
        er.save_loop_closures_as_csv([[[1, 2], [3, 4]], None, [[5, 6]]], filename="/robot0/lc.csv")
        with open(d + "/robot0/sm/rel.csv") as f:
            out_json["csv_transforms"] = f.read()
        with open(d + "/robot0/sm/times.csv") as f:
            out_json["csv_times"] = f.read()
        with open(d + "/robot0/lc.csv") as f:
            out_json["csv_loop_closures"] = f.read()

    np.savez_compressed(os.path.join(HERE, "reference_goldens.npz"), **out)
    with open(os.path.join(HERE, "reference_goldens.json"), "w") as f:
        json.dump(out_json, f, indent=1)
    print("wrote", len(out), "arrays,", len(cases), "loop cases,", len(tri_cases),
          "triangle cases,", len(simple_cases), "simple cases")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
