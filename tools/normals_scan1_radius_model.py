"""CPU model: can the dense half's scan 1 walk a smaller ball first?

The dense half (prep.hip normals_dense_kernel, hybrid kNN-300 / r 0.3 m) walks the whole r-ball
in scan 1 to build the 128-bin histogram of d^2 over [0, r^2), picks the bin holding the 300th
neighbour, and walks the ball of that bin's upper edge again in the final pass. The bins below a
radius rh are complete after a walk of the rh-ball alone: if they already hold > max_nn points,
the chosen bin -- and so everything after it -- is the one the full walk picks (bit-identical
by construction). Otherwise scan 1 walks the full ball as now. This replays both walks on bench
scans with the round-6 grid (0.42 m x / z, 0.21 m y) and reports, per predictor of rh:

  * the success rate (bins below rh hold >= max_nn + 1 points, the query included);
  * scan-1 walk steps per dense point (rh-ball always; plus the r-ball on a failure) against the
    full walk, and the final pass's steps for scale.

Predictors: a fixed rh; rh from the own cell's population (a bucketed 97th percentile of the
needed radius, fitted on the first scan and applied to the others).

    python tools/normals_scan1_radius_model.py [--scans 3] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from normals_pitch_model import AnisoGrid, R, MAX_NN, NB8   # noqa: E402

CX, CY = 0.42, 0.21     # LSM_DEFAULT_GRID_CELL, y half (LSM_YSUB_SHIFT 1)


def covered_edge(rh):
    """d^2 below which every level-0 bin is complete after walking the rh-ball"""
    return np.floor(np.minimum(rh, R) ** 2 * NB8 / R ** 2) * R ** 2 / NB8


def needed_radius(d2_301):
    """smallest rh whose covered bins hold the 301st point: the upper edge of its bin"""
    b = np.floor(d2_301 * NB8 / R ** 2) + 1
    return np.sqrt(np.minimum(b, NB8) * R ** 2 / NB8)


def scan(pts):
    """the dense list: points the own-cell population predicts dense (prep.hip predict_dense:
    n_c >= 0.27 * max_nn / r^2 * cx * cy), truly dense or not"""
    tree = cKDTree(pts)
    cnt = tree.query_ball_point(pts, R, return_length=True)
    o = pts.min(axis=0)
    ijk = np.floor((pts - o) / np.array([CX, CY, CX])).astype(np.int64)
    key = (ijk[:, 2] * 100000 + ijk[:, 1]) * 100000 + ijk[:, 0]
    _, inv, cc = np.unique(key, return_inverse=True, return_counts=True)
    nc_all = cc[inv]
    listed = np.nonzero(nc_all >= 0.27 * MAX_NN / R ** 2 * CX * CY)[0]
    q = pts[listed]
    dense = cnt[listed] > MAX_NN
    d = tree.query(q, k=MAX_NN + 1)[0]
    # a truly sparse point never succeeds (its covered bins cannot hold max_nn + 1 points)
    need = np.where(dense, needed_radius(d[:, -1] ** 2), np.inf)
    d300 = d[:, MAX_NN - 1]
    rfin = np.where(dense, np.sqrt(np.minimum(np.floor(d300 ** 2 * NB8 / R ** 2) + 1, NB8) *
                                   R ** 2 / NB8), R)
    g = AnisoGrid(pts, CY, CX, CX)
    full = g.walk(q, np.full(len(q), R))["steps"]
    fin = g.walk(q, rfin)["steps"]
    return dict(q=q, g=g, need=need, ncell=nc_all[listed], full=full, fin=fin, n=len(pts),
                truly_dense=float(dense.mean()))


def evaluate(s, rh):
    ok = (rh >= s["need"] - 1e-12) | (rh >= R)   # rh = r: the full walk itself
    part = s["g"].walk(s["q"], rh)["steps"]
    cost = part + np.where(ok, 0.0, s["full"])
    return {"success": float(ok.mean()), "scan1_steps": float(cost.mean()),
            "deferred_full_scans": float((~ok).mean()),
            "scan1_vs_full": float(cost.mean() / s["full"].mean()),
            "dense_vs_now": float((cost.mean() + s["fin"].mean()) /
                                  (s["full"].mean() + s["fin"].mean()))}


def fit_buckets(s, q=97.0):
    edges = np.unique(np.percentile(s["ncell"], np.linspace(0, 100, 11)))
    b = np.clip(np.searchsorted(edges, s["ncell"], "right") - 1, 0, len(edges) - 2)
    fin = np.isfinite(s["need"])
    rad = np.array([min(np.percentile(s["need"][(b == i) & fin], q), R)
                    if ((b == i) & fin).any() else R for i in range(len(edges) - 1)])
    return edges, rad


def apply_buckets(s, edges, rad):
    b = np.clip(np.searchsorted(edges, s["ncell"], "right") - 1, 0, len(edges) - 2)
    return rad[b]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=3)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import synthetic
    from oracle import cpu_ref as C
    seq = synthetic.make_sequence(args.scans, seed=3, model=synthetic.HDL64, processes=4)
    t0 = time.time()
    scans = [scan(C.filter_radius_height(seq.scans[k])) for k in range(args.scans)]
    print(f"scans modelled in {time.time() - t0:.0f} s", flush=True)
    res = {"grid": {"x": CX, "y": CY, "z": CX}, "r": R, "max_nn": MAX_NN, "per_scan": []}
    for k, s in enumerate(scans):
        e = {"points": s["n"], "listed": int(len(s["q"])), "listed_truly_dense": s["truly_dense"],
             "full_scan1_steps": float(s["full"].mean()), "final_steps": float(s["fin"].mean()),
             "needed_radius_pct": {p: float(np.percentile(s["need"], p))
                                   for p in (10, 50, 90, 97, 99)},
             "fixed": {}, "own_cell": {}}
        for rh in (0.22, 0.24, 0.25, 0.26, 0.27, 0.28):
            e["fixed"][str(rh)] = evaluate(s, np.full(len(s["q"]), rh))
        for qq in (90.0, 95.0, 97.0, 99.0):
            edges, rad = fit_buckets(scans[0], qq)
            e["own_cell"][str(qq)] = evaluate(s, apply_buckets(s, edges, rad))
        # the planar-density form the kernel can compute for any (r, max_nn, cell): the own cell
        # holds n_c points of a surface crossing its cx * cz face, so max_nn points lie within
        # rh^2 = kappa * max_nn * cx * cz / (pi * n_c); kappa from the first scan's percentiles
        fin_ = np.isfinite(s["need"])
        kap = s["need"][fin_] ** 2 * np.pi * s["ncell"][fin_] / (MAX_NN * CX * CX)
        e["kappa_pct"] = {p: float(np.percentile(kap, p)) for p in (50, 90, 95, 97, 99)}
        f0 = np.isfinite(scans[0]["need"])
        k0 = scans[0]["need"][f0] ** 2 * np.pi * scans[0]["ncell"][f0] / (MAX_NN * CX * CX)
        e["density"] = {}
        for qq in (90.0, 95.0, 97.0):
            kappa = float(np.percentile(k0, qq))
            rh = np.sqrt(np.minimum(kappa * MAX_NN * CX * CX / (np.pi * s["ncell"]), R * R))
            e["density"][f"{qq} (kappa {kappa:.2f})"] = evaluate(s, rh)
        res["per_scan"].append(e)
        print(json.dumps({kk: v for kk, v in e.items() if kk not in ("fixed", "own_cell", "density")}))
        for name in ("fixed", "own_cell", "density"):
            for kk, v in e[name].items():
                print(f"  {name:8s} {kk:>5}: success {v['success']:.3f}  scan1 {v['scan1_vs_full']:.3f}x"
                      f"  dense walks {v['dense_vs_now']:.3f}x")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
