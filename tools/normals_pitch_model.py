"""CPU model: would a y/z cell pitch finer than the x pitch cut the normals' walk steps?

VERDICT r5 item 1. The normals walk a ball (radius r = 0.3 m) as rows of grid cells: every (y, z)
cell row the ball's box touches (pruned by its slab distance), each row's points in the x window of
the chord at the row's nearest slab (prep.hip ball_visit_runs / scan_run_pred). With 0.375 m cells
a row is 0.375 m wide in y and z, so a planar patch is walked over about twice the disc's area.
This replays those walks on bench scans for anisotropic cells -- x pitch 0.375 m (64-cell blocks),
y / z pitch P -- and counts per point:

  * scan 1 (every point, r = 0.3 m): rows visited (non-empty row parts = row setups: two
    cell-table loads each), entry-search rounds (4-ary, while a run holds > 16 points, down to 8),
    walk steps (points the walk loads: the window's points, the entry search's slack before it,
    the stop point past it);
  * the final pass (dense points: > max_nn in the ball), over the ball of the chosen level-0 bin's
    upper edge (128 bins of d^2 over [0, r^2): the bin holding the 300th neighbour);
  * the correspondence box search's rows at the same pitch: rows within a pruning radius of the
    query (its true nearest-neighbour distance + 1 mm, the certified passes' margin) -- the NN
    kernel shares the grid.

    python tools/normals_pitch_model.py [--scans 3] [--json OUT]
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

R = 0.3
MAX_NN = 300
NB8 = 128
XP = 0.375            # x pitch (LSM_DEFAULT_GRID_CELL)
BLKX = 64             # cells per layout block in x
BSEARCH, SLACK = 16, 8


class AnisoGrid:
    """Points sorted by (y row, z row, x): a row = one (iy, iz) pair over the whole x extent (the
    block split in x is counted separately: a row part ends at every 64-cell block edge)."""

    def __init__(self, pts, py, pz, px=XP, blkx=BLKX):
        p = np.asarray(pts, np.float64)
        self.o = p.min(axis=0)
        self.py, self.pz, self.px, self.blkx = py, pz, px, blkx
        ext = p.max(axis=0) - self.o
        self.ny = int(np.floor(ext[1] / py)) + 1
        self.nz = int(np.floor(ext[2] / pz)) + 1
        self.nx = int(np.floor(ext[0] / px)) + 1
        iy = np.clip(np.floor((p[:, 1] - self.o[1]) / py).astype(np.int64), 0, self.ny - 1)
        iz = np.clip(np.floor((p[:, 2] - self.o[2]) / pz).astype(np.int64), 0, self.nz - 1)
        row = iz * self.ny + iy
        x = p[:, 0] - self.o[0]
        self.key = np.sort(row.astype(np.float64) * 1024.0 + x)   # rows apart by > x extent

    def count(self, row, xl, xh):
        """points of `row` with xl <= x <= xh (x relative to the origin)"""
        base = row.astype(np.float64) * 1024.0
        return (np.searchsorted(self.key, base + xh, "right") -
                np.searchsorted(self.key, base + xl, "left"))

    def walk(self, q, rad):
        """Per query (rows: arrays over queries) the walk's counts for balls of radius rad."""
        n = len(q)
        qx, qy, qz = q[:, 0] - self.o[0], q[:, 1] - self.o[1], q[:, 2] - self.o[2]
        prune = rad * 1.0001 + 1e-6
        rows = np.zeros(n, np.int64)
        visited = np.zeros(n, np.int64)   # row parts the walk visits (slab-pruned), empty or not
        parts = np.zeros(n, np.int64)
        esearch = np.zeros(n, np.float64)
        steps = np.zeros(n, np.float64)
        inwin = np.zeros(n, np.int64)
        cy, cz = np.floor(qy / self.py).astype(np.int64), np.floor(qz / self.pz).astype(np.int64)
        ky = int(np.ceil(R / self.py)) + 1
        kz = int(np.ceil(R / self.pz)) + 1
        xlo_c = np.clip(np.floor((qx - prune) / self.px - 1e-3), 0, self.nx - 1)
        xhi_c = np.clip(np.floor((qx + prune) / self.px + 1e-3), 0, self.nx - 1)
        # cells of the box in x -> row parts split at the layout blocks' x edges
        nparts = (xhi_c // self.blkx - xlo_c // self.blkx + 1).astype(np.int64)
        cxl, cxh = xlo_c * self.px, (xhi_c + 1) * self.px
        for dz in range(-kz, kz + 1):
            iz = cz + dz
            lo, hi = iz * self.pz, (iz + 1) * self.pz
            dz2 = np.where(qz < lo, lo - qz, np.where(qz > hi, qz - hi, 0.0)) ** 2
            okz = (iz >= 0) & (iz < self.nz) & (dz2 <= prune ** 2)
            for dy in range(-ky, ky + 1):
                iy = cy + dy
                lo, hi = iy * self.py, (iy + 1) * self.py
                dyz2 = dz2 + np.where(qy < lo, lo - qy, np.where(qy > hi, qy - hi, 0.0)) ** 2
                ok = okz & (iy >= 0) & (iy < self.ny) & (dyz2 <= prune ** 2)
                if not ok.any():
                    continue
                row = np.where(ok, iz * self.ny + iy, 0)
                ch = np.sqrt(np.maximum(prune ** 2 - dyz2, 0.0))
                cells = self.count(row, cxl, cxh)          # the row's cells in the box
                # (with parts > 1 the run and its entry search split; counted as one run here)
                live = ok & (cells > 0)
                win = self.count(row, qx - ch, qx + ch)
                before = self.count(row, cxl, qx - ch) - (win > 0) * 0
                rows += live
                visited += np.where(ok, nparts, 0)
                parts += np.where(live, nparts, 0)
                inwin += np.where(live, win, 0)
                # entry search: runs of > BSEARCH points, 4-ary rounds down to SLACK points
                long_run = cells > BSEARCH
                rounds = np.where(long_run, np.ceil(np.log(np.maximum(cells, 1) / SLACK) /
                                                    np.log(4.0)), 0)
                esearch += np.where(live, rounds, 0)
                slack = np.where(long_run, np.minimum(before, SLACK / 2.0), before)
                steps += np.where(live, win + slack + 1.0, 0)
        return dict(rows=rows, parts=parts, visited_parts=visited, entry_rounds=esearch,
                    steps=steps, in_window=inwin)


def model_scan(pts, pitches, nn_src=None):
    tree = cKDTree(pts)
    cnt = tree.query_ball_point(pts, R, return_length=True)
    dense = cnt > MAX_NN
    d300 = tree.query(pts[dense], k=MAX_NN)[0][:, -1]
    # the final pass's ball: the upper edge of the level-0 bin holding the 300th neighbour
    top = np.minimum(np.floor(d300 ** 2 * NB8 / R ** 2) + 1, NB8) * R ** 2 / NB8
    rfin = np.sqrt(top)
    nnd = None
    if nn_src is not None:
        nnd = tree.query(nn_src, k=1)[0] + 1e-3
    out = {"points": int(len(pts)), "dense_fraction": float(dense.mean()),
           "ball_members_mean": float(cnt.mean()),
           "knn300_radius_median": float(np.median(d300)) if len(d300) else None,
           "final_radius_median": float(np.median(rfin)) if len(rfin) else None}
    for px, py, pz in pitches:
        g = AnisoGrid(pts, py, pz, px)
        s1 = g.walk(pts, np.full(len(pts), R))
        fin = g.walk(pts[dense], rfin)
        e = {"scan1_sparse": {k: float(v[~dense].mean()) for k, v in s1.items()},
             "scan1_dense": {k: float(v[dense].mean()) for k, v in s1.items()},
             "final_dense": {k: float(v.mean()) for k, v in fin.items()},
             "cells_per_cloud_padded": int(((g.nx + BLKX - 1) // BLKX * BLKX) *
                                           ((g.ny + 3) // 4 * 4) * ((g.nz + 3) // 4 * 4))}
        if nnd is not None:
            nn = g.walk(nn_src, nnd)
            e["nn_box_rows_mean"] = float(nn["rows"].mean())
            e["nn_row_parts_mean"] = float(nn["parts"].mean())
        out[f"{px}/{py}/{pz}"] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--measured", default="",
                    help="normals ms per C3 step at isotropic cells, e.g. 0.25=118.3,0.3=113.2,"
                         "0.375=118.2,0.45=128.0 (bench.py --grid-cell)")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import synthetic
    from oracle import cpu_ref as C
    # (x, y, z) pitches: the isotropic grids bench.py --grid-cell can run (to calibrate the cost
    # of a walk step against a row setup on the GPU), then x 0.375 with finer y / z
    pitches = [(0.25, 0.25, 0.25), (0.3, 0.3, 0.3), (0.375, 0.375, 0.375), (0.45, 0.45, 0.45),
               (0.375, 0.25, 0.25), (0.375, 0.1875, 0.1875), (0.375, 0.125, 0.125),
               (0.375, 0.1875, 0.375), (0.375, 0.375, 0.1875), (0.375, 0.125, 0.375),
               (0.375, 0.125, 0.1875)]
    res = {}
    t0 = time.time()
    seq = synthetic.make_sequence(args.scans + 1, seed=3, model=synthetic.HDL64, processes=4)
    per = []
    for k in range(args.scans):
        tgt = C.filter_radius_height(seq.scans[k])
        src = C.filter_radius_height(seq.scans[k + 1])
        T = seq.priors[k]
        srcT = src @ T[:3, :3].T + T[:3, 3]
        per.append(model_scan(tgt, pitches, srcT))
        print(f"scan {k}: {time.time() - t0:.0f} s", flush=True)
    res["hdl64_seq (C3)"] = per
    # summary: mean over scans, relative to the 0.375 grid
    summ = {}
    for key in per[0]:
        if "/" not in key:
            continue
        e = {}
        for part in ("scan1_sparse", "scan1_dense", "final_dense"):
            e[part] = {m: float(np.mean([p[key][part][m] for p in per]))
                       for m in per[0][key][part]}
        e["nn_box_rows_mean"] = float(np.mean([p[key]["nn_box_rows_mean"] for p in per]))
        e["cells_per_cloud_padded"] = int(np.mean([p[key]["cells_per_cloud_padded"] for p in per]))
        summ[key] = e
    b = summ["0.375/0.375/0.375"]
    df = float(np.mean([p["dense_fraction"] for p in per]))
    for key, e in summ.items():
        # walk steps per point of the whole normals launch (sparse points: scan 1; dense: scan 1 +
        # final), and row setups, against the 0.375 m grid
        st = (1 - df) * e["scan1_sparse"]["steps"] + df * (e["scan1_dense"]["steps"] +
                                                          e["final_dense"]["steps"])
        rs = (1 - df) * e["scan1_sparse"]["parts"] + df * (e["scan1_dense"]["parts"] +
                                                          e["final_dense"]["parts"])
        st0 = (1 - df) * b["scan1_sparse"]["steps"] + df * (b["scan1_dense"]["steps"] +
                                                           b["final_dense"]["steps"])
        rs0 = (1 - df) * b["scan1_sparse"]["parts"] + df * (b["scan1_dense"]["parts"] +
                                                           b["final_dense"]["parts"])
        er = (1 - df) * e["scan1_sparse"]["entry_rounds"] + df * (
            e["scan1_dense"]["entry_rounds"] + e["final_dense"]["entry_rounds"])
        vs = (1 - df) * e["scan1_sparse"]["visited_parts"] + df * (
            e["scan1_dense"]["visited_parts"] + e["final_dense"]["visited_parts"])
        e["visited_row_parts_per_point"] = vs
        e["steps_per_point"] = st
        e["row_setups_per_point"] = rs
        e["entry_rounds_per_point"] = er
        e["steps_vs_0375"] = st / st0
        e["row_setups_vs_0375"] = rs / rs0
        e["nn_rows_vs_0375"] = e["nn_box_rows_mean"] / b["nn_box_rows_mean"]
    res["summary"] = summ
    res["dense_fraction"] = df
    for key, e in summ.items():
        print(f"{key:>18}: steps/pt {e['steps_per_point']:7.1f} ({e['steps_vs_0375']:.3f}x)  "
              f"row setups/pt {e['row_setups_per_point']:5.1f} ({e['row_setups_vs_0375']:.2f}x)  "
              f"entry rounds/pt {e['entry_rounds_per_point']:5.1f}  "
              f"visited parts/pt {e['visited_row_parts_per_point']:5.1f}  "
              f"dense s1 {e['scan1_dense']['steps']:6.1f} fin {e['final_dense']['steps']:6.1f}  "
              f"nn rows {e['nn_box_rows_mean']:.2f} ({e['nn_rows_vs_0375']:.2f}x)  "
              f"cells {e['cells_per_cloud_padded'] / 1e6:.1f} M")
    if args.measured:
        # normals ms per C3 step measured at isotropic grid cells (bench.py --grid-cell): fit
        # t = c0 + a * steps + b * visited row parts (per point), then predict every pitch
        meas = {float(k): float(v) for k, v in (kv.split("=") for kv in args.measured.split(","))}
        iso = [(c, summ[f"{c}/{c}/{c}"]) for c in sorted(meas) if f"{c}/{c}/{c}" in summ]
        A = np.array([[1.0, e["steps_per_point"], e["visited_row_parts_per_point"]] for _, e in iso])
        y = np.array([meas[c] for c, _ in iso])
        coef, *_ = np.linalg.lstsq(A, y, rcond=None)
        fit = {"normals_ms_per_step_measured": meas, "coef": {"c0": coef[0], "per_step": coef[1],
                                                             "per_visited_part": coef[2]},
               "step_equivalents_per_visited_part": coef[2] / coef[1] if coef[1] else None,
               "residuals_ms": (A @ coef - y).tolist(),
               "predicted_normals_ms": {k: float(coef[0] + coef[1] * e["steps_per_point"] +
                                                 coef[2] * e["visited_row_parts_per_point"])
                                        for k, e in summ.items()}}
        res["calibration"] = fit
        print(json.dumps(fit, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
