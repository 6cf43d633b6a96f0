"""CPU model: would the dense half's final-pass cumulant sums pay as f64 MFMA tiles?

VERDICT r5 item 5. The dense half's final pass (prep.hip hybrid_lane, NL_DENSE_NR) walks, per lane
(one dense point), the rows of the chosen level-0 bin's ball and adds every member's centred f64
cumulants (3 v_cvt_f64_f32 + 3 f64 subtractions + 9 f64 add / fma per member). An
MFMA form would give a WAVE 16 queries: per v_mfma_f64_16x16x4f64, A = the 16 x 4 membership mask
of 4 candidates (one (query, candidate) test per lane), B = 4 candidates x 16 features (1, x, y, z,
xx, xy, xz, yy, yz, zz about a group origin; 10 of 16 columns used), C += A B: 16 queries x 16
cumulants. The candidates are the union of the 16 queries' windows.

This counts, on bench scans, for groups of 16 consecutive dense points in the layout's cell order:
  * the union-window overhead: candidates of the group's union / the mean per-query window;
  * the per-lane form's divergence: per 64-lane wave, max / mean of the final-pass walk steps;
and prices both forms in SIMD issue cycles with measured rates (tools/calib/valu_calib.hip on the
box: v_fma_f32, v_fma_f64 / v_add_f64, v_mfma_f64_16x16x4f64; profiles/r06*/valu_calib.log).

    python tools/normals_mfma_model.py [--scans 2] [--mfma-cycles C] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import normals_pitch_model as PM  # noqa: E402

# SIMD issue cycles per wave-instruction at 2.4 GHz, from the calibration's chip rates
# (profiles/r05h/valu_calib.log: v_fma_f32 868 G/s, v_fma_f64 498, v_add_f64 507 over 1024 SIMDs)
F32_CYC = 1024 * 2.4e9 / 868e9      # 2.83
F64_CYC = 1024 * 2.4e9 / 500e9      # 4.92


def final_windows(g, q, rad, with_rows=False):
    """Per query: list of (lo, hi) index ranges into g.key of its final-pass row windows
    (with_rows: (row, lo, hi))."""
    qx, qy, qz = q[:, 0] - g.o[0], q[:, 1] - g.o[1], q[:, 2] - g.o[2]
    prune = rad * 1.0001 + 1e-6
    cy, cz = np.floor(qy / g.py).astype(np.int64), np.floor(qz / g.pz).astype(np.int64)
    ky, kz = int(np.ceil(PM.R / g.py)) + 1, int(np.ceil(PM.R / g.pz)) + 1
    out = [[] for _ in range(len(q))]
    for dz in range(-kz, kz + 1):
        iz = cz + dz
        lo, hi = iz * g.pz, (iz + 1) * g.pz
        dz2 = np.where(qz < lo, lo - qz, np.where(qz > hi, qz - hi, 0.0)) ** 2
        for dy in range(-ky, ky + 1):
            iy = cy + dy
            lo, hi = iy * g.py, (iy + 1) * g.py
            dyz2 = dz2 + np.where(qy < lo, lo - qy, np.where(qy > hi, qy - hi, 0.0)) ** 2
            ok = (iz >= 0) & (iz < g.nz) & (iy >= 0) & (iy < g.ny) & (dyz2 <= prune ** 2)
            row = (iz * g.ny + iy).astype(np.float64) * 1024.0
            ch = np.sqrt(np.maximum(prune ** 2 - dyz2, 0.0))
            a = np.searchsorted(g.key, row + qx - ch, "left")
            b = np.searchsorted(g.key, row + qx + ch, "right")
            rid = (iz * g.ny + iy)
            for k in np.flatnonzero(ok & (b > a)):
                out[k].append((int(rid[k]), int(a[k]), int(b[k])) if with_rows else
                              (int(a[k]), int(b[k])))
    return out


def hull_len(wins):
    """Candidates of a group that walks, per row any of its queries touches, one window from the
    smallest left end to the largest right end (what a wave can enumerate cheaply)."""
    rows = {}
    for w in wins:
        for r, a, b in w:
            lo, hi = rows.get(r, (a, b))
            rows[r] = (min(lo, a), max(hi, b))
    return sum(hi - lo for lo, hi in rows.values())


def union_len(ranges):
    if not ranges:
        return 0
    rs = sorted(ranges)
    tot, (ca, cb) = 0, rs[0]
    for a, b in rs[1:]:
        if a > cb:
            tot += cb - ca
            ca, cb = a, b
        else:
            cb = max(cb, b)
    return tot + cb - ca


def model_scan(pts, mfma_cyc):
    tree = cKDTree(pts)
    cnt = tree.query_ball_point(pts, PM.R, return_length=True)
    dense = np.flatnonzero(cnt > PM.MAX_NN)
    # the layout's cell order (0.375 m cells, 64-wide blocks: blocks z-major, rows, x)
    c = np.floor((pts - pts.min(0)) / 0.375).astype(np.int64)
    nb = c.max(0) // np.array([64, 4, 4]) + 1
    lin = ((((c[:, 2] // 4) * nb[1] + c[:, 1] // 4) * nb[0] + c[:, 0] // 64) * 1024 +
           (c[:, 2] % 4) * 256 + (c[:, 1] % 4) * 64 + c[:, 0] % 64)
    dense = dense[np.lexsort((pts[dense, 0], lin[dense]))]
    q = pts[dense]
    d300 = tree.query(q, k=PM.MAX_NN)[0][:, -1]
    top = np.minimum(np.floor(d300 ** 2 * PM.NB8 / PM.R ** 2) + 1, PM.NB8) * PM.R ** 2 / PM.NB8
    rad = np.sqrt(top)
    g = PM.AnisoGrid(pts, 0.375, 0.375)
    winr = final_windows(g, q, rad, with_rows=True)
    win = [[(a, b) for _, a, b in w] for w in winr]
    steps = np.array([sum(b - a for a, b in w) for w in win], np.float64)
    members = np.array([len(tree.query_ball_point(p, r * 0.99999)) for p, r in zip(q, rad)],
                       np.float64)
    n = len(q)
    # per-lane form: a wave of 64 dense points runs its slowest lane's trips; every trip issues
    # the walk body (14 VALU) and, when any lane adds a member (nearly every trip), the adds
    # (3 cvt + 3 sub + 9 add/fma, all f64-rate)
    W = 64
    wmax = np.array([steps[i:i + W].max() for i in range(0, n, W)])
    wlen = np.array([len(steps[i:i + W]) for i in range(0, n, W)])
    lane_cyc = float((wmax * (14 * F32_CYC + 15 * F64_CYC)).sum() / n)
    # MFMA form: groups of 16; per 4 union candidates one MFMA plus per lane: candidate load,
    # f32 d2 + thresholds (9 VALU), mask -> f64 A operand (2), its feature of B (cvt, sub, mul:
    # 3 f64-rate); VALU and the matrix pipe overlap across waves: max of the two per step
    Q = 16
    uni = np.array([union_len([r for w in win[i:i + Q] for r in w]) for i in range(0, n, Q)],
                   np.float64)
    hull = np.array([hull_len(winr[i:i + Q]) for i in range(0, n, Q)], np.float64)
    gsz = np.array([len(win[i:i + Q]) for i in range(0, n, Q)], np.float64)
    mstep_valu = 11 * F32_CYC + 3 * F64_CYC
    mfma_steps = np.ceil(uni / 4.0)
    mfma_cyc_total = float((mfma_steps * max(mfma_cyc, mstep_valu)).sum() / n)
    hull_cyc_total = float((np.ceil(hull / 4.0) * max(mfma_cyc, mstep_valu)).sum() / n)
    mean_win = float(steps.mean())
    return {
        "dense_points": int(n),
        "final_window_mean": mean_win,
        "final_members_mean": float(members.mean()),
        "per_lane_wave_divergence": float((wmax * wlen).sum() / steps.sum()),
        # candidates a group tests per query, over the candidates a lane walks for its own query
        "union_overhead_16": float(uni.sum() / (steps.sum() / Q)),
        "union_candidates_per_group_mean": float(uni.mean()),
        "row_hull_overhead_16": float(hull.sum() / (steps.sum() / Q)),
        "issue_cycles_per_dense_point": {"per_lane_f64_valu": lane_cyc,
                                         "mfma_f64_16x16x4": mfma_cyc_total,
                                         "mfma_f64_16x16x4_row_hull": hull_cyc_total},
        "mfma_over_per_lane": mfma_cyc_total / lane_cyc,
        "mfma_row_hull_over_per_lane": hull_cyc_total / lane_cyc,
        "group_sizes": float(gsz.mean()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=2)
    ap.add_argument("--mfma-cycles", type=float, default=64.0,
                    help="SIMD cycles per v_mfma_f64_16x16x4f64 (calibration log; 64 = the "
                         "78.6 TFLOP/s FP64 matrix spec: 2048 FLOP at 32 FLOP/cycle/SIMD)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import synthetic
    from oracle import cpu_ref as C
    seq = synthetic.make_sequence(args.scans, seed=3, model=synthetic.HDL64, processes=4)
    per = []
    for k in range(args.scans):
        r = model_scan(C.filter_radius_height(seq.scans[k]), args.mfma_cycles)
        print(json.dumps(r), flush=True)
        per.append(r)
    summ = {k: float(np.mean([p[k] for p in per])) for k in
            ("final_window_mean", "final_members_mean", "per_lane_wave_divergence",
             "union_overhead_16", "row_hull_overhead_16", "mfma_over_per_lane",
             "mfma_row_hull_over_per_lane")}
    summ["issue_cycles_per_dense_point"] = {
        k: float(np.mean([p["issue_cycles_per_dense_point"][k] for p in per]))
        for k in per[0]["issue_cycles_per_dense_point"]}
    summ["mfma_cycles_assumed"] = args.mfma_cycles
    summ["rates"] = {"f32_cycles": F32_CYC, "f64_cycles": F64_CYC}
    res = {"hdl64_seq (C3) scans": per, "summary": summ}
    print(json.dumps(summ, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
