"""CPU model of LDS-staged target tiles for the correspondence search's full passes (0 and 1).

Question: if each 256-query workgroup of nn_kernel staged, into LDS, every
target cell its queries could need, how large would the tiles be? A workgroup's queries are 256
consecutive points of the cell-sorted source (prep.hip's blocked layout: 4x4x4-cell blocks z-major,
cells z-major inside a block, x inside a cell), transformed by the pair's transform of the pass.
A tile must hold every target cell within R of the queries' bounding box, R = the largest
nearest-neighbour distance among the queries the tile should resolve (queries whose neighbour is
farther than R_cap are left to the global path). Reported per workload and pass: the fraction of
workgroups whose tile fits 64 / 96 / 160 KiB (16 B per point, as stored; 12 B packed), tile
sizes, and the staged-bytes amplification over the target cloud.

    python tools/nn_tile_model.py [--pairs 6] [--rcap 0.5]
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

CELL = 0.375


def blocked_order(p):
    """Sorted positions of the library's grid layout (cell 0.375 m over the cloud's bbox)."""
    o = p.min(axis=0)
    c = np.floor((p - o) / CELL).astype(np.int64)
    n = c.max(axis=0) + 1
    nb = (n + 3) // 4
    b = c >> 2
    lin = (((b[:, 2] * nb[1] + b[:, 1]) * nb[0] + b[:, 0]) << 6) | ((c[:, 2] & 3) << 4) | \
          ((c[:, 1] & 3) << 2) | (c[:, 0] & 3)
    return np.lexsort((p[:, 0], lin))


def tiles(src, tgt, T, rcap, wg=256, margin_cells=None):
    q = src[blocked_order(src)] @ T[:3, :3].T + T[:3, 3]
    tree = cKDTree(tgt)
    d, _ = tree.query(q, k=1)
    o = tgt.min(axis=0)
    tc = np.floor((tgt - o) / CELL).astype(np.int64)
    n = tc.max(axis=0) + 1
    lin = (tc[:, 2] * n[1] + tc[:, 1]) * n[0] + tc[:, 0]
    counts = np.bincount(lin, minlength=int(np.prod(n))).reshape(n[2], n[1], n[0])
    cum = counts.cumsum(0).cumsum(1).cumsum(2)
    cum = np.pad(cum, ((1, 0), (1, 0), (1, 0)))

    def box_count(lo, hi):   # points in cells [lo, hi] (inclusive, clipped)
        lo = np.clip(lo, 0, n - 1)
        hi = np.clip(hi, 0, n - 1)
        if np.any(hi < lo):
            return 0
        x0, y0, z0 = lo
        x1, y1, z1 = hi + 1
        return int(cum[z1, y1, x1] - cum[z0, y1, x1] - cum[z1, y0, x1] - cum[z1, y1, x0] +
                   cum[z0, y0, x1] + cum[z0, y1, x0] + cum[z1, y0, x0] - cum[z0, y0, x0])

    out = []
    for s in range(0, len(q), wg):
        qq, dd = q[s:s + wg], d[s:s + wg]
        if margin_cells is None:
            keep = dd <= rcap
            R = float(dd[keep].max()) if keep.any() else 0.0
            lo = np.floor((qq.min(axis=0) - R - o) / CELL).astype(np.int64)
            hi = np.floor((qq.max(axis=0) + R - o) / CELL).astype(np.int64)
            out.append((box_count(lo, hi), int((~keep).sum()), len(qq), 0))
            continue
        # the kernel's design: the cells of the queries' bbox (clamped to the grid) +- margin;
        # a query resolves in the tile when its neighbour is nearer than every face of the
        # staged box that is not the grid's boundary
        f = (qq - o) / CELL
        c = np.clip(np.floor(f).astype(np.int64), 0, n - 1)
        lo = np.maximum(c.min(axis=0) - margin_cells, 0)
        hi = np.minimum(c.max(axis=0) + margin_cells, n - 1)
        dlo = np.where(lo > 0, f - lo, np.inf)
        dhi = np.where(hi < n - 1, hi + 1 - f, np.inf)
        face = np.minimum(dlo, dhi).min(axis=1) * CELL
        rows = int((hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1))
        out.append((box_count(lo, hi), int((dd > face).sum()), len(qq), rows))
    return np.array(out), len(tgt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=6)
    ap.add_argument("--rcap", type=float, default=0.5)
    ap.add_argument("--out", default="")
    ap.add_argument("--margin", type=int, default=-1,
                    help=">= 0: the kernel design (bbox cells +- this many cells) instead of the "
                         "neighbour-distance tile")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import synthetic
    from oracle import cpu_ref as C
    res = {}
    for wl in ("hdl64_seq", "loop_closure"):
        rows = {0: [], 1: []}
        amp = {0: [], 1: []}
        for m in range(args.pairs):
            if wl == "hdl64_seq":
                s = synthetic.make_sequence(2, seed=3, first_index=300 * m)
                tgt, src, T0 = s.scans[0], s.scans[1], s.priors[0]
            else:
                ps = synthetic.make_revisit_pairs(1, seed=4, first_index=60 * m)
                tgt, src, T0 = ps.targets[0], ps.sources[0], ps.init[0]
            tgt = C.filter_radius_height(tgt)
            src = C.filter_radius_height(src)
            T1 = C.registration_icp(src, tgt, 10.0, T0, "p2plane", C.estimate_normals(tgt),
                                    max_iteration=1)["transformation"]
            for ps_, T in ((0, T0), (1, T1)):
                t, nt = tiles(src, tgt, T, args.rcap,
                              margin_cells=None if args.margin < 0 else args.margin)
                rows[ps_].append(t)
                amp[ps_].append(t[:, 0].sum() / nt)
        res[wl] = {}
        for ps_ in (0, 1):
            t = np.concatenate(rows[ps_])
            kb = t[:, 0] * 16 / 1024
            res[wl][f"pass{ps_}"] = {
                "workgroups": int(len(t)),
                "fit_16B": {f"{c}KiB": round(float((kb <= c).mean()), 4) for c in (64, 96, 160)},
                "fit_12B": {f"{c}KiB": round(float((kb * 0.75 <= c).mean()), 4)
                            for c in (64, 96, 160)},
                "tile_KiB_quantiles_16B": {q: round(float(np.quantile(kb, q / 100)), 1)
                                          for q in (10, 50, 90, 99)},
                "queries_beyond_rcap" if args.margin < 0 else "queries_unresolved_in_tile":
                    round(float(t[:, 1].sum() / t[:, 2].sum()), 5),
                "fit_points": {f"{c}": round(float((t[:, 0] <= c).mean()), 4)
                               for c in (2048, 3072, 4096)},
                "rows_quantiles": {q: int(np.quantile(t[:, 3], q / 100)) for q in (50, 90, 99)},
                "staged_over_target_bytes": round(float(np.mean(amp[ps_])), 2)}
        print(wl, json.dumps(res[wl], indent=1), flush=True)
    res["model"] = {"rcap_m": args.rcap, "pairs_per_workload": args.pairs, "cell_m": CELL}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
