"""CPU model of the correspondence search's per-query work and its lane divergence.

The PMC counts of round 5 (profiles/r05g/nn_cache_counters.json) give nn_kernel<false> -- the
full passes 0 and 1 -- about 6 200 VALU wave-instructions per wave, several times what one query's
box search costs on its own. This replays nn_query's box search (icp.hip: cold start with the
own-cell seed, warm start from the previous pass, K-cell box, rows centre-out pruned by their slab
distance, block parts, x-window walks, Top3 / prune2) in Python on the bench's own clouds and
counts per query the loop iterations it runs: row iterations, scanned block parts, entry-search
steps and points examined. A wave runs its 64 lanes' loops together, so its cost is set by its
slowest lanes: the model reports per-wave max / mean of a per-lane cost (a weighted sum of the
counts), i.e. how much of the issued work is divergence.

    python tools/nn_work_model.py [--pairs 2] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CELL = np.float32(0.375)   # x / z cell edge (--cell)
YSUB = 1          # y cells are CELL / YSUB (--ysub; lsm_common.h LSM_YSUB: 2 since round 6)
CELLY = CELL
BLK = 4           # cells per layout block edge in z
BLKY = 4          # ... in y (4 * YSUB)
BLKX = 64         # ... and in x (lsm_common.h LSM_BLKX)
LIN = 8            # runs of at most this many points are scanned whole
KCOLD, KMAX = 4, 4
INF = np.float32(np.inf)


class Grid:
    """The library's blocked cell layout of a target cloud (prep.hip grid_keys / grid_fill)."""

    def __init__(self, pts):
        p = pts.astype(np.float32)
        self.o = p.min(axis=0)
        self.inv = np.float32(1.0) / CELL
        self.invy = np.float32(1.0) / CELLY
        self.inv3 = np.array([self.inv, self.invy, self.inv], np.float32)
        ext = p.max(axis=0) - self.o
        self.n = (np.floor(ext * self.inv3).astype(np.int64) + 1)
        self.nb = (self.n + np.array([BLKX, BLKY, BLK]) - 1) // np.array([BLKX, BLKY, BLK])
        c = np.floor((p - self.o) * self.inv3).astype(np.int64)
        c = np.minimum(np.maximum(c, 0), self.n - 1)
        lin = self.lin(c[:, 0], c[:, 1], c[:, 2])
        order = np.lexsort((p[:, 0], lin))
        self.p = p[order]
        self.x = self.p[:, 0]
        ncell = int(self.nb[0] * self.nb[1] * self.nb[2] * BLKX * BLKY * BLK)
        cnt = np.bincount(lin, minlength=ncell)
        self.cs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)

    def rb(self, x, y, z):
        """row-bounds table index: per layout block, x-major, then z, then y (16 rows of one x
        cell adjacent: 64 B)"""
        bx, by, bz = x // BLKX, y >> 2, z >> 2
        return ((((bz * self.nb[1] + by) * self.nb[0] + bx) * (BLKX * 16)) + (x % BLKX) * 16 +
                (z & 3) * 4 + (y & 3))

    def lin(self, x, y, z):
        """lsm_cell_lin"""
        bx, by, bz = x // BLKX, y // BLKY, z >> 2
        return (((bz * self.nb[1] + by) * self.nb[0] + bx) * (BLKX * BLKY * BLK)) + \
               ((z & 3) * BLKY * BLKX) + ((y % BLKY) * BLKX) + (x % BLKX)

    def occ_line(self, x, y, z):
        """the 128-B line of the 64-bit occupancy word of (y, z)'s row in x's layout block"""
        blk = self.lin(x, y, z) // (BLKX * BLKY * BLK)
        row = (z & 3) * BLKY + (y % BLKY)
        return (blk * BLKY * BLK + row) * 8 // 128


def sqd(t, q):
    dx = np.float32(q[0] - t[0])
    dy = np.float32(q[1] - t[1])
    dz = np.float32(q[2] - t[2])
    return np.float32(np.float32(dz * dz) + np.float32(np.float32(dy * dy) + np.float32(dx * dx)))


class Top3:
    def __init__(self, bidx, bd2, m):
        self.bd2, self.bidx, self.sd2, self.sidx, self.td2, self.m = bd2, bidx, INF, -1, INF, m
        self.lim = self.prune()

    def prune(self):
        c = np.float32(math.sqrt(self.bd2)) + self.m if self.bd2 < INF else INF
        return max(self.bd2, min(self.td2, c * c))

    def add(self, d2, k):
        if k == self.bidx or k == self.sidx or not (d2 <= self.td2):
            return
        if d2 < self.bd2 or (d2 == self.bd2 and k < self.bidx):
            self.td2, self.sd2, self.sidx, self.bd2, self.bidx = self.sd2, self.bd2, self.bidx, d2, k
        elif d2 < self.sd2 or (d2 == self.sd2 and k < self.sidx):
            self.td2, self.sd2, self.sidx = self.sd2, d2, k
        else:
            self.td2 = d2
        self.lim = self.prune()


def query(G, q, prev, m, st):
    t2 = Top3(-1, INF, m)
    if prev >= 0:
        t2 = Top3(prev, sqd(G.p[prev], q), m)
    f = (q - G.o) * G.inv3
    c = [int(min(max(math.floor(f[a]), 0), G.n[a] - 1)) for a in range(3)]
    K = KCOLD
    if t2.bidx < 0:
        cl = G.lin(c[0], c[1], c[2])
        a, b = G.cs[cl], G.cs[cl + 1]
        if b > a:
            k = (a + b) >> 1
            t2 = Top3(k, sqd(G.p[k], q), m)
    elif t2.bd2 < INF:
        rc = math.sqrt(t2.bd2) * G.inv * 1.0001 + 1e-4
        K = KMAX if rc >= KMAX else max(1, math.ceil(rc))
    Ks = [K, K * YSUB, K]
    lo = [max(c[a] - Ks[a], 0) for a in range(3)]
    hi = [min(c[a] + Ks[a], G.n[a] - 1) for a in range(3)]
    c2 = float(CELL * CELL * np.float32(0.9999))
    c2y = float(CELLY * CELLY * np.float32(0.9999))
    W = 2 * K + 1
    Wy = 2 * K * YSUB + 1

    def slab(fv, k):
        d = k - fv if fv < k else (fv - (k + 1) if fv > k + 1 else 0.0)
        return d * d

    for iz in range(W):
        adz = (iz + 1) >> 1
        if adz >= 2 and (adz - 1) ** 2 * c2 >= t2.lim:
            break
        z = c[2] + (-adz if iz & 1 else adz)
        st["row_iters"] += 1
        if z < lo[2] or z > hi[2]:
            continue
        wz = slab(f[2], z) * c2
        if wz >= t2.lim:
            continue
        for iy in range(Wy):
            ady = (iy + 1) >> 1
            if ady >= 2 and wz + (ady - 1) ** 2 * c2y >= t2.lim:
                break
            y = c[1] + (-ady if iy & 1 else ady)
            st["row_iters"] += 1
            if y < lo[1] or y > hi[1]:
                continue
            wyz = wz + slab(f[1], y) * c2y
            lim = t2.lim
            if wyz >= lim:
                continue
            st["rows"] += 1
            xa, xb = lo[0], hi[0]
            if lim < INF:
                ch = math.sqrt((lim - wyz) * 1.0002) * G.inv + 1e-4
                xa = max(xa, math.floor(f[0] - ch))
                xb = min(xb, math.floor(f[0] + ch))
            x = xa
            while x <= xb:
                xe = min(xb, x | (BLKX - 1))
                la, lb = G.lin(x, y, z), G.lin(xe, y, z) + 1
                a, b = G.cs[la], G.cs[lb]
                st["parts"] += 1
                if LINES is not None:
                    # cell-table lines (128 B): the blocked table as built, and a row-bounds table
                    # ordered (block, x, z, y) with a start and an end array
                    LINES["cell"].update((la * 4 // 128, lb * 4 // 128))
                    LINES["rb"].update((("s", G.rb(x, y, z) * 4 // 128),
                                        ("e", G.rb(xe, y, z) * 4 // 128)))
                    # occupancy bits: one 64-bit word per block row (x cells), the block's 16
                    # rows in one 128-B line; the cell table is read only for occupied parts
                    LINES["occ"].add(("o", G.occ_line(x, y, z)))
                    if b > a:
                        LINES["occ"].update((la * 4 // 128, lb * 4 // 128))
                        st["parts_nonempty"] += 1
                if b > a:
                    run(G, a, b, q, wyz, t2, st)
                x = xe + 1
    return t2


LINES = None   # per-workgroup sets of 128-B lines touched (line model)


def _pt(k):
    if LINES is not None:
        LINES["pts"].add(k * 16 // 128)


def run(G, a, b, q, dyz2, t2, st):
    if b - a <= LIN:
        for k in range(a, b):
            st["points"] += 1
            _pt(k)
            t2.add(sqd(G.p[k], q), k)
        return
    lo, hi = a, b
    while lo < hi:
        st["search"] += 1
        mid = (lo + hi) >> 1
        _pt(mid)
        if G.x[mid] < q[0]:
            lo = mid + 1
        else:
            hi = mid
    for k in range(lo, b):
        st["points"] += 1
        _pt(k)
        dx = np.float32(G.x[k] - q[0])
        if dx * dx + dyz2 > t2.lim:
            break
        t2.add(sqd(G.p[k], q), k)
    for k in range(lo - 1, a - 1, -1):
        st["points"] += 1
        _pt(k)
        dx = np.float32(q[0] - G.x[k])
        if dx * dx + dyz2 > t2.lim:
            break
        t2.add(sqd(G.p[k], q), k)


def src_order(S):
    """The source's sorted order (the same layout): workgroups take 256 consecutive points."""
    return Grid(S).p


def one_pass(G, src, T, prevs, m, limit, lines=None):
    """lines (a list): per 256-query workgroup, the distinct 128-B lines its queries touch in the
    cell table as built, in a row-bounds table, and in the target points"""
    global LINES
    q64 = src.astype(np.float64) @ T[:3, :3].T + T[:3, 3]
    q = q64.astype(np.float32)
    rows = []
    res = np.full(len(q), -1, np.int64)
    for i in range(min(limit, len(q))):
        if lines is not None and i % 256 == 0:
            if LINES is not None:
                lines.append({k: len(v) for k, v in LINES.items()})
            LINES = {"cell": set(), "rb": set(), "occ": set(), "pts": set()}
        st = {"row_iters": 0, "rows": 0, "parts": 0, "search": 0, "points": 0, "parts_nonempty": 0}
        t2 = query(G, q[i], prevs[i], np.float32(m[i]), st)
        res[i] = t2.bidx
        rows.append([st[k] for k in ("row_iters", "rows", "parts", "search", "points",
                                     "parts_nonempty")])
    if lines is not None and LINES is not None:
        lines.append({k: len(v) for k, v in LINES.items()})
    LINES = None
    return np.array(rows), res


def wave_stats(w, weights):
    cost = w @ np.array(weights, float)
    n = len(cost) // 64 * 64
    c = cost[:n].reshape(-1, 64)
    return {"lane_mean": round(float(c.mean()), 1), "wave_max_mean": round(float(c.max(axis=1).mean()), 1),
            "divergence": round(float(c.max(axis=1).mean() / max(c.mean(), 1e-9)), 2),
            "lane_p50": round(float(np.median(cost)), 1), "lane_p99": round(float(np.quantile(cost, 0.99)), 1),
            "lane_max": round(float(cost.max()), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--queries", type=int, default=16384, help="queries per pair (cell order)")
    ap.add_argument("--json", default="")
    ap.add_argument("--cell", type=float, default=0.375, help="x / z cell edge (round 6: 0.42)")
    ap.add_argument("--ysub", type=int, default=1, help="y cells per x / z cell (round 6: 2)")
    args = ap.parse_args()
    global CELL, CELLY, YSUB, BLKY
    CELL = np.float32(args.cell)
    YSUB = args.ysub
    CELLY = np.float32(args.cell / args.ysub)
    BLKY = 4 * YSUB
    from lidar_slam_arvc_amd import synthetic
    from oracle import cpu_ref as C
    # rough VALU weights per counted iteration (icp.hip nn_query / scan_run)
    weights = [6, 25, 12, 6, 18, 0]
    names = ["row_iters", "rows", "parts", "search", "points", "parts_nonempty"]
    out = {"weights_valu_per_item": dict(zip(names, weights))}
    for wl in ("hdl64_seq", "loop_closure"):
        per = {0: [], 1: []}
        lines = {0: [], 1: []}
        for mi in range(args.pairs):
            if wl == "hdl64_seq":
                s = synthetic.make_sequence(2, seed=3, first_index=500 * mi + 17)
                tgt, src, T0 = s.scans[0], s.scans[1], s.priors[0]
            else:
                ps = synthetic.make_revisit_pairs(1, seed=4, first_index=100 * mi + 3)
                tgt, src, T0 = ps.targets[0], ps.sources[0], ps.init[0]
            tgt = C.filter_radius_height(tgt)
            src = src_order(C.filter_radius_height(src))
            G = Grid(tgt)
            T1 = C.registration_icp(src, tgt, 10.0, T0, "p2plane", C.estimate_normals(tgt),
                                    max_iteration=1)["transformation"]
            n = min(args.queries, len(src))
            w0, r0 = one_pass(G, src, T0, np.full(n, -1), np.zeros(n), n, lines[0])
            # pass 1: warm start from pass 0, margin = the query's motion + 1 mm
            q0 = src[:n].astype(np.float64) @ T0[:3, :3].T + T0[:3, 3]
            q1 = src[:n].astype(np.float64) @ T1[:3, :3].T + T1[:3, 3]
            m1 = np.linalg.norm(q1.astype(np.float32) - q0.astype(np.float32), axis=1) + 1e-3
            w1, _ = one_pass(G, src, T1, r0, m1, n, lines[1])
            per[0].append(w0)
            per[1].append(w1)
        out[wl] = {}
        for p in (0, 1):
            w = np.concatenate(per[p])
            out[wl][f"pass{p}"] = {"mean_counts": dict(zip(names, np.round(w.mean(axis=0), 2).tolist())),
                                   "p99_counts": dict(zip(names, np.quantile(w, 0.99, axis=0).tolist())),
                                   "cost": wave_stats(w, weights),
                                   "lines_per_workgroup": {
                                       k: round(float(np.mean([d[k] for d in lines[p]])), 1)
                                       for k in ("cell", "rb", "occ", "pts")}}
        print(wl, json.dumps(out[wl], indent=1), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
