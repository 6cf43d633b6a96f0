"""C4 sharding on hardware, one GPU: per-rank step time of the contiguous split bench.py ships
(rank r registers revisit pairs r*P .. r*P+P-1) against the LPT packing of distributed.balance_pairs
(cost = N_src x ICP iterations from a warm-up batch of the same pairs), for WORLD ranks.

The ranks' shards run one after another on the one GPU (each alone, as on its own GPU of an
8-GPU node): the step of a rank is bench.py's C4 step for its pairs (pre-process both keyframes
of every pair, lazy normals, one P2Plane batch). The job's time is the slowest rank's, so the
figure of merit is max over ranks / mean over ranks for either split.

    python tools/c4_balance.py [--world 8 --pairs-per-rank 512 --reps 3 --out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--pairs-per-rank", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from lidar_slam_arvc_amd import synthetic
    W, P = args.world, args.pairs_per_rank
    t0 = time.time()
    ps = synthetic.make_revisit_pairs(W * P, seed=args.seed, model=synthetic.HDL64,
                                      processes=16)   # forked workers: before any GPU context
    print(f"{W * P} revisit pairs generated in {time.time() - t0:.1f} s", flush=True)
    from lidar_slam_arvc_amd import _lib
    from lidar_slam_arvc_amd.distributed import balance_contiguous, balance_pairs
    dev = _lib.device(0)
    tg = [dev.upload(s) for s in ps.targets]
    sr = [dev.upload(s) for s in ps.sources]
    prep = _lib.prep_params(want_normals="lazy")
    icp = _lib.icp_params()

    def step(idx):
        dev.preprocess([tg[i] for i in idx] + [sr[i] for i in idx], prep)
        return dev.icp_batch_arrays([sr[i] for i in idx], [tg[i] for i in idx], ps.init[idx], icp)

    def timed(idx):
        step(idx)
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            step(idx)
            ts.append(time.perf_counter() - t)
        return float(np.median(ts))

    contiguous = [np.arange(r * P, (r + 1) * P) for r in range(W)]
    iters = np.zeros(W * P)
    for idx in contiguous:
        iters[idx] = step(idx)["iterations"]
    nsrc = np.array([dev.info(h)[1] for h in sr], dtype=np.float64)
    cost = nsrc * iters
    lpt = balance_pairs(cost, W)
    bal = [np.arange(a, b) for a, b in balance_contiguous(cost, W)]
    t_c = [timed(idx) for idx in contiguous]
    t_l = [timed(idx) for idx in lpt]
    t_b = [timed(idx) for idx in bal]
    res = {
        "workload": f"C4 revisit pairs, seed {args.seed}: {W} ranks x {P} pairs, one GPU, ranks "
                    "run one after another (tools/c4_balance.py)",
        "contiguous_ms": [round(t * 1e3, 2) for t in t_c],
        "lpt_ms": [round(t * 1e3, 2) for t in t_l],
        "lpt_pairs_per_rank": [int(len(v)) for v in lpt],
        "balanced_contiguous_ms": [round(t * 1e3, 2) for t in t_b],
        "balanced_contiguous_pairs_per_rank": [int(len(v)) for v in bal],
        "balanced_contiguous_max_over_mean": round(max(t_b) / np.mean(t_b), 4),
        "contiguous_max_over_mean": round(max(t_c) / np.mean(t_c), 4),
        "lpt_max_over_mean": round(max(t_l) / np.mean(t_l), 4),
        "contiguous_max_over_lpt_max": round(max(t_c) / max(t_l), 4),
        "cost_model": "N_src x iterations of a warm-up batch",
        "cost_max_over_mean": {"contiguous": round(max(float((nsrc * iters)[v].sum()) for v in contiguous) /
                                                   (float((nsrc * iters).sum()) / W), 4),
                               "lpt": round(max(float((nsrc * iters)[v].sum()) for v in lpt) /
                                            (float((nsrc * iters).sum()) / W), 4)},
    }
    print(json.dumps(res, indent=1), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    for h in tg + sr:
        dev.release(h)


if __name__ == "__main__":
    main()
