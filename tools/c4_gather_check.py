"""BASELINE.json configs[3] at its stated size: are the transforms an N-rank C4 run gathered
(bench.py --workload loop_closure --save-gathered, gather_pair_results over every rank's 512
revisit pairs -- loopclosing.py:80-99 scaled to 4096 candidate pairs) bit-identical to ONE context
registering all the same pairs in ONE batch?

Each rank's pairs are make_revisit_pairs(P, seed, first_index = rank * P) (bench.make_data); the
generator is index-addressed, so generating the shards here in the same chunks gives the same
clouds. The relative transforms of independent pairs do not depend on the batch they run in (the
ICP path is deterministic: fixed-order reductions), so the comparison is exact.

usage: python tools/c4_gather_check.py GATHERED.npz [--out SUMMARY.json]
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
    ap.add_argument("gathered")
    ap.add_argument("--out", default="")
    ap.add_argument("--cache-dir", default="", help="keep the generated shards here (bench.py "
                                                    "--seq-cache format); default: no cache")
    args = ap.parse_args()
    z = np.load(args.gathered)
    G = np.asarray(z["transformation"])
    world, P, seed = int(z["world"]), int(z["pairs_per_rank"]), int(z["seed"])
    n = world * P
    assert G.shape == (n, 4, 4), G.shape

    import bench
    procs = max(1, min(8, len(os.sched_getaffinity(0))))
    t0 = time.time()
    shards = [bench.make_data("loop_closure", P, seed, r * P, procs,
                              os.path.join(args.cache_dir, f"lsm_c4_r{r}.npz")
                              if args.cache_dir else "")
              for r in range(world)]
    gen_s = time.time() - t0
    targets = [s for sh in shards for s in sh.scans[:P]]
    sources = [s for sh in shards for s in sh.scans[P:]]
    init = np.concatenate([sh.priors for sh in shards])
    del shards

    from lidar_slam_arvc_amd import _lib
    dev = _lib.device(0)
    t0 = time.time()
    ids = [dev.upload(s) for s in targets + sources]
    del targets, sources
    try:
        # pre-processing is per cloud; chunks of 1024 keep each call's cell keys within 32 bits
        for a in range(0, len(ids), 1024):
            dev.preprocess(ids[a:a + 1024], _lib.prep_params(want_normals="lazy"))
        res = dev.icp_batch_arrays(ids[n:], ids[:n], init, _lib.icp_params())
    finally:
        for h in ids:
            dev.release(h)
    run_s = time.time() - t0
    T = np.asarray(res["transformation"])
    equal = np.all(T == G, axis=(1, 2))
    summary = {"config": "BASELINE.json configs[3]: loop-closure batch, 64k-point HDL-64 revisit "
                         "pairs", "global_pairs": n, "ranks": world, "pairs_per_rank": P,
               "seed": seed, "gathered": os.path.relpath(args.gathered, ROOT),
               "single_context": f"one context, one {n}-pair batch (lazy normals), {run_s:.1f} s "
                                 f"(data {gen_s:.1f} s)",
               "bit_identical_pairs": int(equal.sum()),
               "bit_identical": bool(equal.all()),
               "differing_pairs": [int(k) for k in np.flatnonzero(~equal)][:50],
               "max_abs_diff": float(np.abs(T - G).max()),
               "iterations_mean": float(np.mean(res["iterations"]))}
    text = json.dumps(summary, indent=1)
    print(text, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    if not equal.all():
        raise SystemExit(1)


if __name__ == "__main__":
    main()
