"""Headline-workload parity: every pair of bench.py's C3 sequence (seed 3, 2000 HDL-64 keyframes,
1999 consecutive P2Plane pairs) through the GPU path and through the f64 C++/OpenMP CPU
implementation of the same path (oracle/cpu/lsm_cpu.cpp, the checker), then a summary.

Reference semantics: keyframe.py:246-252 (registration_icp, P2Plane, max_corr 10 m, Open3D's
default criteria) on the pairs of run_scanmatcher.py:196-213 (each pair seeded with its
odometry prior).

Two modes:

  python tools/bench_parity.py --make-cpu OUT.npz
      CPU side only (any host; all cores): writes the oracle's per-pair results together with a
      SHA-256 of the generated sequence, so a GPU run elsewhere can prove it saw the same data.

  python tools/bench_parity.py [--cpu FIXTURE.npz | --cpu-live] [--out SUMMARY.json]
      GPU side (the bench's own batch: pre-process all 2000 keyframes, one 1999-pair ICP batch),
      compared against the fixture (or against the C++ oracle run live on this host's cores).

Summary (JSON): pairs within north_star's tolerance (|dR| <= 1e-4, |dt| <= 1e-3 m), the worst
|dR| / |dt| among pairs both sides converged, iteration-count agreement, and for the pairs that
hit max_iteration on either side their indices with fitness / rmse deltas.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TOL_R, TOL_T = 1e-4, 1e-3
MAX_ITER = 30


def sequence(P: int, seed: int):
    from lidar_slam_arvc_amd import synthetic
    procs = max(1, min(16, len(os.sched_getaffinity(0))))
    return synthetic.make_sequence(P + 1, seed=seed, model=synthetic.HDL64, processes=procs)


def seq_hash(seq) -> str:
    h = hashlib.sha256()
    for s in seq.scans:
        h.update(np.ascontiguousarray(s, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(seq.priors, dtype=np.float64).tobytes())
    return h.hexdigest()


def run_cpu(seq, threads: int, log=print):
    """The C++ oracle on every pair: filter + normals per keyframe, then registration_icp."""
    from oracle import cpu_ref as C
    C.set_threads(threads)
    P = len(seq.scans) - 1
    T = np.zeros((P, 4, 4))
    fit, rmse = np.zeros(P), np.zeros(P)
    iters, ncorr = np.zeros(P, np.int32), np.zeros(P, np.int64)
    t0 = time.time()
    last = t0
    prev = None
    for k in range(P):
        if prev is None:
            tp = C.filter_radius_height(seq.scans[k])
            prev = (tp, C.estimate_normals(tp))
        sp = C.filter_radius_height(seq.scans[k + 1])
        cur = (sp, C.estimate_normals(sp))
        r = C.registration_icp(sp, prev[0], 10.0, seq.priors[k], "p2plane", prev[1])
        T[k] = r["transformation"]
        fit[k], rmse[k] = r["fitness"], r["inlier_rmse"]
        iters[k], ncorr[k] = r["iterations"], r["n_corr"]
        prev = cur
        if time.time() - last > 30:
            last = time.time()
            log(f"cpu: {k + 1}/{P} pairs, {last - t0:.0f} s", flush=True)
    return dict(transformation=T, fitness=fit, inlier_rmse=rmse, iterations=iters,
                n_corr=ncorr, seconds=time.time() - t0, threads=threads)


def run_gpu(seq):
    """The bench's batch; returns (results, device, handles) -- the handles stay resident for
    explain()."""
    from lidar_slam_arvc_amd import _lib
    dev = _lib.device(0)
    ids = [dev.upload(s) for s in seq.scans]
    dev.preprocess(ids, _lib.prep_params())
    res = dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, _lib.icp_params())
    return {k: np.array(v) for k, v in res.items()}, dev, ids


def _dRdt(A, B):
    return (float(np.abs(A[:3, :3] - B[:3, :3]).max()), float(np.abs(A[:3, 3] - B[:3, 3]).max()))


def explain(seq, pairs, gpu, cpu, dev, ids, threads, log=print):
    """Pairs outside the bar, three ways: the GPU, the C++ oracle and the NumPy oracle on the
    same clouds; the target normals of the GPU against both oracles' (points whose normals
    differ by more than 1e-6 in |cos|, with their neighbourhood sizes); and the C++ oracle's ICP
    run with the GPU's normals, which isolates the normals' share of the difference."""
    from oracle import cpu_ref as C
    from oracle import open3d_restated as O
    C.set_threads(threads)
    out = []
    for k in pairs:
        tgt = C.filter_radius_height(seq.scans[k])
        src = C.filter_radius_height(seq.scans[k + 1])
        g_pts, g_nrm = dev.download(ids[k], normals=True)
        assert np.array_equal(g_pts, tgt)
        c_nrm, c_cnt = C.estimate_normals(tgt, return_counts=True)
        p_nrm = O.estimate_normals(tgt)
        dot_c = np.abs((g_nrm * c_nrm).sum(1))
        dot_p = np.abs((g_nrm * p_nrm).sum(1))
        dot_cp = np.abs((c_nrm * p_nrm).sum(1))
        bad = np.flatnonzero(dot_c < 1 - 1e-6)
        Tg, Tc = gpu["transformation"][k], cpu["transformation"][k]
        r_p = O.registration_icp(src, tgt, 10.0, seq.priors[k], "p2plane", p_nrm)
        r_cg = C.registration_icp(src, tgt, 10.0, seq.priors[k], "p2plane", g_nrm)
        row = {"pair": int(k),
               "gpu_vs_cpp": _dRdt(Tg, Tc), "gpu_vs_numpy": _dRdt(Tg, r_p["transformation"]),
               "cpp_vs_numpy": _dRdt(Tc, r_p["transformation"]),
               "cpp_icp_with_gpu_normals_vs_gpu": _dRdt(r_cg["transformation"], Tg),
               "iters": [int(gpu["iterations"][k]), int(cpu["iterations"][k]),
                         int(r_p["iterations"])],
               "normals_differing_gpu_cpp": int(len(bad)),
               "normals_differing_gpu_numpy": int((dot_p < 1 - 1e-6).sum()),
               "normals_differing_cpp_numpy": int((dot_cp < 1 - 1e-6).sum()),
               "neighbourhood_sizes_of_differing": sorted(int(c) for c in c_cnt[bad])[:40],
               "points": int(len(tgt))}
        out.append(row)
        log(json.dumps(row), flush=True)
    return out


def compare(gpu, cpu) -> dict:
    Tg = np.asarray(gpu["transformation"]).reshape(-1, 4, 4)
    Tc = np.asarray(cpu["transformation"]).reshape(-1, 4, 4)
    P = len(Tc)
    dR = np.abs(Tg[:, :3, :3] - Tc[:, :3, :3]).reshape(P, -1).max(axis=1)
    dt = np.abs(Tg[:, :3, 3] - Tc[:, :3, 3]).max(axis=1)
    ig, ic = np.asarray(gpu["iterations"]), np.asarray(cpu["iterations"])
    conv = (ig < MAX_ITER) & (ic < MAX_ITER)
    inside = (dR <= TOL_R) & (dt <= TOL_T)
    dfit = np.asarray(gpu["fitness"]) - np.asarray(cpu["fitness"])
    drmse = np.asarray(gpu["inlier_rmse"]) - np.asarray(cpu["inlier_rmse"])
    nonconv = np.flatnonzero(~conv)
    worst_c = int(np.argmax(np.maximum(dR / TOL_R, dt / TOL_T) * conv)) if conv.any() else -1
    return {
        "pairs": int(P),
        "within_tolerance": int(inside.sum()),
        "within_tolerance_fraction": round(float(inside.mean()), 6),
        "tolerance": {"R_abs": TOL_R, "t_abs_m": TOL_T},
        "converged_both": int(conv.sum()),
        "converged_within_tolerance": int((inside & conv).sum()),
        "worst_converged": {"dR": float(dR[conv].max()) if conv.any() else None,
                            "dt_m": float(dt[conv].max()) if conv.any() else None,
                            "pair": worst_c},
        "median_converged": {"dR": float(np.median(dR[conv])) if conv.any() else None,
                             "dt_m": float(np.median(dt[conv])) if conv.any() else None},
        "iterations_equal": int((ig == ic).sum()),
        "iterations_abs_diff_max_converged": int(np.abs(ig - ic)[conv].max()) if conv.any() else 0,
        "fitness_abs_diff_max_converged": float(np.abs(dfit[conv]).max()) if conv.any() else 0.0,
        "rmse_abs_diff_max_converged": float(np.abs(drmse[conv]).max()) if conv.any() else 0.0,
        "nonconverged": {
            "count": int(len(nonconv)),
            "gpu_hit_max_iteration": int((ig >= MAX_ITER).sum()),
            "cpu_hit_max_iteration": int((ic >= MAX_ITER).sum()),
            "within_tolerance": int(inside[nonconv].sum()),
            "pairs": [{"pair": int(k), "iters_gpu": int(ig[k]), "iters_cpu": int(ic[k]),
                       "dR": float(dR[k]), "dt_m": float(dt[k]),
                       "fitness_gpu": float(gpu["fitness"][k]),
                       "fitness_cpu": float(cpu["fitness"][k]),
                       "rmse_gpu": float(gpu["inlier_rmse"][k]),
                       "rmse_cpu": float(cpu["inlier_rmse"][k])} for k in nonconv],
        },
        "outside_tolerance_converged": [int(k) for k in np.flatnonzero(conv & ~inside)],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1999)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--make-cpu", default="", help="CPU side only: write the oracle fixture here")
    ap.add_argument("--cpu", default=os.path.join(ROOT, "tests", "golden",
                                                  "seed3_seq_cpu_oracle.npz"))
    ap.add_argument("--cpu-live", action="store_true",
                    help="run the C++ oracle here instead of reading the fixture")
    ap.add_argument("--threads", type=int, default=0, help="0: every core this process may use")
    ap.add_argument("--out", default="")
    ap.add_argument("--explain", action="store_true",
                    help="three-way analysis (GPU / C++ / NumPy oracle, normals) of every pair "
                         "outside the bar")
    ap.add_argument("--save-gpu", default="", help="write the GPU's per-pair results here")
    args = ap.parse_args()
    threads = args.threads or len(os.sched_getaffinity(0))

    t0 = time.time()
    seq = sequence(args.pairs, args.seed)
    digest = seq_hash(seq)
    print(f"sequence: {len(seq.scans)} keyframes in {time.time() - t0:.1f} s, sha256 {digest}",
          flush=True)
    if args.make_cpu:
        cpu = run_cpu(seq, threads)
        np.savez_compressed(args.make_cpu, sha256=digest, seed=args.seed, **cpu)
        print(f"cpu oracle: {args.pairs} pairs in {cpu['seconds']:.1f} s on {threads} threads "
              f"-> {args.make_cpu}", flush=True)
        return

    gpu, dev, ids = run_gpu(seq)
    print(f"gpu: {args.pairs} pairs done", flush=True)
    if args.cpu_live:
        cpu = run_cpu(seq, threads)
        src = f"C++ oracle run live on {threads} threads ({cpu['seconds']:.1f} s)"
    else:
        z = np.load(args.cpu)
        if str(z["sha256"]) != digest:
            raise SystemExit(f"fixture {args.cpu} was made from a different sequence")
        cpu = {k: z[k] for k in z.files}
        src = (f"{os.path.relpath(args.cpu, ROOT)} (C++ oracle, {int(z['threads'])} threads, "
               f"{float(z['seconds']):.0f} s; same sequence sha256)")
    summary = compare(gpu, cpu)
    summary = {"workload": f"hdl64_64k_p2plane_seq seed {args.seed}, {args.pairs} pairs",
               "sequence_sha256": digest, "checker": src, **summary}
    if args.explain:
        P = len(cpu["transformation"])
        Tg = np.asarray(gpu["transformation"]).reshape(P, 4, 4)
        Tc = np.asarray(cpu["transformation"]).reshape(P, 4, 4)
        far = [k for k in range(P)
               if np.abs(Tg[k, :3, :3] - Tc[k, :3, :3]).max() > TOL_R or
               np.abs(Tg[k, :3, 3] - Tc[k, :3, 3]).max() > TOL_T]
        summary["outside_explained"] = explain(seq, far, gpu, cpu, dev, ids, threads)
    if args.save_gpu:
        np.savez_compressed(args.save_gpu, sha256=digest, **gpu)
    for h in ids:
        dev.release(h)
    text = json.dumps(summary, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
