"""Bench-workload parity: every pair of one of bench.py's batches through the GPU path and
through the f64 C++/OpenMP CPU implementation of the same path (oracle/cpu/lsm_cpu.cpp, the
checker), then a summary. Workloads (``--workload``, the same names and seeds as bench.py):

* hdl64_seq (C3): the seed-3 sequence, 2000 HDL-64 keyframes, 1999 consecutive P2Plane pairs --
  keyframe.py:246-252 (registration_icp, P2Plane, max_corr 10 m, Open3D's default criteria) on
  the pairs of run_scanmatcher.py:196-213, each seeded with its odometry prior;
* loop_closure (C4): rank 0's 512 independent seed-4 revisit pairs (the loop-closure ICPs of
  loopclosing.py:80-99 / 163-180, scaled to a batch), both keyframes pre-processed, P2Plane,
  init = the perturbed revisit pose; the GPU side runs them as bench.py does (lazy normals);
* ouster_multiscale (C5): rank 0's 512 consecutive pairs of the seed-5 Ouster-128 sequence
  through the 3-scale chain (filter, voxel 0.4 / 0.2 / 0.1 m -- keyframe.py:150-151 / 158-159 --,
  normals, P2Plane ICP with max_corr 2 / 1 / 0.5 m; lidar_slam_arvc_amd/multiscale.py); every
  stage is compared.

Two modes:

  python tools/bench_parity.py [--workload W] --make-cpu OUT.npz
      CPU side only (any host; all cores): writes the oracle's per-pair results together with a
      SHA-256 of the generated sequence, so a GPU run elsewhere can prove it saw the same data.

  python tools/bench_parity.py [--workload W] [--cpu FIXTURE.npz | --cpu-live] [--out SUMMARY.json]
      GPU side (the bench's own batch: pre-process every keyframe, one ICP batch per stage),
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


WORKLOADS = {   # name -> (default pairs, default seed, fixture under tests/golden)
    "hdl64_seq": (1999, 3, "seed3_seq_cpu_oracle.npz"),
    "loop_closure": (512, 4, "seed4_loop_cpu_oracle.npz"),
    "ouster_multiscale": (512, 5, "seed5_ouster_cpu_oracle.npz"),
}


def sequence(P: int, seed: int, workload: str = "hdl64_seq", processes: int = 0):
    """bench.py's rank-0 data of `workload` (first_index 0). loop_closure: a Sequence whose scans
    are the P targets then the P sources and whose priors are the P initial guesses (bench.py's
    layout)."""
    from lidar_slam_arvc_amd import synthetic
    procs = processes or max(1, min(16, len(os.sched_getaffinity(0))))
    if workload == "loop_closure":
        ps = synthetic.make_revisit_pairs(P, seed=seed, model=synthetic.HDL64, processes=procs)
        return synthetic.Sequence(ps.targets + ps.sources, np.zeros((0, 4, 4)), ps.init)
    model = synthetic.OUSTER128 if workload == "ouster_multiscale" else synthetic.HDL64
    return synthetic.make_sequence(P + 1, seed=seed, model=model, processes=procs)


def pair_clouds(seq, workload: str):
    """(source index, target index) of every pair into seq.scans, in bench.py's order."""
    if workload == "loop_closure":
        P = len(seq.priors)
        return [(P + k, k) for k in range(P)]
    return [(k + 1, k) for k in range(len(seq.scans) - 1)]


def seq_hash(seq) -> str:
    h = hashlib.sha256()
    for s in seq.scans:
        h.update(np.ascontiguousarray(s, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(seq.priors, dtype=np.float64).tobytes())
    return h.hexdigest()


def run_cpu_multiscale(seq, threads: int, log=print):
    """C5: the C++ oracle's 3-scale chain on every consecutive pair (cpu_ref.registration_multiscale:
    filter, then per scale voxel + normals of the target + ICP from the previous stage's T).
    Results per stage: arrays with a leading stage axis."""
    from oracle import cpu_ref as C
    C.set_threads(threads)
    P = len(seq.scans) - 1
    S = 3
    T = np.zeros((S, P, 4, 4))
    fit, rmse = np.zeros((S, P)), np.zeros((S, P))
    iters, ncorr = np.zeros((S, P), np.int32), np.zeros((S, P), np.int64)
    t0 = last = time.time()
    for k in range(P):
        for s, r in enumerate(C.registration_multiscale(seq.scans[k + 1], seq.scans[k],
                                                        seq.priors[k])):
            T[s, k] = r["transformation"]
            fit[s, k], rmse[s, k] = r["fitness"], r["inlier_rmse"]
            iters[s, k], ncorr[s, k] = r["iterations"], r["n_corr"]
        if time.time() - last > 30:
            last = time.time()
            log(f"cpu: {k + 1}/{P} pairs, {last - t0:.0f} s", flush=True)
    return dict(transformation=T, fitness=fit, inlier_rmse=rmse, iterations=iters,
                n_corr=ncorr, seconds=time.time() - t0, threads=threads)


def run_cpu(seq, threads: int, log=print, workload: str = "hdl64_seq"):
    """The C++ oracle on every pair: filter + normals per keyframe, then registration_icp."""
    from oracle import cpu_ref as C
    if workload == "ouster_multiscale":
        return run_cpu_multiscale(seq, threads, log)
    C.set_threads(threads)
    if workload == "loop_closure":
        P = len(seq.priors)
        T = np.zeros((P, 4, 4))
        fit, rmse = np.zeros(P), np.zeros(P)
        iters, ncorr = np.zeros(P, np.int32), np.zeros(P, np.int64)
        t0 = last = time.time()
        for k, (si, ti) in enumerate(pair_clouds(seq, workload)):
            tp = C.filter_radius_height(seq.scans[ti])
            sp = C.filter_radius_height(seq.scans[si])
            r = C.registration_icp(sp, tp, 10.0, seq.priors[k], "p2plane",
                                   C.estimate_normals(tp))
            T[k] = r["transformation"]
            fit[k], rmse[k] = r["fitness"], r["inlier_rmse"]
            iters[k], ncorr[k] = r["iterations"], r["n_corr"]
            if time.time() - last > 30:
                last = time.time()
                log(f"cpu: {k + 1}/{P} pairs, {last - t0:.0f} s", flush=True)
        return dict(transformation=T, fitness=fit, inlier_rmse=rmse, iterations=iters,
                    n_corr=ncorr, seconds=time.time() - t0, threads=threads)
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


def run_gpu(seq, workload: str = "hdl64_seq", dev=None):
    """The bench's batch, as bench.py's step runs it (normals: eager for hdl64_seq, lazy for the
    other two); returns (results, device, handles) -- the handles stay resident for explain().
    ouster_multiscale: arrays with a leading stage axis (the handles are the raw scans)."""
    from lidar_slam_arvc_amd import _lib
    dev = dev or _lib.device(0)
    ids = [dev.upload(s) for s in seq.scans]
    if workload == "ouster_multiscale":
        from lidar_slam_arvc_amd.multiscale import MultiScaleSet
        P = len(seq.scans) - 1
        with MultiScaleSet(dev, ids) as ms:
            ms.preprocess(want_normals="lazy")
            stages = ms.register(list(range(1, P + 1)), list(range(P)), seq.priors, arrays=True)
        res = {k: np.stack([np.asarray(st[k]) for st in stages]) for k in stages[0]}
        return res, dev, ids
    if workload == "loop_closure":
        P = len(seq.priors)
        dev.preprocess(ids, _lib.prep_params(want_normals="lazy"))
        res = dev.icp_batch_arrays(ids[P:], ids[:P], seq.priors, _lib.icp_params())
    else:
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
        # every pair outside the bar, itemised (both sides' iterations, fitness and rmse)
        "outside_tolerance": [{"pair": int(k), "dR": float(dR[k]), "dt_m": float(dt[k]),
                               "iters_gpu": int(ig[k]), "iters_cpu": int(ic[k]),
                               "fitness_gpu": float(gpu["fitness"][k]),
                               "fitness_cpu": float(cpu["fitness"][k]),
                               "rmse_gpu": float(gpu["inlier_rmse"][k]),
                               "rmse_cpu": float(cpu["inlier_rmse"][k])}
                              for k in np.flatnonzero(~inside)],
    }


def compare_workload(gpu, cpu, workload: str) -> dict:
    """compare() of the final results; ouster_multiscale: of the last stage, plus every stage's
    within-tolerance count (each stage is the reference's single-scale operator)."""
    if workload != "ouster_multiscale":
        return compare(gpu, cpu)
    S = np.asarray(cpu["transformation"]).shape[0]
    keys = ("transformation", "fitness", "inlier_rmse", "iterations")
    out = compare({k: np.asarray(gpu[k])[S - 1] for k in keys},
                  {k: np.asarray(cpu[k])[S - 1] for k in keys})
    out["stages"] = [{"stage": s, **{k: v for k, v in compare(
        {k: np.asarray(gpu[k])[s] for k in keys},
        {k: np.asarray(cpu[k])[s] for k in keys}).items()
        if k in ("pairs", "within_tolerance", "converged_both", "iterations_equal",
                 "worst_converged", "outside_tolerance_converged",
                 "outside_tolerance")}} for s in range(S)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="hdl64_seq", choices=sorted(WORKLOADS))
    ap.add_argument("--pairs", type=int, default=0, help="0: the workload's bench.py default")
    ap.add_argument("--seed", type=int, default=-1, help="-1: the workload's bench.py default")
    ap.add_argument("--make-cpu", default="", help="CPU side only: write the oracle fixture here")
    ap.add_argument("--cpu", default="", help="fixture (default: tests/golden/<workload's>)")
    ap.add_argument("--cpu-live", action="store_true",
                    help="run the C++ oracle here instead of reading the fixture")
    ap.add_argument("--threads", type=int, default=0, help="0: every core this process may use")
    ap.add_argument("--out", default="")
    ap.add_argument("--explain", action="store_true",
                    help="hdl64_seq: three-way analysis (GPU / C++ / NumPy oracle, normals) of "
                         "every pair outside the bar")
    ap.add_argument("--save-gpu", default="", help="write the GPU's per-pair results here")
    args = ap.parse_args()
    threads = args.threads or len(os.sched_getaffinity(0))
    P0, seed0, fixture = WORKLOADS[args.workload]
    args.pairs = args.pairs or P0
    args.seed = args.seed if args.seed >= 0 else seed0
    args.cpu = args.cpu or os.path.join(ROOT, "tests", "golden", fixture)

    t0 = time.time()
    seq = sequence(args.pairs, args.seed, args.workload)
    digest = seq_hash(seq)
    print(f"{args.workload}: {len(seq.scans)} clouds in {time.time() - t0:.1f} s, "
          f"sha256 {digest}", flush=True)
    if args.make_cpu:
        cpu = run_cpu(seq, threads, workload=args.workload)
        np.savez_compressed(args.make_cpu, sha256=digest, seed=args.seed,
                            workload=args.workload, **cpu)
        print(f"cpu oracle: {args.pairs} pairs in {cpu['seconds']:.1f} s on {threads} threads "
              f"-> {args.make_cpu}", flush=True)
        return

    gpu, dev, ids = run_gpu(seq, args.workload)
    print(f"gpu: {args.pairs} pairs done", flush=True)
    if args.cpu_live:
        cpu = run_cpu(seq, threads, workload=args.workload)
        src = f"C++ oracle run live on {threads} threads ({cpu['seconds']:.1f} s)"
    else:
        z = np.load(args.cpu)
        if str(z["sha256"]) != digest:
            raise SystemExit(f"fixture {args.cpu} was made from a different sequence")
        cpu = {k: z[k] for k in z.files}
        src = (f"{os.path.relpath(args.cpu, ROOT)} (C++ oracle, {int(z['threads'])} threads, "
               f"{float(z['seconds']):.0f} s; same clouds' sha256)")
    summary = compare_workload(gpu, cpu, args.workload)
    summary = {"workload": f"{args.workload} seed {args.seed}, {args.pairs} pairs",
               "sequence_sha256": digest, "checker": src, **summary}
    if args.explain and args.workload == "hdl64_seq":
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
