"""Benchmark: ICP keyframe-pair registrations/s on 64k-point HDL-64-style scans (BASELINE.json).

One step = the reference's scan-matcher hot path (run_scanmatcher.py:196-213) over one batch of
synthetic input already resident in HBM: pre-process P+1 keyframes (filter_radius_height +
estimate_normals, keyframe.py:156-162), register the P consecutive pairs with point-to-plane ICP
(keyframe.py:249-252, Open3D criteria), fetch the P relative transforms to the host and compose
the global poses (homogeneousmatrix.py:184-205; RCCL all-gather of chunk totals when N > 1).
The default P = 1999 is BASELINE.json's C3 workload, a 2000-keyframe sequence on one GPU.
Weak scaling: every GPU owns P pairs of one long sequence (distributed.py).

    python bench.py [--gpus N --steps K --warmup W --pairs-per-gpu P]

Prints one JSON line (rank 0) with the roofline of the NN correspondence kernel (HIP events on
the library's own stream, SURVEY.md §8d algorithmic bytes), the roofline of the normals kernel
(VALU issue from the committed PMC instruction count, and algorithmic FLOPs from the device's
neighbourhood sizes), a CPU baseline (the C++/OpenMP f64 implementation under oracle/cpu, rank 0
at N = 1 only, bounded sample, every usable core and 1 core) and the lines of configs C1 (8k-point
P2P pairs) and C2 (one 64k P2Plane pair): the CPU implementation, and the same pairs on the GPU.
"""
from __future__ import annotations

import argparse
import functools
import json
import os
import threading
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
FP32_VALU_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md chip-level parameters (vector)
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz, one 64-lane wave instruction per 2 cycles per
# SIMD (MI355X_MICROARCH.md 'Wave scheduling'), in G wave-instructions/s
VALU_ISSUE_PEAK_G = 256 * 4 * 2.4 / 2   # = 1228.8
# f64 add / fma wave-instructions issue at about half that: 498 (v_fma_f64) / 507 (v_add_f64) G/s
# measured with 8 waves per SIMD and 8 independent chains (v_fma_f32 in the same kernel: 868 G/s;
# tools/calib/valu_calib.hip, profiles/r05h/valu_calib.log)
VALU_F64_PEAK_G = 500.0
KERNELS = ["filter", "grid", "normals", "normals_lazy", "normals_refine", "nn", "nn_fallback",
           "accumulate", "solve", "voxel"]


def source_sha() -> str:
    """SHA-256 of the library's sources (lidar_slam_arvc_amd/csrc, include/lidarsm.h): the PMC
    counts committed under profiles/ carry the hash of the build they were counted on, and the
    bench line uses them only while it matches."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "lidar_slam_arvc_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")))
    for f in [os.path.join(csrc, f) for f in files] + [os.path.join(ROOT, "include", "lidarsm.h")]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


# The kernels whose machine code a PMC count depends on: the counted kernels and the grid build
# that lays out what they read (the clouds themselves are pinned bit-exact by the parity tests).
PMC_KERNELS = {
    "nn_traffic.json": ("nn_kernel", "grid_keys", "grid_scatter", "grid_fill"),
    "normals_valu.json": ("normals_sparse_kernel", "normals_dense_kernel", "normals_refine_kernel",
                          "grid_keys", "grid_scatter", "grid_fill"),
}


_GPU_STARTED = [False]   # set before the first GPU call: no child processes from then on


@functools.lru_cache(maxsize=None)
def kernel_sha(prefixes) -> dict:
    """Hashes of the loaded library's gfx950 machine code of the kernels named by `prefixes`
    (tools/kernel_hash.py: disassembly with addresses made relative); {} when unavailable, or
    when first asked for after the GPU was initialised (bench.main computes them before)."""
    if _GPU_STARTED[0]:
        return {}
    try:
        import importlib.util
        from lidar_slam_arvc_amd import _lib
        spec = importlib.util.spec_from_file_location("kernel_hash",
                                                      os.path.join(ROOT, "tools", "kernel_hash.py"))
        kh = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(kh)
        return kh.kernel_hashes(_lib.LIB_PATH, prefixes)
    except Exception:
        return {}


def pmc_entry(name: str, workload: str, pairs: int, mode: str | None = None):
    """The committed PMC summary of this workload (profiles/<name>, keyed by workload), or
    (None, reason) when it is absent, of another size or mode, or counted on other code. A count
    holds for the library sources it was counted on (source_sha256) and for any build whose
    counted kernels and grid build compile to the same machine code (kernel_sha)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, "no PMC file"
    with open(path) as f:
        e = json.load(f).get(workload)
    if not e:
        return None, f"no PMC count for {workload}"
    if e.get("pairs_per_gpu") != pairs or (mode is not None and e.get("normals_mode") != mode):
        return None, "PMC count of another configuration"
    if e.get("source_sha256") == source_sha():
        return e, None
    if e.get("kernel_sha") and e["kernel_sha"] == kernel_sha(tuple(PMC_KERNELS[name])):
        return e, None
    return None, "stale: PMC counted on other kernel code"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="hdl64_seq",
                    choices=["hdl64_seq", "ouster_multiscale", "loop_closure"],
                    help="hdl64_seq: C2/C3 64k HDL-64 sequence pairs (the headline line); "
                         "ouster_multiscale: C5 256k Ouster-128, voxel 0.4/0.2/0.1 m chain; "
                         "loop_closure: C4 independent 64k revisit pairs (sharded, no halo)")
    ap.add_argument("--pairs-per-gpu", type=int, default=0,
                    help="0: 1999 (hdl64: the C3 2000-keyframe sequence), 512 (ouster), "
                         "512 (loop_closure: C4's 4096 pairs over 8 GPUs)")
    ap.add_argument("--seed", type=int, default=-1, help="-1: 3 (hdl64), 5 (ouster)")
    ap.add_argument("--method", default="p2plane", choices=["p2plane", "p2p"])
    ap.add_argument("--normals", default="auto", choices=["auto", "lazy", "eager"],
                    help="eager: every normal of every keyframe in the pre-process; lazy "
                         "(LSM_NORMALS_LAZY): a keyframe's normals are computed when it is first "
                         "a P2Plane target (bit-identical registrations; sources never compute "
                         "theirs); auto: eager for hdl64_seq (every keyframe but the last is a "
                         "target), lazy for loop_closure and ouster_multiscale")
    ap.add_argument("--streams", type=int, default=1,
                    help="hdl64_seq: independent contexts (HIP streams) per GPU, each registering a "
                         "contiguous run of the pairs from its own host thread, so one run's "
                         "latency-bound ICP passes overlap another's normal estimation")
    ap.add_argument("--stagger", action="store_true",
                    help="with --streams S: run k starts its pre-processing when run k - 1's "
                         "ends, so each chunk's registration overlaps the next chunk's normals")
    ap.add_argument("--cpu-sample-pairs", type=int, default=0,
                    help="bounded CPU-baseline sample, 1/12 of it again on 1 core (0: 144 pairs "
                         "for hdl64_seq, 72 for loop_closure, 32 for ouster_multiscale: ~10 s "
                         "each on 16 cores of the GPU box's EPYC)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: every core this process may use (affinity mask, capped by the "
                         "cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-gathered", default="",
                    help="loop_closure (C4): rank 0 writes the last step's gathered transforms of "
                         "all ranks' pairs (global order) to this .npz")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearse the multi-rank path on one GPU: all ranks on device 0, gloo "
                         "collectives on host tensors (tests only; not a scaling measurement)")
    ap.add_argument("--no-c1", action="store_true",
                    help="skip the lines of configs C1 (8k-point P2P pairs) and C2 (one 64k "
                         "P2Plane pair), CPU and GPU")
    ap.add_argument("--no-c45", action="store_true",
                    help="skip the c4 / c5 blocks (configs C4 loop-closure pairs and C5 Ouster-128 "
                         "multi-scale, 512 pairs per GPU each, timed like the main line); "
                         "profiling runs of one workload use it")
    ap.add_argument("--grid-cell", type=float, default=0.0, help="spatial grid cell (m); 0 = library default")
    ap.add_argument("--grid-cell-scales", default="",
                    help="ouster_multiscale: comma-separated grid cell per voxel scale (overrides --grid-cell)")
    ap.add_argument("--seq-cache", default="",
                    help="profiling / A/B runs: load the synthetic data from this .npz if it "
                         "holds this workload's, else generate it and save it there")
    return ap.parse_args()


def load_or_make(path, tag, make):
    """make() -> Sequence, or the one saved at `path` under the same tag (profiling runs: data
    generation forks, which must not happen under the profiler, so a plain run fills the cache)."""
    from lidar_slam_arvc_amd import synthetic
    if path and os.path.exists(path):
        z = np.load(path)
        if str(z["tag"]) == tag:
            n = int(z["nscans"])
            return synthetic.Sequence([z[f"s{k}"] for k in range(n)], z["poses"], z["priors"])
    seq = make()
    if path:
        np.savez(path, tag=tag, nscans=len(seq.scans), poses=seq.poses, priors=seq.priors,
                 **{f"s{k}": s for k, s in enumerate(seq.scans)})
    return seq


def usable_cores() -> int:
    """Cores this process may run on: the affinity mask, capped by a cgroup v2 CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(per))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_host():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model or "unknown CPU", os.cpu_count()


def _cpu_timed(run, n_pairs: int, threads: int, what: str):
    """Time run(n) on `threads` OpenMP threads and a smaller sample on 1 thread."""
    from oracle import cpu_ref as C
    threads = max(1, threads)
    C.load()
    def timed(n, min_s):   # the sample again until it has run >= min_s (small workloads)
        done, t0 = 0, time.perf_counter()
        while True:
            run(n)
            done += n
            dt = time.perf_counter() - t0
            if dt >= min_s:
                return done, dt

    C.set_threads(threads)
    n_all, dt = timed(n_pairs, 5.0)
    C.set_threads(1)
    n1, dt1 = timed(max(1, n_pairs // 12), 5.0)
    model, ncpu = _cpu_host()
    return {"value": round(n_all / dt, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
            "value_1core": round(n1 / dt1, 3),
            "sample": f"{what}: {n_all} pairs on {threads} threads ({dt:.1f} s) and {n1} on 1 "
                      f"thread ({dt1:.1f} s); the C++/OpenMP f64 KD-tree implementation of the "
                      f"path (oracle/cpu/lsm_cpu.cpp, SURVEY.md 8d) on {model}, nproc {ncpu}, "
                      f"{len(os.sched_getaffinity(0))} in the affinity mask, {usable_cores()} "
                      f"usable (cgroup quota)"}


def cpu_baseline(seq, n_pairs: int, method: str, threads: int,
                 what: str = "consecutive pairs of the same synthetic HDL-64 sequence"):
    """The CPU implementation on the first pairs of the same sequence (P+1 keyframes pre-processed
    per P pairs, as in a GPU step)."""
    from oracle import cpu_ref as C

    def run(n):
        pre = []
        for k in range(n + 1):
            pts = C.filter_radius_height(seq.scans[k])
            pre.append((pts, C.estimate_normals(pts) if method == "p2plane" else None))
        for k in range(n):
            C.registration_icp(pre[k + 1][0], pre[k][0], 10.0, seq.priors[k], method, pre[k][1])
    return _cpu_timed(run, n_pairs, threads, what)


def cpu_baseline_multiscale(seq, n_pairs: int, method: str, threads: int):
    """The CPU implementation's multi-scale chain on the first pairs of the same data."""
    from oracle import cpu_ref as C

    def run(n):
        for k in range(n):
            C.registration_multiscale(seq.scans[k + 1], seq.scans[k], seq.priors[k], method=method)
    return _cpu_timed(run, n_pairs, threads, "pairs of the same Ouster-128 sequence through the "
                                             "3-scale chain (both keyframes pre-processed per pair)")


def cpu_baseline_pairs(seq, P: int, n_pairs: int, method: str, threads: int):
    """The CPU implementation on the first independent revisit pairs (both clouds pre-processed)."""
    from oracle import cpu_ref as C

    def run(n):
        for k in range(n):
            tgt = C.filter_radius_height(seq.scans[k])
            src = C.filter_radius_height(seq.scans[P + k])
            nrm = C.estimate_normals(tgt) if method == "p2plane" else None
            if method == "p2plane":
                C.estimate_normals(src)      # the reference pre-processes both keyframes
            C.registration_icp(src, tgt, 10.0, seq.priors[k], method, nrm)
    return _cpu_timed(run, n_pairs, threads, "revisit pairs (both keyframes pre-processed per "
                                             "pair)")


C1_PAIRS = 256


def c1_line(dev, seq, threads: int, cpu_pairs: int = 96):
    """Config C1 (BASELINE.json configs[0]): single 8k-point P2P registrations, Open3D defaults.
    GPU: the 256 consecutive pairs of a seed-1 VLP-16 sequence as one batch (filter + ICP, no
    normals), wall clock per batch with the batch's inputs resident; CPU: the C++ f64
    implementation on the first pairs of the same sequence (every usable core and 1 core)."""
    from lidar_slam_arvc_amd import _lib
    ids = [dev.upload(s) for s in seq.scans]
    prep = _lib.prep_params(want_normals=False)
    icp = _lib.icp_params(method="p2p")
    try:
        def run():
            dev.preprocess(ids, prep)
            return dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, icp)
        run()
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 1.0:
            res = run()
            reps += 1
        dt = (time.perf_counter() - t0) / reps
    finally:
        for h in ids:
            dev.release(h)
    cpu = cpu_baseline(seq, min(cpu_pairs, len(seq.priors)), "p2p", threads,
                       "consecutive pairs of the same synthetic VLP-16 (8k-ray) sequence, P2P")
    return {"workload": "vlp16_8k_p2p_seq (BASELINE.json configs[0]: 8k-pt P2P pairs)",
            "pairs": len(seq.priors), "points_per_scan_post_filter":
                int(np.mean([len(s) for s in seq.scans])),
            "gpu_value": round(len(seq.priors) / dt, 3), "gpu_ms_per_batch": round(dt * 1e3, 3),
            "mean_icp_iterations": float(np.mean(res["iterations"])),
            "unit": "pairs/s", "cpu_baseline": cpu}


def c2_line(dev, seq, threads: int):
    """Config C2 (BASELINE.json configs[1]): one 64k-point HDL-64 scan pair, point-to-plane ICP
    on one GPU (keyframe.py:246-252 after pre_process of both keyframes, keyframe.py:113-124):
    the seed-2 pair test_icp_parity checks against the oracle. GPU: per registration, with the
    raw scans resident, pre-process both keyframes (filter + normals) and register the pair --
    wall-clock latency per pair (mean over repeats) and its inverse; the kernel time split into
    pre-process and ICP. CPU: the C++ implementation on the same pair."""
    from lidar_slam_arvc_amd import _lib
    ids = [dev.upload(s) for s in seq.scans]
    prep = _lib.prep_params()
    icp = _lib.icp_params()
    try:
        def run():
            dev.preprocess(ids, prep)
            return dev.icp_batch_arrays(ids[1:], ids[:1], seq.priors, icp)
        for _ in range(3):
            run()
        dev.reset_stats()
        dev.set_timing(True)
        reps, t0 = 0, time.perf_counter()
        while reps < 20 or time.perf_counter() - t0 < 1.0:
            res = run()
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        dev.set_timing(False)
        k_ms = {k: dev.kernel_stats(k)["ms"] / reps for k in KERNELS}
    finally:
        for h in ids:
            dev.release(h)
    cpu = cpu_baseline(seq, 1, "p2plane", threads,
                       "the same seed-2 HDL-64 pair, P2Plane (both keyframes pre-processed)")
    prep_ms = sum(k_ms[k] for k in ("filter", "grid", "normals", "voxel"))
    icp_ms = sum(k_ms[k] for k in ("nn", "nn_fallback", "accumulate", "solve"))
    return {"workload": "hdl64_64k_p2plane_pair (BASELINE.json configs[1]: one 64k-pt P2Plane "
                        "pair, 1 GPU)",
            "points_per_scan_post_filter": int(np.mean([len(s) for s in seq.scans])),
            "gpu_ms_per_pair": round(dt * 1e3, 3), "gpu_value": round(1.0 / dt, 3),
            "unit": "pairs/s", "icp_iterations": int(res["iterations"][0]),
            "gpu_kernel_ms_per_pair": {"preprocess": round(prep_ms, 3), "icp": round(icp_ms, 3)},
            "cpu_baseline": cpu, "cpu_ms_per_pair": round(1e3 / cpu["value"], 1)}


WORKLOAD_DEFAULTS = {   # bench workload -> (pairs per GPU, seed, LiDAR model name, normals mode)
    "hdl64_seq": (1999, 3, "HDL64", "eager"),           # C3 (and C2's scans)
    "loop_closure": (512, 4, "HDL64", "lazy"),          # C4: 4096 pairs over 8 GPUs
    "ouster_multiscale": (512, 5, "OUSTER128", "lazy"),  # C5
}


def make_data(workload: str, P: int, seed: int, first: int, procs: int, cache: str = ""):
    """The rank's synthetic data of `workload` (forked ray-cast workers: call before the GPU is
    touched). loop_closure: scans = the P targets then the P sources, priors = the P initial
    guesses; otherwise P + 1 consecutive keyframes of one sequence."""
    from lidar_slam_arvc_amd import synthetic
    model = getattr(synthetic, WORKLOAD_DEFAULTS[workload][2])
    tag = f"{workload}_{P}_{seed}_{model.rings}x{model.azimuths}_{first}"
    if workload == "loop_closure":
        def make():
            ps = synthetic.make_revisit_pairs(P, seed=seed, model=model, first_index=first,
                                              processes=procs)
            return synthetic.Sequence(ps.targets + ps.sources, np.zeros((0, 4, 4)), ps.init)
    else:
        def make():
            return synthetic.make_sequence(P + 1, seed=seed, model=model, first_index=first,
                                           processes=procs)
    return load_or_make(cache, tag, make)


def run_workload(workload, seq, P, args, *, gpu, local, rank, world, group, cuda, normals,
                 streams=1, grid_cell=0.0, grid_cells=None, do_cpu=False, cpu_threads=1,
                 cpu_sample=0):
    """Upload `seq`, run W untimed and K timed steps of `workload` (barrier + synchronize on both
    sides, max over ranks) and return (rank 0) its bench line without the top-level extras:
    metric, value, config, roofline, roofline_normals, cpu_baseline, breakdown. Every rank must
    call it (the steps' collectives)."""
    from lidar_slam_arvc_amd import _lib
    from lidar_slam_arvc_amd.distributed import compose_global_sharded, gather_pair_results
    import torch
    import torch.distributed as dist

    ouster = workload == "ouster_multiscale"
    loop = workload == "loop_closure"
    first = rank * P
    extra_ids = []                                   # (context, handle) of extra runs
    dev = _lib.device(gpu)
    ids = [dev.upload(s) for s in seq.scans]        # raw scans resident in HBM
    devs = [dev]
    want_normals = args.method == "p2plane"
    # pre-process normals mode: "lazy" computes only the target normals the registration reads
    wn_mode = ("lazy" if normals == "lazy" else True) if want_normals else False
    ms = None
    S = 1
    gathered = [None]   # loop_closure: every rank's pair results of the last step, global order
    if ouster:
        from lidar_slam_arvc_amd.multiscale import MultiScaleSet
        ms = MultiScaleSet(dev, ids)                 # per-scale device clones, made once
        n_fine = []   # points per scan at the finest scale: the same every step, read once

        def step():
            ms.preprocess(want_normals=wn_mode, grid_cell=grid_cell, grid_cells=grid_cells)
            stages = ms.register(list(range(1, P + 1)), list(range(P)), seq.priors,
                                 method=args.method, arrays=True)
            res = stages[-1]
            compose_global_sharded(res["transformation"], group=group, device=cuda)
            if not n_fine:
                n_fine.extend(dev.info(h)[1] for h in ms.handles[-1])
            return n_fine, res
    elif loop:
        prep = _lib.prep_params(want_normals=wn_mode, grid_cell=grid_cell)
        icp = _lib.icp_params(method=args.method)

        def step():
            n = dev.preprocess(ids, prep)
            res = dev.icp_batch_arrays(ids[P:], ids[:P], seq.priors, icp)
            rel = res["transformation"]
            if group is not None:   # the sequence-level exchange: gather every pair's result
                gathered[0] = gather_pair_results(rel, np.arange(first, first + P), world * P,
                                                  group=group, device=cuda)
            else:
                gathered[0] = rel
            return n, res
    else:
        prep = _lib.prep_params(want_normals=wn_mode, grid_cell=grid_cell)
        icp = _lib.icp_params(method=args.method)
        S = max(1, min(streams, P))
        cut = [round(k * P / S) for k in range(S + 1)]          # pair runs [cut[s], cut[s+1])
        devs = [dev] + [_lib.Device(gpu) for _ in range(S - 1)]
        # run s owns keyframes cut[s] .. cut[s+1] (the shared end keyframe is in both runs)
        run_ids = [ids[cut[0]:cut[1] + 1]] + [[devs[k].upload(seq.scans[j])
                                                for j in range(cut[k], cut[k + 1] + 1)]
                                               for k in range(1, S)]
        extra_ids.extend((devs[k], h) for k in range(1, S) for h in run_ids[k])

        def run(k, out, gates):
            d, hs = devs[k], run_ids[k]
            if gates is not None and k > 0:
                gates[k - 1].wait()     # --stagger: pre-process after the previous run's
            try:
                n = d.preprocess(hs, prep)
            finally:
                if gates is not None:
                    gates[k].set()
            out[k] = (n if k == 0 else n[1:], d.icp_batch_arrays(hs[1:], hs[:-1],
                                                                 seq.priors[cut[k]:cut[k + 1]],
                                                                 icp))

        def step():
            out = [None] * S
            # --stagger: run k pre-processes (VALU-bound normals) while run k - 1 registers
            # (latency-bound ICP passes) -- a pipeline over the sequence's chunks
            gates = [threading.Event() for _ in range(S)] if args.stagger else None
            th = [threading.Thread(target=run, args=(k, out, gates)) for k in range(1, S)]
            for t in th:
                t.start()
            run(0, out, gates)
            for t in th:
                t.join()
            if any(o is None for o in out):
                raise RuntimeError("a registration run failed")
            n = np.concatenate([o[0] for o in out])
            res = {key: np.concatenate([o[1][key] for o in out]) for key in out[0][1]}
            rel = res["transformation"]
            compose_global_sharded(rel, group=group, device=cuda)
            return n, res

    try:
        for _ in range(args.warmup):
            step()
        for d in devs:
            d.reset_stats()
            d.set_timing(True)
        if group is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        last = None
        for _ in range(args.steps):
            last = step()
        torch.cuda.synchronize()
        if group is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        for d in devs:
            d.set_timing(False)
        if group is not None:
            t = torch.tensor([dt], dtype=torch.float64, device=cuda)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())

        def kstats(name):   # summed over the contexts (their kernels may overlap in time)
            tot = {"launches": 0, "ms": 0.0, "algo_bytes": 0.0}
            for d in devs:
                st = d.kernel_stats(name)
                for key in tot:
                    tot[key] += st[key]
            return tot

        stats = {k: kstats(k) for k in KERNELS}
        nn = kstats("nn_pass")   # check + search + fallback of every ICP pass
        cnt = {k: kstats(k)["launches"] for k in ("nn_uncertified", "nn_queries",
                                                  "nn_queries_first_pass", "nn_pending",
                                                  "nn_pending_first_pass")}
        roof_n = None
        norm_ms = stats["normals"]["ms"] + stats["normals_lazy"]["ms"]   # every normals launch
        if want_normals and norm_ms > 0 and len(devs) == 1:
            # neighbourhood sizes of the normals one step computes: one more (untimed) step in
            # statistics mode (every rank runs it: the step's collectives need all ranks)
            d0 = devs[0]
            d0.reset_stats()
            d0.set_timing(True, statistics=True)
            try:
                step()
            finally:
                d0.set_timing(False)
            nb = d0.kernel_stats("normals_neighbours")["launches"]
            npts = d0.kernel_stats("normals_points")["launches"]
            step_s = norm_ms / args.steps * 1e-3
            flops = 18.0 * nb + 150.0 * npts
            valu, valu_k, f64 = None, None, None
            # PMC count of the same workload and normals mode (profiles/normals_valu.json)
            vj, v_why = pmc_entry("normals_valu.json", workload, P, normals)
            if vj:
                # the refine kernel (0.2 % of the VALU) runs on the library's side stream,
                # overlapping the ICP, outside the timed normals windows: left out of the count too
                pk = {k: v for k, v in vj.get("per_kernel_per_step", {}).items()
                      if k != "normals_refine_kernel"}
                valu_k = {k: v.get("SQ_INSTS_VALU") for k, v in pk.items()}
                valu = sum(v or 0.0 for v in valu_k.values()) if valu_k else vj.get("valu_per_step")
                f64 = sum(v.get("SQ_INSTS_VALU_ADD_F64", 0.0) + v.get("SQ_INSTS_VALU_FMA_F64", 0.0)
                          for v in pk.values())
            ach = valu / step_s / 1e9 if valu else None
            # issue time at peak with the f64 add / fma instructions at their measured rate (the
            # other f64 instructions -- mul, conversions, compares -- are counted at the f32 rate)
            t_peak = ((valu - f64) / (VALU_ISSUE_PEAK_G * 1e9) + f64 / (VALU_F64_PEAK_G * 1e9)
                      if valu and f64 is not None else None)
            roof_n = {"bound": "valu", "kernel": "normals_sparse_kernel + normals_dense_kernel "
                                                 "(the split launch, its refine kernel overlapped "
                                                 "with the ICP on a side stream; " +
                                                 ("each keyframe's normals when it is first a "
                                                  "P2Plane target" if normals == "lazy" else
                                                  "every keyframe, once per step") +
                                                 "): hybrid kNN-300 / r 0.3 m",
                      "mode": normals, "unit": "G wave-instructions/s",
                      "valu_source": "profiles/normals_valu.json" if vj else v_why,
                      "achieved": round(ach, 2) if ach else None, "peak": VALU_ISSUE_PEAK_G,
                      "frac": round(ach / VALU_ISSUE_PEAK_G, 5) if ach else None,
                      "valu_instructions_per_step": valu,
                      "valu_instructions_per_kernel": valu_k,
                      "f64_add_fma_per_step": f64,
                      "f64_weighted": ({"issue_ms_at_peak": round(t_peak * 1e3, 3),
                                        "frac": round(t_peak / step_s, 5),
                                        "peaks_G_per_s": {"f64_add_fma": VALU_F64_PEAK_G,
                                                          "other": VALU_ISSUE_PEAK_G},
                                        "source": "tools/calib/valu_calib.hip "
                                                  "(profiles/r05h/valu_calib.log)"}
                                       if t_peak else None),
                      "ms_per_step": round(step_s * 1e3, 4),
                      # the refine kernel's own window on the side stream (it overlaps the ICP's
                      # first correspondence pass, so it is not part of ms_per_step)
                      "refine_ms_per_step_overlapped": round(stats["normals_refine"]["ms"] /
                                                             args.steps, 4),
                      "launches_per_step": (stats["normals"]["launches"] +
                                            stats["normals_lazy"]["launches"]) / args.steps,
                      "flops": {"unit": "TFLOP/s", "achieved": round(flops / step_s / 1e12, 4),
                                "peak": FP32_VALU_PEAK_TFLOPS,
                                "frac": round(flops / step_s / 1e12 / FP32_VALU_PEAK_TFLOPS, 6),
                                "flops_per_step": flops,
                                "model": "SURVEY.md 8d: 18 FLOP per neighbour (9 cumulant FMAs, "
                                         "computed in f64) + 150 per point (covariance, "
                                         "FastEigen3x3); neighbourhood sizes counted on the "
                                         "device",
                                "normals_per_step": npts,
                                "neighbours_per_normal": round(nb / max(npts, 1), 3)}}
        # The boundary's host -> device leg: the timed steps read raw scans already
        # resident in HBM; a pipeline that uploads every keyframe first also pays this (pageable
        # numpy buffers through lsm_cloud_upload: one allocation, copy and synchronisation each)
        # -- as one batch (lsm_cloud_upload_batch) and scan by scan (lsm_cloud_upload), twice
        # alternating, the faster of each
        torch.cuda.synchronize()
        up_s = up1_s = float("inf")
        for _ in range(2):
            t1 = time.perf_counter()
            up_ids = dev.upload_many(seq.scans)
            up_s = min(up_s, time.perf_counter() - t1)
            for h in up_ids:
                dev.release(h)
            t1 = time.perf_counter()
            up_ids = [dev.upload(s) for s in seq.scans]
            up1_s = min(up1_s, time.perf_counter() - t1)
            for h in up_ids:
                dev.release(h)
        up_bytes = sum(int(np.asarray(s).shape[0]) * 12 for s in seq.scans)
    finally:
        if ms is not None:
            ms.release()
        for i in ids:
            dev.release(i)
        for d, h in extra_ids:
            d.release(h)
        for d in devs[1:]:
            d.close()

    n_pts, res = last
    iters = list(res["iterations"])
    if loop and rank == 0 and args.save_gathered:
        # the gathered transforms of all world x P pairs (tools/c4_gather_check.py compares them
        # with one context registering every pair in one batch)
        np.savez_compressed(args.save_gathered, transformation=gathered[0], world=world,
                            pairs_per_rank=P, seed=args.seed if args.seed >= 0 else 4)
    if rank != 0:
        return None
    achieved = nn["algo_bytes"] / (nn["ms"] * 1e-3) / 1e9 if nn["ms"] > 0 else 0.0
    # PMC traffic of the same workload (profiles/nn_traffic.json, tools/pmc_nn.sh)
    tj, t_why = pmc_entry("nn_traffic.json", workload, P)
    traffic = tj.get("hbm_bytes_per_launch") if tj else None
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": "profiles/nn_traffic.json" if tj else t_why,
            "traffic_over_algorithmic": (round(traffic / (nn["algo_bytes"] /
                                                          max(nn["launches"], 1)), 3)
                                         if traffic and nn["algo_bytes"] else None),
            "kernel": "correspondence pass: nn_kernel (stability check + box search) + "
                      "nn_fallback",
            "algo_bytes_per_launch": nn["algo_bytes"] / max(nn["launches"], 1),
            "avg_launch_ms": nn["ms"] / max(nn["launches"], 1),
            "launches": nn["launches"],
            "per_kernel_ms_per_pass": {k: round(stats[k]["ms"] / max(nn["launches"], 1), 5)
                                       for k in ("nn", "nn_fallback")}}
    cpu = None
    if do_cpu:
        ns = cpu_sample or (32 if ouster else (72 if loop else 144))
        ns = max(1, min(ns, P))
        if ouster:
            cpu = cpu_baseline_multiscale(seq, ns, args.method, cpu_threads)
        elif loop:
            cpu = cpu_baseline_pairs(seq, P, ns, args.method, cpu_threads)
        else:
            cpu = cpu_baseline(seq, ns, args.method, cpu_threads)
    ms_step = dt / args.steps * 1e3
    return {
        "metric": ("ICP keyframe-pair registrations/sec (256k-ray Ouster-128, multi-scale)"
                   if ouster else "ICP keyframe-pair registrations/sec (64k-pt scans)"),
        "value": round(world * P * args.steps / dt, 3),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+f64",
        "data": "synthetic (seeded ray-cast %s scans of a procedural scene)"
                % ("Ouster-128" if ouster else "HDL-64"),
        "config": ({"workload": f"ouster128_256k_{args.method}_multiscale_seq",
                    "baseline_config": "BASELINE.json configs[4] (C5)",
                    "pairs_per_gpu": P, "global_pairs": world * P,
                    "points_per_scan_finest_voxel": int(np.mean(n_pts)),
                    "rays_per_scan": 262144, "method": args.method,
                    "voxel_scales": [0.4, 0.2, 0.1],
                    "max_correspondence_distance": [2.0, 1.0, 0.5],
                    "normals": f"hybrid r=0.3 max_nn=300, {normals}",
                    "parallelism": f"dp{world}"}
                   if ouster else
                   {"workload": f"hdl64_64k_{args.method}_loop_closure_pairs",
                    "baseline_config": "BASELINE.json configs[3] (C4: 4096 pairs over 8 GPUs)",
                    "pairs_per_gpu": P, "global_pairs": world * P,
                    "points_per_scan_post_filter": int(np.mean(n_pts)),
                    "rays_per_scan": 65536, "method": args.method,
                    "init": "GT (+) N(0.3 m, 3 deg yaw)",
                    "max_correspondence_distance": 10.0,
                    "normals": f"hybrid r=0.3 max_nn=300, {normals}",
                    "parallelism": f"dp{world}"}
                   if loop else
                   {"workload": f"hdl64_64k_{args.method}_seq",
                    "baseline_config": "BASELINE.json configs[2] (C3)",
                    "pairs_per_gpu": P, "global_pairs": world * P,
                    "streams_per_gpu": S,
                    "points_per_scan_post_filter": int(np.mean(n_pts)),
                    "rays_per_scan": 65536, "method": args.method,
                    "max_correspondence_distance": 10.0,
                    "normals": f"hybrid r=0.3 max_nn=300, {normals}",
                    "parallelism": f"dp{world}"}),
        "roofline": roof,
        "roofline_normals": roof_n,
        "cpu_baseline": cpu,
        # PCIe-inclusive rate (never `value`): the step after uploading its raw scans
        "pcie_inclusive": {"value": round(world * P / (ms_step * 1e-3 + up_s), 3),
                           "unit": "pairs/s", "upload_ms_per_step": round(up_s * 1e3, 3),
                           "host_to_device_GB_per_s": round(up_bytes / up_s / 1e9, 3),
                           "scans": len(seq.scans), "bytes": up_bytes,
                           "per_scan_uploads": {
                               "value": round(world * P / (ms_step * 1e-3 + up1_s), 3),
                               "upload_ms_per_step": round(up1_s * 1e3, 3)},
                           "source": "rank 0: every raw scan the step reads, from pageable "
                                     "host memory, as one lsm_cloud_upload_batch (value) and "
                                     "as one lsm_cloud_upload per scan (per_scan_uploads); "
                                     "the faster of two alternating runs each"},
        "mean_icp_iterations": float(np.mean(iters)),
        "breakdown_ms_per_step": {k: round(v["ms"] / args.steps, 3)
                                  for k, v in stats.items() if v["launches"]},
        "nn_uncertified_fraction_after_pass0": round(
            cnt["nn_uncertified"] /
            max(cnt["nn_queries"] - cnt["nn_queries_first_pass"], 1), 5),
        "nn_fallback_fraction": {
            "all_passes": round(cnt["nn_pending"] / max(cnt["nn_queries"], 1), 5),
            "first_pass": round(cnt["nn_pending_first_pass"] /
                                max(cnt["nn_queries_first_pass"], 1), 5)},
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from lidar_slam_arvc_amd import synthetic

    W = args.workload
    P0, seed0, _, normals0 = WORKLOAD_DEFAULTS[W]
    normals = normals0 if args.normals == "auto" else args.normals
    P = args.pairs_per_gpu or P0
    seed = args.seed if args.seed >= 0 else seed0
    # synthetic scans first, in forked worker processes: nothing in this process has touched the
    # GPU yet (a fork after HIP initialisation is not safe)
    procs = max(1, min(8, os.cpu_count() or 1))
    seq = make_data(W, P, seed, rank * P, procs, args.seq_cache)
    # the C4 / C5 blocks of the default line: each rank's own 512 pairs of BASELINE.json
    # configs[3] / [4], the same bench step as --workload loop_closure / ouster_multiscale
    extra = [] if args.no_c45 else [w for w in ("loop_closure", "ouster_multiscale") if w != W]
    extra_seq = {w: make_data(w, WORKLOAD_DEFAULTS[w][0], WORKLOAD_DEFAULTS[w][1],
                              rank * WORKLOAD_DEFAULTS[w][0], procs) for w in extra}
    c1 = c2 = None
    do_cpu = world == 1 and not args.no_cpu_baseline
    if do_cpu and not args.no_c1:
        # C1: 8k-point (16 x 512 ray) P2P pairs, seed 1 -- the reference's CPU-runnable case
        c1 = synthetic.make_sequence(C1_PAIRS + 1, seed=1, model=synthetic.VLP16_8K,
                                     processes=procs)
        # C2: one 64k HDL-64 pair, seed 2
        c2 = synthetic.make_sequence(2, seed=2, model=synthetic.HDL64, processes=procs)
    cpu_threads = args.cpu_threads or usable_cores()
    # the kernel hashes spawn llvm-objdump: before this process touches the GPU (every rank: the
    # normals' PMC lookup runs on all of them)
    for kernels in PMC_KERNELS.values():
        kernel_sha(tuple(kernels))
    _GPU_STARTED[0] = True

    import torch
    import torch.distributed as dist

    # --share-gpu (a rehearsal of the N-rank path on a one-GPU box): every rank on device 0,
    # collectives over gloo on host tensors; otherwise one GPU per rank and RCCL over xGMI
    gpu = 0 if args.share_gpu else local
    torch.cuda.set_device(gpu)
    group = None
    if world > 1:
        if args.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        group = dist.group.WORLD
    cuda = torch.device("cpu") if args.share_gpu else torch.device("cuda", local)   # collectives
    common = dict(gpu=gpu, local=local, rank=rank, world=world, group=group, cuda=cuda,
                  cpu_threads=cpu_threads)
    grid_cells = ([float(c) for c in args.grid_cell_scales.split(",")]
                  if args.grid_cell_scales else None)
    out = run_workload(W, seq, P, args, normals=normals, streams=args.streams,
                       grid_cell=args.grid_cell, grid_cells=grid_cells, do_cpu=do_cpu,
                       cpu_sample=args.cpu_sample_pairs, **common)
    del seq
    blocks = {}
    for w in extra:
        blocks[{"loop_closure": "c4", "ouster_multiscale": "c5"}[w]] = run_workload(
            w, extra_seq.pop(w), WORKLOAD_DEFAULTS[w][0], args, normals=WORKLOAD_DEFAULTS[w][3],
            do_cpu=do_cpu, **common)
    if rank == 0:
        from lidar_slam_arvc_amd import _lib
        dev = _lib.device(gpu)
        c1_out = c1_line(dev, c1, cpu_threads) if c1 is not None else None
        c2_out = c2_line(dev, c2, cpu_threads) if c2 is not None else None
        line = {k: v for k, v in out.items() if k not in ("mean_icp_iterations",
                                                         "breakdown_ms_per_step",
                                                         "nn_uncertified_fraction_after_pass0",
                                                         "nn_fallback_fraction")}
        line.update({"c1": c1_out, "c2": c2_out, **blocks,
                     "mean_icp_iterations": out["mean_icp_iterations"],
                     "library_sources_sha256": source_sha(),
                     "breakdown_ms_per_step": out["breakdown_ms_per_step"],
                     "nn_uncertified_fraction_after_pass0":
                         out["nn_uncertified_fraction_after_pass0"],
                     "nn_fallback_fraction": out["nn_fallback_fraction"]})
        print(json.dumps(line), flush=True)
    if group is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
