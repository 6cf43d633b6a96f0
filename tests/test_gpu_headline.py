"""GPU parity on the headline workload itself: pairs of bench.py's seed-3 HDL-64 sequence (C3,
BASELINE.json configs[2]; keyframe.py:246-252 via run_scanmatcher.py:196-213) against the two
f64 restatements of Open3D's path, from committed fixtures:

* tests/golden/seed3_pairs_o3d_oracle.npz -- the NumPy/SciPy oracle (oracle/open3d_restated.py)
  on 32 pairs: 8 on which the oracle hits max_iteration = 30 without converging and 24
  converging ones (tests/golden/make_seed3_oracle.py);
* tests/golden/seed3_seq_cpu_oracle.npz -- the C++/OpenMP oracle (oracle/cpu) on all 1999 pairs
  (tools/bench_parity.py --make-cpu); test_headline_full_sequence_vs_cpp_oracle runs the whole
  batch against it.

Bars (north_star): |dR| <= 1e-4 per element and |dt| <= 1e-3 m on converged pairs, against
both oracles: they agree on all 32 pairs (normals of rank-deficient neighbourhoods -- e.g. three
collinear points -- are decided by rounding, and both oracles now use Open3D's raw cumulants
divided by n for them), so no pair may lean on either one alone. Pairs that do not converge within
30 updates are held to equal quality: fitness within 1e-3 and rmse no worse than 5 % above the
oracle's (chaotic registrations).
"""
import hashlib
import os

import numpy as np
import pytest

from lidar_slam_arvc_amd import _lib, synthetic

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
R_TOL, T_TOL = 1e-4, 1e-3


def _sha(seq):
    h = hashlib.sha256()
    for s in seq.scans:
        h.update(np.ascontiguousarray(s, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(seq.priors, dtype=np.float64).tobytes())
    return h.hexdigest()


def _within(Ta, Tb):
    return (np.abs(Ta[:3, :3] - Tb[:3, :3]).max() <= R_TOL and
            np.abs(Ta[:3, 3] - Tb[:3, 3]).max() <= T_TOL)


@pytest.fixture(scope="module")
def headline(dev):
    py = np.load(os.path.join(HERE, "seed3_pairs_o3d_oracle.npz"))
    cpp = np.load(os.path.join(HERE, "seed3_seq_cpu_oracle.npz"))
    pairs = py["pairs"]
    scans, priors = [], []
    for k, sha in zip(pairs, py["sha256"]):
        seq = synthetic.make_sequence(2, seed=3, model=synthetic.HDL64, first_index=int(k))
        assert _sha(seq) == str(sha), f"pair {k}: not the fixture's clouds"
        scans += seq.scans
        priors.append(seq.priors[0])
    ids = [dev.upload(s) for s in scans]
    try:
        dev.preprocess(ids, _lib.prep_params())
        got = dev.icp_batch_arrays(ids[1::2], ids[0::2], np.stack(priors), _lib.icp_params())
    finally:
        for h in ids:
            dev.release(h)
    return pairs, got, py, cpp


def test_headline_pairs_vs_both_oracles(headline):
    pairs, got, py, cpp = headline
    rows = []
    for m, k in enumerate(pairs):
        Tg = got["transformation"][m]
        Tp, Tc = py["transformation"][m], cpp["transformation"][k]
        conv = got["iterations"][m] < 30 and py["iterations"][m] < 30
        oracles_agree = _within(Tp, Tc)
        ok_py, ok_c = _within(Tg, Tp), _within(Tg, Tc)
        rows.append((int(k), conv, oracles_agree, ok_py, ok_c))
        if conv:
            # the two oracles agree on every one of these pairs (since round 4's C++ oracle
            # divides its cumulants as Open3D does), so the GPU must be within the bar of both
            assert oracles_agree, f"pair {k}: the oracles disagree (fixture changed?)"
            assert ok_py and ok_c, f"pair {k}: GPU outside the bar (NumPy {ok_py}, C++ {ok_c})"
        else:
            assert abs(got["fitness"][m] - py["fitness"][m]) < 1e-3, f"pair {k}"
            assert got["inlier_rmse"][m] < 1.05 * py["inlier_rmse"][m], f"pair {k}"
    conv = [r for r in rows if r[1]]
    assert len(conv) >= 20
    # the fixture holds at least 4 pairs that hit max_iteration in the oracle
    assert int((py["iterations"] >= 30).sum()) >= 4
    print("headline pairs (pair, converged, oracles agree, GPU~py, GPU~C++):", rows)


# Every pair of the bench's own batch within the bar of the C++ oracle (tools/bench_parity.py,
# 1999 of 1999 since the small-neighbourhood normals follow Open3D's arithmetic).
# Pairs where the two oracles themselves disagree beyond the bar would be exempt: none is
# outside, so none is listed.
HEADLINE_WITHIN_MIN = 1999
ORACLES_DISAGREE = ()


def _full_sequence(tmp_path):
    """The 2000-keyframe seed-3 sequence, generated in a child process (forked ray-cast workers
    must not share this process's GPU context) and handed over as .npy files."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(HERE))
    code = ("import sys, numpy as np; sys.path.insert(0, %r); "
            "from lidar_slam_arvc_amd import synthetic; "
            "s = synthetic.make_sequence(2000, seed=3, model=synthetic.HDL64, processes=16); "
            "np.save(%r, np.concatenate(s.scans)); "
            "np.save(%r, np.array([len(x) for x in s.scans])); np.save(%r, s.priors)"
            % (root, str(tmp_path / "pts.npy"), str(tmp_path / "n.npy"),
               str(tmp_path / "priors.npy")))
    subprocess.run([sys.executable, "-c", code], check=True, timeout=600)
    pts = np.load(tmp_path / "pts.npy")
    n = np.load(tmp_path / "n.npy")
    priors = np.load(tmp_path / "priors.npy")
    scans = np.split(pts, np.cumsum(n)[:-1])
    return synthetic.Sequence(scans, None, priors)


def test_headline_full_sequence_vs_cpp_oracle(dev, tmp_path):
    """The whole headline workload (bench.py's C3 step: 2000 keyframes pre-processed, 1999 P2Plane
    pairs in one batch, run_scanmatcher.py:196-213 -> keyframe.py:246-252) against the C++
    oracle's results on the same clouds (tests/golden/seed3_seq_cpu_oracle.npz, checked by the
    sequence's SHA-256): at least HEADLINE_WITHIN_MIN pairs within 1e-4 / 1e-3 m, every
    converged pair outside the bar one where the two oracles disagree (ORACLES_DISAGREE), and
    every pair that hits max_iteration doing so on both sides."""
    cpp = np.load(os.path.join(HERE, "seed3_seq_cpu_oracle.npz"))
    seq = _full_sequence(tmp_path)
    assert _sha(seq) == str(cpp["sha256"]), "not the fixture's sequence"
    ids = [dev.upload(s) for s in seq.scans]
    try:
        dev.preprocess(ids, _lib.prep_params())
        got = dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, _lib.icp_params())
    finally:
        for h in ids:
            dev.release(h)
    Tg, Tc = got["transformation"], cpp["transformation"]
    within = [_within(Tg[k], Tc[k]) for k in range(len(Tc))]
    outside = [k for k, w in enumerate(within) if not w]
    print(f"headline: {sum(within)} of {len(Tc)} pairs within the bar; outside: {outside}")
    assert sum(within) >= HEADLINE_WITHIN_MIN, outside
    for k in outside:
        if got["iterations"][k] < 30 and cpp["iterations"][k] < 30:
            assert k in ORACLES_DISAGREE, f"pair {k}: outside the bar, oracles agree"
    hit_g = np.asarray(got["iterations"]) >= 30
    hit_c = np.asarray(cpp["iterations"]) >= 30
    assert int((hit_g != hit_c).sum()) <= 2, np.flatnonzero(hit_g != hit_c)


def test_headline_converged_iterations_close(headline):
    """Converged pairs take the same number of updates as the oracle, within 2 (the stop rule
    |d fitness| < 1e-6 and |d rmse| < 1e-6 is a threshold on the last digits)."""
    pairs, got, py, _ = headline
    for m, k in enumerate(pairs):
        if got["iterations"][m] < 30 and py["iterations"][m] < 30:
            assert abs(int(got["iterations"][m]) - int(py["iterations"][m])) <= 2, f"pair {k}"
            assert abs(got["fitness"][m] - py["fitness"][m]) < 1e-4


def test_headline_correspondence_near_ties(dev):
    """The f32 ranking of candidate distances may flip the nearest neighbour only between target
    points at (nearly) equal distance. Counted on 8 of the headline pairs, one correspondence pass
    (max_iteration = 0) at the odometry prior and one at the oracle's final transform: the GPU's
    set against the exact f64 nearest neighbours (cKDTree). Every differing query must be an f32
    near-tie: the two candidates' exact distances within 1e-5 m (the search ranks from the f32
    rounding of the transformed query, up to 3.3e-6 m from the f64 point at 35 m, which moves the
    difference of two distances by at most twice that), and the flips stay within
    the allowance of the single-pass test (2 per 20 000 queries). LSM_TIES_OUT=<file>: the counts
    as JSON."""
    import json

    from scipy.spatial import cKDTree

    from oracle import open3d_restated as O

    py = np.load(os.path.join(HERE, "seed3_pairs_o3d_oracle.npz"))
    rows = []
    for m in range(0, len(py["pairs"]), 4):
        k = int(py["pairs"][m])
        seq = synthetic.make_sequence(2, seed=3, model=synthetic.HDL64, first_index=k)
        assert _sha(seq) == str(py["sha256"][m])
        tgt = O.filter_radius_height(seq.scans[0])
        src = O.filter_radius_height(seq.scans[1])
        tree = cKDTree(tgt)
        ids = [dev.upload(s) for s in seq.scans]
        try:
            dev.preprocess(ids, _lib.prep_params(want_normals=False))
            for tag, T in (("prior", seq.priors[0]), ("final", py["transformation"][m])):
                dev.icp_batch([ids[1]], [ids[0]], T[None],
                              _lib.icp_params(method="p2p", max_iteration=0))
                got = dev.last_correspondences()
                ps = src @ T[:3, :3].T + T[:3, 3]
                d, nn = tree.query(ps, k=1)
                keep = d < 10.0
                ref = np.stack([np.flatnonzero(keep), nn[keep]], axis=1)
                g = dict(map(tuple, got.tolist()))
                r = dict(map(tuple, ref.tolist()))
                diff = [q for q in set(g) | set(r) if g.get(q) != r.get(q)]
                for q in diff:
                    assert q in g and q in r, f"pair {k} {tag}: query {q} matched on one side only"
                    dg = np.linalg.norm(ps[q] - tgt[g[q]])
                    dr = np.linalg.norm(ps[q] - tgt[r[q]])
                    assert abs(dg - dr) <= 1e-5, f"pair {k} {tag}: not a near-tie ({dg}, {dr})"
                assert len(diff) <= 2 * max(1, len(r) // 20000), f"pair {k} {tag}: {len(diff)}"
                rows.append({"pair": k, "at": tag, "queries": int(len(src)),
                             "correspondences": int(len(r)), "flips": int(len(diff))})
        finally:
            for h in ids:
                dev.release(h)
    out = os.environ.get("LSM_TIES_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"rows": rows, "flips": sum(x["flips"] for x in rows),
                       "correspondences": sum(x["correspondences"] for x in rows)}, f, indent=1)
