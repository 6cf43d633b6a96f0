"""GPU parity: the HIP path (through the C ABI) against the float64 oracle on the same inputs.

Bars (BASELINE.json north_star): bit-exact for the filter mask, voxel keys and loop-closure
indices; transforms within 1e-4 (R, per element) / 1e-3 m (t); normals compared up to sign.
"""
import numpy as np
import pytest

from lidar_slam_arvc_amd import _lib, synthetic
from oracle import open3d_restated as O

pytestmark = pytest.mark.gpu

R_TOL, T_TOL = 1e-4, 1e-3


@pytest.fixture(scope="module")
def seq8k():
    return synthetic.make_sequence(3, seed=21, model=synthetic.VLP16_8K)


@pytest.fixture(scope="module")
def seq64k():
    return synthetic.make_sequence(2, seed=2, model=synthetic.HDL64)


def _prep(dev, scans, **kw):
    ids = [dev.upload(s) for s in scans]
    dev.preprocess(ids, _lib.prep_params(**kw))
    return ids


def _release(dev, ids):
    for i in ids:
        dev.release(i)


# ------------------------------------------------------------------ boundary (8b)
def test_batch_upload_matches_single_uploads(dev, seq64k):
    """lsm_cloud_upload_batch (one allocation, one synchronisation for the batch) against one
    lsm_cloud_upload per cloud: the same raw counts and, pre-processed, the same points and
    normals bit for bit -- with an empty cloud, float64 input and an odd-sized cloud in the batch
    (each slice 256-byte aligned); an empty batch; the batch's handles released one by one (its
    allocation lives until the last) while the single uploads stay usable; an invalid count
    creates no handle."""
    import ctypes as C

    rng = np.random.default_rng(8)
    clouds = [seq64k.scans[0], np.zeros((0, 3), np.float32),
              np.asarray(seq64k.scans[1], np.float64),
              rng.uniform(-5.0, 5.0, (1001, 3)).astype(np.float32)]
    prm = _lib.prep_params()
    a = [dev.upload(c) for c in clouds]
    b = dev.upload_many(clouds)
    try:
        assert dev.upload_many([]) == []
        assert [dev.info(i)[0] for i in b] == [len(c) for c in clouds]
        dev.preprocess(a, prm)
        dev.preprocess(b, prm)
        for x, y in zip(a, b):
            px, nx = dev.download(x, normals=True)
            py, ny = dev.download(y, normals=True)
            assert np.array_equal(px, py) and np.array_equal(nx, ny)
        for y in b[:2]:
            dev.release(y)
        dev.preprocess(b[2:], prm)
        assert np.array_equal(dev.download(b[3])[0], dev.download(a[3])[0])
        b = b[2:]
        ns = np.array([-1], dtype=np.int64)
        out = np.array([-7], dtype=np.int64)
        ptrs = (C.POINTER(C.c_float) * 1)(clouds[0].ctypes.data_as(C.POINTER(C.c_float)))
        rc = dev.lib.lsm_cloud_upload_batch(dev.handle, ptrs, ns.ctypes.data_as(
            C.POINTER(C.c_int64)), 1, out.ctypes.data_as(C.POINTER(C.c_int64)))
        assert rc != 0 and out[0] == -7
    finally:
        _release(dev, a + b)


# ------------------------------------------------------------------ filter (a2)
def test_filter_bit_exact(dev, seq64k):
    ids = _prep(dev, seq64k.scans, want_normals=False)
    try:
        for cid, scan in zip(ids, seq64k.scans):
            got = dev.download(cid)
            ref = O.filter_radius_height(scan)
            assert got.shape == ref.shape
            assert np.array_equal(got, ref)
    finally:
        _release(dev, ids)


def test_filter_edges(dev):
    pts = np.array([[0.5, 0.0, 0.0], [0.5000001, 0, 0], [35.0, 0, 0], [34.999998, 0, 0],
                    [1, 1, -1.0], [1, 1, -0.9999999], [1, 1, 50.0], [1, 1, 49.999996],
                    [np.nan, 1, 1], [1, np.inf, 1], [3, 4, 0], [0, 0, 0]], dtype=np.float32)
    empty = np.zeros((0, 3), np.float32)
    gone = np.array([[0.1, 0.1, 0.1]], np.float32)
    ids = _prep(dev, [pts, empty, gone], want_normals=False)
    try:
        assert np.array_equal(dev.download(ids[0]), O.filter_radius_height(pts))
        assert dev.info(ids[1])[1] == 0
        assert dev.info(ids[2])[1] == 0
    finally:
        _release(dev, ids)


# ------------------------------------------------------------------ voxel (a3)
@pytest.mark.parametrize("v", [0.01, 0.1, 0.25, 0.4])   # 0.01: a 64-bit key space
def test_voxel_bit_exact(dev, seq8k, v):
    ids = _prep(dev, seq8k.scans[:2], want_normals=False, voxel_size=v)
    try:
        for cid, scan in zip(ids, seq8k.scans[:2]):
            keys_ref, cent_ref = O.voxel_down_sample(O.filter_radius_height(scan), v)
            keys = dev.voxel_keys(cid)
            cent = dev.download(cid)
            assert np.array_equal(keys.astype(np.int64), keys_ref)
            assert np.array_equal(cent, cent_ref)
    finally:
        _release(dev, ids)


# ------------------------------------------------------------------ normals (a4)
def _normal_agreement(n_gpu, n_ref):
    d = np.abs(np.sum(n_gpu * n_ref, axis=1))
    return d


@pytest.mark.parametrize("which", ["8k", "64k"])
def test_normals(dev, seq8k, seq64k, which):
    """Normals against both f64 oracles (keyframe.py:160-162). Every point whose covariance has
    a separated spectrum (the two smallest eigenvalues apart by more than 1e-4 of the largest;
    n >= 4 always is on these scans) agrees with the NumPy oracle to |n . n_ref| > 1 - 1e-6
    (f32 storage of a unit normal: ~1e-7), truncated neighbourhoods included. The small
    neighbourhoods (3 <= n <= NSMALL = 8, rank-deficient when their points are near-collinear)
    take Open3D's own covariance arithmetic (small_normal) -- the C++ oracle's: their f32
    normals equal its normals rounded to f32 bit for bit on >= 99.5 % of the points (the rest:
    the device's and the host's acos / cos differ in the last bit), all within 1e-6, and the
    three-point ones that differ are counted apart."""
    from oracle import cpu_ref as C
    scan = (seq8k if which == "8k" else seq64k).scans[0]
    ids = _prep(dev, [scan])
    try:
        xyz, nrm = dev.download(ids[0], normals=True)
        ref_pts = O.filter_radius_height(scan)
        assert np.array_equal(xyz, ref_pts)
        ref_n, counts, covs = O.estimate_normals(ref_pts, return_counts=True, return_covs=True)
        ev = np.linalg.eigvalsh(covs)
        sep = (ev[:, 1] - ev[:, 0]) > 1e-4 * np.maximum(np.abs(ev[:, 2]), 1e-300)
        d = _normal_agreement(nrm, ref_n)
        assert sep[counts >= 4].mean() > 0.999
        assert (d[sep] > 1.0 - 1e-6).all(), np.sort(d[sep])[:10]
        trunc = counts >= 300   # points whose neighbourhood was truncated to max_nn
        assert (d[trunc & sep] > 1.0 - 1e-6).all()
        c_n, c_cnt = C.estimate_normals(ref_pts, return_counts=True)
        assert np.array_equal(c_cnt, counts)
        small = (counts >= 3) & (counts <= 8)
        g, f = nrm.astype(np.float32), c_n.astype(np.float32)
        bit = np.all(g == f, axis=1) | np.all(g == -f, axis=1)
        assert bit[small].mean() >= 0.995, bit[small].mean()
        assert (_normal_agreement(nrm, c_n)[small] > 1.0 - 1e-6).all()
        three = counts == 3
        assert (~bit[three]).sum() <= max(2, 0.005 * three.sum()), (~bit[three]).sum()
    finally:
        _release(dev, ids)


@pytest.mark.parametrize("max_nn", [300, 100, 30])
def test_normals_preclassification_bit_identical(dev, seq64k, max_nn, monkeypatch):
    """The kNN truncation's final pass settles most points with the f32 distance against the
    selection state's thresholds (2e-6 relative margin) and leaves only a band to the exact f64
    classification. That may never change a neighbourhood: normals must be bit-identical to
    LSM_NORMALS_EXACT=1 (every point through the f64 test), also under heavier truncation."""
    ids = [dev.upload(s) for s in seq64k.scans]
    try:
        prm = _lib.prep_params(max_nn=max_nn)
        dev.preprocess(ids, prm)
        fast = [dev.download(i, normals=True)[1] for i in ids]
        monkeypatch.setenv("LSM_NORMALS_EXACT", "1")
        dev.preprocess(ids, prm)
        monkeypatch.delenv("LSM_NORMALS_EXACT")
        exact = [dev.download(i, normals=True)[1] for i in ids]
        for a, b in zip(fast, exact):
            assert np.array_equal(a, b)
    finally:
        _release(dev, ids)


@pytest.mark.parametrize("max_nn", [300, 30])
def test_normals_split_launch_bit_identical(dev, seq64k, max_nn, monkeypatch):
    """The split launch (default: the points predicted sparse, then every deferred point in
    full waves of the clouds' dense lists, then the rare refine scans) against the one-kernel
    launch (LSM_NORMALS_SPLIT=0) and against the split launch with its refine kernel on the main
    stream instead of the side stream (LSM_NORMALS_SIDE=0):
    bit-identical normals on bench scans, under heavier truncation, on degenerate neighbourhoods
    (duplicates saturating a u8 bin, a dense patch) and on clouds that carry prior normals
    (EstimateNormals re-run on a cloud with normals orients to them)."""
    rng = np.random.default_rng(11)
    patch = np.c_[5.0 + rng.uniform(-0.2, 0.2, 1500), rng.uniform(-0.2, 0.2, 1500),
                  0.002 * rng.standard_normal(1500)]
    dup = np.repeat([[5.05, 0.03, 0.0]], 400, axis=0)
    clouds = list(seq64k.scans[:3]) + [np.r_[patch, dup].astype(np.float32)]
    prm = _lib.prep_params(max_nn=max_nn)
    keep = _lib.prep_params(max_nn=max_nn, min_radius=-np.inf, max_radius=1e15,
                            min_height=-1e15, max_height=1e15)
    out = {}
    for split in ("1", "0", "side0"):
        # "side0": the split launch with its refine kernel on the main stream (LSM_NORMALS_SIDE=0)
        monkeypatch.setenv("LSM_NORMALS_SPLIT", "1" if split == "side0" else split)
        monkeypatch.setenv("LSM_NORMALS_SIDE", "0" if split == "side0" else "1")
        ids = [dev.upload(c) for c in clouds]
        try:
            dev.preprocess(ids, prm)
            first = [dev.download(i, normals=True)[1] for i in ids]
            dev.preprocess(ids, keep)          # again, now with prior normals
            second = [dev.download(i, normals=True)[1] for i in ids]
            out[split] = first + second
        finally:
            _release(dev, ids)
    monkeypatch.delenv("LSM_NORMALS_SPLIT")
    monkeypatch.delenv("LSM_NORMALS_SIDE")
    for a, b, c in zip(out["1"], out["0"], out["side0"]):
        assert np.array_equal(a, b) and np.array_equal(a, c)


@pytest.mark.parametrize("voxel", [0.0, 0.1])
def test_grid_layout_invariants(dev, seq64k, voxel):
    """The device layout (lsm_cloud_layout) of clouds pre-processed as one batch -- bench scans,
    an empty cloud, exact duplicates and signed zeros: perm is a permutation, the cell table
    rises from 0 to n, and inside every cell the points are sorted by x with x ties in reference
    order (the stable (cell, x) radix order the searches and their tie-breaking rely on), every
    cell spatially compact."""
    rng = np.random.default_rng(5)
    dup = np.repeat([[3.0, 1.0, 0.2], [-0.0, 2.0, 0.1], [0.0, 2.0, 0.1]], 7, axis=0)
    ties = np.r_[dup, np.c_[rng.uniform(-4, 4, 3000), rng.uniform(-4, 4, 3000),
                            rng.uniform(-0.5, 0.5, 3000)]].astype(np.float32)
    clouds = list(seq64k.scans[:3]) + [np.zeros((0, 3), np.float32), ties]
    keep = dict(min_radius=-np.inf, max_radius=1e15, min_height=-1e15, max_height=1e15)
    ids = [dev.upload(c) for c in clouds]
    try:
        dev.preprocess(ids, _lib.prep_params(voxel_size=voxel or None, **keep))
        for h in ids:
            perm, cells = dev.layout(h)
            pts = dev.download(h).astype(np.float32)
            n = len(pts)
            assert np.array_equal(np.sort(perm), np.arange(n))
            assert cells[0] == 0 and cells[-1] == n and np.all(np.diff(cells.astype(np.int64)) >= 0)
            sp = pts[perm]
            occ = np.flatnonzero(np.diff(cells.astype(np.int64)) > 0)
            for c in occ:
                a, b = int(cells[c]), int(cells[c + 1])
                x = sp[a:b, 0]
                dx = np.diff(x)
                assert np.all(dx >= 0)
                assert np.all(np.diff(perm[a:b])[dx == 0] > 0)   # x ties in reference order
                ext = sp[a:b].max(0) - sp[a:b].min(0)
                # cells: c in x and z, c / 2 in y (c: 0.42 m, voxelised max(0.75, 2.5 voxel))
                c = max(0.75, 2.5 * voxel) if voxel else 0.42
                assert np.all(ext <= np.array([c, c / 2, c]) * (1 + 1e-5)), ext
    finally:
        _release(dev, ids)


def test_normals_degenerate_neighbourhoods(dev):
    """kNN-300 truncation on pathological neighbourhoods: 400 exact duplicates of one point (one
    d2 value holds more than a u8 histogram bin can count and more than the selection buffer
    can rank, so the u32 restart and the tie cap both run), a dense planar patch, and points
    whose neighbours sit at exactly equal distances (a regular grid). Ties at one distance are
    ties between identical contributions (duplicates) or symmetric ones, so the normal is
    determined; it must match the oracle."""
    rng = np.random.default_rng(7)
    patch = np.c_[5.0 + rng.uniform(-0.2, 0.2, 1500), rng.uniform(-0.2, 0.2, 1500),
                  0.002 * rng.standard_normal(1500)]
    dup = np.repeat([[5.05, 0.03, 0.0]], 400, axis=0)
    g = np.arange(-10, 11) * 0.02
    gx, gy = np.meshgrid(g, g)
    grid = np.c_[8.0 + gx.ravel(), 1.0 + gy.ravel(), 0.5 + 0.0 * gx.ravel()]
    wall = np.c_[np.full(900, 12.0) + 0.001 * rng.standard_normal(900),
                 rng.uniform(-0.3, 0.3, 900), rng.uniform(0.0, 0.6, 900)]
    cloud = np.vstack([patch, dup, grid, wall]).astype(np.float32)
    ids = _prep(dev, [cloud])
    try:
        xyz, nrm = dev.download(ids[0], normals=True)
        ref_pts = O.filter_radius_height(cloud)
        assert np.array_equal(xyz, ref_pts)
        ref_n, counts = O.estimate_normals(ref_pts, return_counts=True)
        assert (counts >= 300).sum() > 1000
        # a patch point next to the duplicates can keep itself + 299 copies: a rank-1
        # covariance whose normal is any vector of a plane (not determined) -- skip those
        from scipy.spatial import cKDTree
        p64 = ref_pts.astype(np.float64)
        idx, _, cnt = O.hybrid_search(cKDTree(p64), p64, p64, 0.3, 300)
        ev = np.linalg.eigvalsh(O.compute_covariance(p64, idx, cnt))
        determined = (ev[:, 1] - ev[:, 0]) > 1e-6 * np.maximum(ev[:, 2], 1e-30)
        assert determined.mean() > 0.99
        d = _normal_agreement(nrm, ref_n)
        assert (d[determined] > 1.0 - 1e-5).all(), np.sort(d[determined])[:10]
    finally:
        _release(dev, ids)


# ------------------------------------------------------------------ ICP (a6)
def _oracle_pair(seq, i, method, max_iteration=30):
    tgt = O.filter_radius_height(seq.scans[i])
    src = O.filter_radius_height(seq.scans[i + 1])
    nrm = O.estimate_normals(tgt) if method == "p2plane" else None
    return O.registration_icp(src, tgt, 10.0, seq.priors[i], method, nrm,
                              max_iteration=max_iteration)


@pytest.mark.parametrize("method", ["p2plane", "p2p"])
@pytest.mark.parametrize("which", ["8k", "64k"])
def test_icp_parity(dev, seq8k, seq64k, method, which):
    seq = seq8k if which == "8k" else seq64k
    ids = _prep(dev, seq.scans[:2], want_normals=(method == "p2plane"))
    try:
        got = dev.icp_batch([ids[1]], [ids[0]], seq.priors[:1], _lib.icp_params(method=method))[0]
        ref = _oracle_pair(seq, 0, method)
        T, R = got["transformation"], ref["transformation"]
        assert np.abs(T[:3, :3] - R[:3, :3]).max() < R_TOL
        assert np.abs(T[:3, 3] - R[:3, 3]).max() < T_TOL
        assert abs(got["fitness"] - ref["fitness"]) < 1e-3
        assert abs(got["inlier_rmse"] - ref["inlier_rmse"]) < 1e-3
        assert abs(got["iterations"] - ref["iterations"]) <= 2
    finally:
        _release(dev, ids)


def test_correspondences_single_pass(dev, seq64k):
    """max_iteration = 0: one correspondence pass at the initial guess; compare the set."""
    ids = _prep(dev, seq64k.scans[:2])
    try:
        got = dev.icp_batch([ids[1]], [ids[0]], seq64k.priors[:1],
                            _lib.icp_params(max_iteration=0))[0]
        corr = dev.last_correspondences()
        ref = _oracle_pair(seq64k, 0, "p2plane", max_iteration=0)
        rc = ref["correspondences"]
        assert got["n_corr"] == len(rc)
        assert abs(got["fitness"] - ref["fitness"]) < 1e-12
        assert abs(got["inlier_rmse"] - ref["inlier_rmse"]) < 1e-6
        a = {tuple(x) for x in corr.tolist()}
        b = {tuple(x) for x in rc.tolist()}
        # f32 distances may flip exact near-ties only
        assert len(a ^ b) <= 2 * max(1, len(b) // 20000)
    finally:
        _release(dev, ids)


@pytest.mark.parametrize("method", ["p2plane", "p2p"])
def test_icp_known_transform(dev, seq8k, method):
    tgt = O.filter_radius_height(seq8k.scans[0]).astype(np.float32)
    D = synthetic.pose_from(0.2, -0.1, 0.03, 0.01, -0.015, 0.04)
    src = O.transform_points(np.linalg.inv(D), tgt.astype(np.float64)).astype(np.float32)
    ids = _prep(dev, [tgt, src], want_normals=(method == "p2plane"))
    try:
        got = dev.icp_batch([ids[1]], [ids[0]], None,
                            _lib.icp_params(method=method, max_correspondence_distance=1.0,
                                            max_iteration=60))[0]
        assert np.abs(got["transformation"] - D).max() < 1e-5
        assert got["fitness"] > 0.999
    finally:
        _release(dev, ids)


def test_batch_equals_single_and_deterministic(dev, seq8k):
    ids = _prep(dev, seq8k.scans)
    try:
        prm = _lib.icp_params()
        batch = dev.icp_batch([ids[1], ids[2]], [ids[0], ids[1]], seq8k.priors, prm)
        again = dev.icp_batch([ids[1], ids[2]], [ids[0], ids[1]], seq8k.priors, prm)
        single = [dev.icp_batch([ids[k + 1]], [ids[k]], seq8k.priors[k:k + 1], prm)[0]
                  for k in range(2)]
        for a, b, c in zip(batch, again, single):
            assert np.array_equal(a["transformation"], b["transformation"])
            assert np.array_equal(a["transformation"], c["transformation"])
            assert a["iterations"] == c["iterations"] and a["fitness"] == c["fitness"]
    finally:
        _release(dev, ids)


def test_errors(dev, seq8k):
    ids = _prep(dev, seq8k.scans[:2], want_normals=False)
    try:
        with pytest.raises(RuntimeError, match="normal"):
            dev.icp_batch([ids[1]], [ids[0]], None, _lib.icp_params(method="p2plane"))
        with pytest.raises(RuntimeError, match="max_correspondence_distance"):
            dev.icp_batch([ids[1]], [ids[0]], None,
                          _lib.icp_params(method="p2p", max_correspondence_distance=0.0))
    finally:
        _release(dev, ids)


def test_empty_source(dev, seq8k):
    ids = _prep(dev, [seq8k.scans[0], np.zeros((0, 3), np.float32)])
    try:
        got = dev.icp_batch([ids[1]], [ids[0]], seq8k.priors[:1], _lib.icp_params())[0]
        assert got["fitness"] == 0.0 and got["inlier_rmse"] == 0.0
        assert np.array_equal(got["transformation"], seq8k.priors[0])
    finally:
        _release(dev, ids)


# ------------------------------------------------------------------ loop closure (a10/a11)
def test_loop_candidates_bit_exact(dev):
    rng = np.random.default_rng(5)
    t = np.linspace(0, 4 * np.pi, 900)
    P = np.stack([20 * np.cos(t), 20 * np.sin(t), 0.1 * rng.normal(size=len(t))], 1)
    P[:, :2] += rng.normal(scale=0.3, size=(len(t), 2))
    for m in [10, 300, 600, 900]:
        idx, cand = dev.loop_candidates(P[:m], 9.0, 2.0)
        ref_c, ref_i = O.find_candidates(P[:m], 9.0, 2.0)
        assert idx == ref_i
        assert np.array_equal(cand, ref_c)
        if len(cand):
            part = dev.loop_partners(P[:m], cand)
            trip = O.find_feasible_triplets(P[:m], m - 1, cand)
            got = [[m - 1, int(j1), int(j2)] for j1, j2 in zip(cand, part) if j2 >= 0]
            assert got == trip


# ------------------------------------------------------------------ stability certificate (a6.1)
@pytest.mark.parametrize("method,max_corr", [("p2plane", 10.0), ("p2p", 10.0), ("p2plane", 0.5)])
def test_certified_passes_bit_identical(dev, method, max_corr, monkeypatch):
    """Passes >= 1 skip the search for queries whose neighbour is certified unchanged
    (nn_check_kernel). The certificate only claims what a full search would return, so every
    result must be bit-identical to LSM_NN_NOCERT=1 (every query searched in every pass) --
    including the none-within-max_corr queries a small max_corr produces."""
    seq = synthetic.make_sequence(4, seed=7, model=synthetic.HDL64)
    ids = _prep(dev, seq.scans, want_normals=(method == "p2plane"))
    try:
        prm = _lib.icp_params(method=method, max_correspondence_distance=max_corr)
        src, tgt = ids[1:], ids[:-1]
        dev.reset_stats()
        dev.set_timing(True)
        cert = dev.icp_batch(src, tgt, seq.priors, prm)
        c_cert = dev.last_correspondences()
        dev.set_timing(False)
        queried = dev.kernel_stats("nn_queries")["launches"]
        searched = dev.kernel_stats("nn_uncertified")["launches"]
        monkeypatch.setenv("LSM_NN_NOCERT", "1")
        full = dev.icp_batch(src, tgt, seq.priors, prm)
        c_full = dev.last_correspondences()
        monkeypatch.delenv("LSM_NN_NOCERT")
        for a, b in zip(cert, full):
            assert np.array_equal(a["transformation"], b["transformation"])
            assert a["fitness"] == b["fitness"] and a["inlier_rmse"] == b["inlier_rmse"]
            assert a["iterations"] == b["iterations"] and a["n_corr"] == b["n_corr"]
        assert np.array_equal(c_cert, c_full)
        first = sum(dev.info(i)[1] for i in src)
        # the certificate must actually carry the later passes (P2P creeps: weaker)
        assert searched < (0.5 if method == "p2plane" else 0.9) * (queried - first)
    finally:
        _release(dev, ids)


@pytest.mark.parametrize("env", [{}, {"LSM_NN_SPLIT_PLACE": "1"}, {"LSM_NN_SPLIT_PLACE": "2"},
                                 {"LSM_NN_SPLIT": "32"}, {"LSM_NN_SPLIT": "1"},
                                 {"LSM_NN_TILE": "1"}])
def test_certified_split_searches_bit_identical_on_bench_sequence(dev, env, monkeypatch):
    """The bench's own data (seed-3 HDL-64 sequence), 24 pairs: enough pairs that the later
    passes leave workgroups with few uncertified queries, whose box searches are split over
    2-8 lanes (nn_kernel, group_top3), and enough non-converging pairs to run the 30-update
    tail. Every result and the final correspondences must equal LSM_NN_NOCERT=1 (one lane per
    query, every query searched every pass) bit for bit -- with the split groups from lane 0
    (default), ending in the last wave, in reversed query order, up to 32 lanes per query, or
    no split at all: where a query's group sits in the workgroup must not change its answer
    (round 2's open "waves 2-3" finding)."""
    seq = synthetic.make_sequence(25, seed=3, model=synthetic.HDL64)
    ids = _prep(dev, seq.scans, want_normals=True)
    try:
        prm = _lib.icp_params(method="p2plane")
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        cert = dev.icp_batch(ids[1:], ids[:-1], seq.priors, prm)
        c_cert = dev.last_correspondences()
        for k in env:
            monkeypatch.delenv(k)
        monkeypatch.setenv("LSM_NN_NOCERT", "1")
        full = dev.icp_batch(ids[1:], ids[:-1], seq.priors, prm)
        c_full = dev.last_correspondences()
        monkeypatch.delenv("LSM_NN_NOCERT")
        for a, b in zip(cert, full):
            assert np.array_equal(a["transformation"], b["transformation"])
            assert a["fitness"] == b["fitness"] and a["inlier_rmse"] == b["inlier_rmse"]
            assert a["iterations"] == b["iterations"]
        assert np.array_equal(c_cert, c_full)
    finally:
        _release(dev, ids)


@pytest.mark.parametrize("env", [{"LSM_NN_CERT_FROM": "1"},
                                 {"LSM_NN_CERT_FROM": "4"}, {"LSM_NN_DIRECT": "0"},
                                 {"LSM_NN_DIRECT": "1", "LSM_NN_DIRECT_ITER": "0"},
                                 {"LSM_NN_DIRECT": "2.5", "LSM_NN_DIRECT_ITER": "1"},
                                 {"LSM_NN_KCOLD": "1"}, {"LSM_NN_KCOLD": "2"},
                                 {"LSM_NN_KMAX": "2"}, {"LSM_NN_KCOLD": "6", "LSM_NN_KMAX": "3"},
                                 {"LSM_NN_SPLIT_PLACE": "1"}, {"LSM_NN_SPLIT_PLACE": "2"},
                                 {"LSM_NN_NOCERT": "1"}, {"LSM_NN_COLD_SEED": "0"},
                                 {"LSM_NN_TILE": "1"}, {"LSM_NN_TILE": "1", "LSM_NN_NOCERT": "1"},
                                 {"LSM_NN_FULL_L": "2"}, {"LSM_NN_FULL_L": "4"},
                                 {"LSM_NN_FULL_L": "2", "LSM_NN_NOCERT": "1"},
                                 {"LSM_FB_GL": "16"}, {"LSM_FB_GL": "16", "LSM_NN_DIRECT": "1",
                                                       "LSM_NN_DIRECT_ITER": "0"},
                                 {"LSM_FB_WAVES": "3"}, {"LSM_FB_WIDE_FROM": "0"},
                                 {"LSM_FB_WIDE_FROM": "2"}, {"LSM_FB_FAR": "1.5"},
                                 {"LSM_FB_FAR": "0.5", "LSM_FB_GL": "16"}, {"LSM_FB_GL": "32"},
                                 {"LSM_FB_WIDE_MAX": "0"}, {"LSM_FB_WIDE_MAX": "4000000000"},
                                 {"LSM_FB_WIDE_MAXC": "100"}])
def test_search_path_variants_bit_identical(dev, env, monkeypatch):
    """The exact 1-NN may be reached along different paths: the stability check from pass 1, 2
    or 4, queries with a
    far warm start sent straight to the fallback (from 1 cell in every pass, from 2.5 cells
    after the first update, the default 3 cells after 12 updates, or never), cold-start boxes
    of 3^3 / 5^3 / 9^3 (default) / 13^3 cells, warm boxes capped at 2 / 3 / 4 (default) cells,
    split groups placed anywhere in the workgroup, cold searches seeded with a point of the
    query's own cell (default) or not, the full passes' searches from global memory (default) or
    from LDS-staged target tiles (LSM_NN_TILE=1: nn_tile_kernel + nn_box_kernel), the fallback
    with 16, 32 or 64 lanes per query (chosen per pass from the queue length -- the default --, 64
    from any pass on, or for the queries whose box-search best lies beyond a distance) and any
    grid size. Every choice
    must give the same correspondences, so every result is bit-identical to the default's
    (C4-style revisit pairs: large initial errors, many fallback queries)."""
    ps = synthetic.make_revisit_pairs(6, seed=41, model=synthetic.HDL64)
    ids = _prep(dev, ps.targets + ps.sources, want_normals=True)
    try:
        prm = _lib.icp_params(method="p2plane")
        ref = dev.icp_batch(ids[6:], ids[:6], ps.init, prm)
        c_ref = dev.last_correspondences()
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        got = dev.icp_batch(ids[6:], ids[:6], ps.init, prm)
        c_got = dev.last_correspondences()
        for k in env:
            monkeypatch.delenv(k)
        for a, b in zip(ref, got):
            assert np.array_equal(a["transformation"], b["transformation"])
            assert a["fitness"] == b["fitness"] and a["inlier_rmse"] == b["inlier_rmse"]
            assert a["iterations"] == b["iterations"]
        assert np.array_equal(c_ref, c_got)
    finally:
        _release(dev, ids)


# ------------------------------------------------------------------ multi-scale chain (C5)
@pytest.mark.parametrize("method", ["p2plane", "p2p"])
def test_multiscale_ouster_pair(dev, method):
    """C5: a 256k-ray Ouster-128 pair through voxel scales 0.4 / 0.2 / 0.1 m (max_corr 2 / 1 /
    0.5 m), every stage checked against the oracle's own chain."""
    from lidar_slam_arvc_amd.multiscale import register_multiscale
    seq = synthetic.make_sequence(2, seed=5, model=synthetic.OUSTER128)
    ids = [dev.upload(s) for s in seq.scans]
    try:
        final, stages = register_multiscale(dev, [ids[1]], [ids[0]], seq.priors[:1],
                                            method=method, return_stages=True)
        ref = O.registration_multiscale(seq.scans[1], seq.scans[0], seq.priors[0],
                                        method=method)
        assert len(stages) == len(ref) == 3
        for got, r in zip(stages, ref):
            T, R = got[0]["transformation"], r["transformation"]
            assert np.abs(T[:3, :3] - R[:3, :3]).max() < R_TOL
            assert np.abs(T[:3, 3] - R[:3, 3]).max() < T_TOL
            assert abs(got[0]["fitness"] - r["fitness"]) < 1e-3
        # the chain lands on the ground-truth relative pose (synthetic scans)
        gt = np.linalg.inv(seq.poses[0]) @ seq.poses[1]
        assert np.abs(final[0]["transformation"][:3, 3] - gt[:3, 3]).max() < 0.05
    finally:
        _release(dev, ids)


def test_clone_is_independent(dev, seq8k):
    a = dev.upload(seq8k.scans[0])
    b = dev.clone(a)
    try:
        dev.preprocess([a], _lib.prep_params(want_normals=False))
        dev.preprocess([b], _lib.prep_params(want_normals=False, voxel_size=0.25))
        assert np.array_equal(dev.download(a), O.filter_radius_height(seq8k.scans[0]))
        ref = O.voxel_down_sample(O.filter_radius_height(seq8k.scans[0]), 0.25)[1]
        assert np.array_equal(dev.download(b), ref)
    finally:
        _release(dev, [a, b])


# ------------------------------------------------------------------ sharding (§8e)
def _arrays_equal(a, b):
    for k in ("transformation", "fitness", "inlier_rmse", "iterations", "n_corr"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sequence_bit_identical(dev, world):
    """C3 sharding as bench.py runs it at N GPUs, rank after rank on one GPU: rank r generates
    only keyframes a .. b of the seed-3 sequence (its pairs [a, b) plus the one-keyframe halo,
    synthetic.make_sequence(first_index=a)), pre-processes them in its own context and
    registers its pairs. Every relative transform, fitness, rmse, iteration count and
    correspondence count must equal the unsharded batch bit for bit (run_scanmatcher.py:196-213:
    the pairs are independent given the priors)."""
    from lidar_slam_arvc_amd import distributed
    n = 12
    seq = synthetic.make_sequence(n + 1, seed=3, model=synthetic.HDL64)
    prep, icp = _lib.prep_params(), _lib.icp_params()
    ids = _prep(dev, seq.scans)
    try:
        ref = dev.icp_batch_arrays(ids[1:], ids[:-1], seq.priors, icp)
    finally:
        _release(dev, ids)
    for r in range(world):
        a, b = distributed.shard_pairs(n, world, r)
        part = synthetic.make_sequence(b - a + 1, seed=3, model=synthetic.HDL64, first_index=a)
        d = _lib.Device(0)                      # the rank's own context
        try:
            hs = [d.upload(s) for s in part.scans]
            d.preprocess(hs, prep)
            got = d.icp_batch_arrays(hs[1:], hs[:-1], part.priors, icp)
            _arrays_equal(got, {k: np.asarray(v)[a:b] for k, v in ref.items()})
        finally:
            d.close()


def test_balanced_loop_pairs_bit_identical(dev):
    """C4 sharding: independent revisit pairs packed over 3 ranks by balance_pairs (cost = N_src
    x iterations of a first batch), each rank's subset registered in its own context, then the
    results put back in global order (gather_pair_results without a group): equal to the
    unsharded batch bit for bit."""
    from lidar_slam_arvc_amd import distributed
    P = 7
    ps = synthetic.make_revisit_pairs(P, seed=4, model=synthetic.HDL64)
    prep, icp = _lib.prep_params(), _lib.icp_params()
    ids = _prep(dev, ps.targets + ps.sources)
    try:
        ref = dev.icp_batch_arrays(ids[P:], ids[:P], ps.init, icp)
        nsrc = np.array([dev.info(h)[1] for h in ids[P:]])
    finally:
        _release(dev, ids)
    cost = nsrc * ref["iterations"]
    parts = distributed.balance_pairs(cost, 3)
    rows = np.zeros((P, 4, 4))
    for mine in parts:
        d = _lib.Device(0)
        try:
            hs = [d.upload(ps.targets[k]) for k in mine] + [d.upload(ps.sources[k]) for k in mine]
            d.preprocess(hs, prep)
            m = len(mine)
            got = d.icp_batch_arrays(hs[m:], hs[:m], ps.init[mine], icp)
            _arrays_equal(got, {k: np.asarray(v)[mine] for k, v in ref.items()})
            rows += distributed.gather_pair_results(got["transformation"], mine, P)
        finally:
            d.close()
    assert np.array_equal(rows, ref["transformation"])


# ------------------------------------------------------------------ lazy normals
def _assert_batch_equal(a, b):
    for k in ("transformation", "fitness", "inlier_rmse", "iterations", "n_corr"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_lazy_normals_bit_identical_on_bench_sequence(dev):
    """LSM_NORMALS_LAZY (bench.py's C4 / C5 mode): a keyframe's normals are computed when it is
    first a P2Plane target. The registrations, their correspondence sets and -- once completed
    by the download -- every normal equal the eager pre-process bit for bit (seed-3 sequence, 24
    pairs including non-converging ones); a second batch on the same clouds reuses the computed
    normals and still agrees."""
    seq = synthetic.make_sequence(25, seed=3, model=synthetic.HDL64)
    icp = _lib.icp_params()
    eager = _prep(dev, seq.scans)
    lazy = _prep(dev, seq.scans, want_normals="lazy")
    try:
        ref = dev.icp_batch_arrays(eager[1:], eager[:-1], seq.priors, icp)
        c_ref = dev.last_correspondences()
        dev.reset_stats()
        dev.set_timing(True)
        got = dev.icp_batch_arrays(lazy[1:], lazy[:-1], seq.priors, icp)
        dev.set_timing(False)
        c_got = dev.last_correspondences()
        _assert_batch_equal(ref, got)
        assert np.array_equal(c_ref, c_got)
        again = dev.icp_batch_arrays(lazy[1:], lazy[:-1], seq.priors, icp)
        _assert_batch_equal(ref, again)
        for e, l in zip(eager, lazy):
            pe, ne = dev.download(e, normals=True)
            pl, nl = dev.download(l, normals=True)
            assert np.array_equal(pe, pl) and np.array_equal(ne, nl)
    finally:
        _release(dev, eager + lazy)


def test_lazy_normals_revisit_pairs_and_p2p(dev):
    """C4-style revisit pairs (large initial errors: many fallback queries) with lazy targets and
    lazy sources whose normals are never needed; P2P on lazy clouds (no normals read); a batch
    mixing eager and lazy targets. All equal the eager runs."""
    ps = synthetic.make_revisit_pairs(4, seed=41, model=synthetic.HDL64)
    scans = ps.targets + ps.sources
    eager = _prep(dev, scans)
    lazy = _prep(dev, scans, want_normals="lazy")
    try:
        for m in ("p2plane", "p2p"):
            icp = _lib.icp_params(method=m)
            ref = dev.icp_batch_arrays(eager[4:], eager[:4], ps.init, icp)
            got = dev.icp_batch_arrays(lazy[4:], lazy[:4], ps.init, icp)
            _assert_batch_equal(ref, got)
        icp = _lib.icp_params()
        ref = dev.icp_batch_arrays(eager[4:], eager[:4], ps.init, icp)
        mixed_t = [eager[0], lazy[1], eager[2], lazy[3]]
        got = dev.icp_batch_arrays(lazy[4:], mixed_t, ps.init, icp)
        _assert_batch_equal(ref, got)
    finally:
        _release(dev, eager + lazy)


def test_lazy_normals_mixed_radii_in_one_batch(dev):
    """One P2Plane batch whose lazy targets were pre-processed with different normal parameters
    (three (radius, max_nn) groups: lsm_normals_complete runs one normals launch per group, each
    with a refine kernel on the side stream that reads the group's tables while the next group
    uploads its own): registrations and completed normals equal the eager clouds'."""
    seq = synthetic.make_sequence(7, seed=3, model=synthetic.HDL64)
    groups = [dict(normal_radius=0.3, max_nn=300), dict(normal_radius=0.5, max_nn=30),
              dict(normal_radius=0.2, max_nn=300)]
    icp = _lib.icp_params()
    eager, lazy = [], []
    try:
        for k, s in enumerate(seq.scans):
            kw = groups[k % 3]
            eager += _prep(dev, [s], **kw)
            lazy += _prep(dev, [s], want_normals="lazy", **kw)
        ref = dev.icp_batch_arrays(eager[1:], eager[:-1], seq.priors, icp)
        got = dev.icp_batch_arrays(lazy[1:], lazy[:-1], seq.priors, icp)
        _assert_batch_equal(ref, got)
        for e, l in zip(eager, lazy):
            assert np.array_equal(dev.download(e, normals=True)[1], dev.download(l, normals=True)[1])
    finally:
        _release(dev, eager + lazy)


def test_lazy_normals_completed_for_other_uses(dev, seq64k):
    """Every other use of the normals (FPFH, the plane split's priors, voxel_down_sample with
    normals, download) completes the pending ones first: the same results as eager clouds."""
    e = _prep(dev, seq64k.scans[:1])[0]
    l = _prep(dev, seq64k.scans[:1], want_normals="lazy")[0]
    try:
        fe = dev.fpfh(e)
        fl = dev.fpfh(l)
        assert np.array_equal(fe, fl)
        plane = np.array([0.0, 0.0, 1.0, 0.69])
        ge, re_ = dev.split_plane(e, plane)
        l2 = _prep(dev, seq64k.scans[:1], want_normals="lazy")[0]
        gl, rl = dev.split_plane(l2, plane)
        for a, b in ((ge, gl), (re_, rl)):
            dev.preprocess([a, b], _lib.prep_params(min_radius=-np.inf, max_radius=1e15,
                                                    min_height=-1e15, max_height=1e15))
            assert np.array_equal(dev.download(a, normals=True)[1], dev.download(b, normals=True)[1])
        l3 = _prep(dev, seq64k.scans[:1], want_normals="lazy")[0]
        ve, vl = dev.voxel_normals(e, 0.2), dev.voxel_normals(l3, 0.2)
        assert np.array_equal(dev.download(ve, normals=True)[1], dev.download(vl, normals=True)[1])
        _release(dev, [ge, re_, gl, rl, l2, l3, ve, vl])
    finally:
        _release(dev, [e, l])
