"""CPU: known-answer tests that pin the Open3D restatement (parity unpinned by reference
fixtures: Open3D is absent)."""
import math

import numpy as np
import pytest

from lidar_slam_arvc_amd import synthetic
from oracle import open3d_restated as O


def test_filter_strict_bounds():
    p = np.array([[0.5, 0, 0], [0.50001, 0, 0], [35, 0, 0], [34.9999, 0, 0], [1, 1, -1.0],
                  [1, 1, -0.999], [1, 1, 50.0], [1, 1, 49.99], [np.nan, 1, 1], [np.inf, 0, 0],
                  [1, 1, np.inf], [1, 1, -np.inf], [1, np.nan, 0]])
    out = O.filter_radius_height(p)
    assert out.tolist() == [[0.50001, 0, 0], [34.9999, 0, 0], [1, 1, -0.999], [1, 1, 49.99]]


def test_voxel_keys_hand_computed():
    # bbox min = (0,0,0) -> origin = -v/2; key = floor((p + v/2) / v)
    v = 0.5
    p = np.array([[0.0, 0.0, 0.0], [0.2499, 0.0, 0.0], [0.25, 0.0, 0.0], [0.74, 1.0, 2.0],
                  [0.75, 1.0, 2.0]])
    keys, cent = O.voxel_down_sample(p, v)
    # origin (-0.25, -0.25, -0.25): 0.2499 -> floor(0.9998) = 0, 0.25 -> 1, 0.74 -> 1, 0.75 -> 2
    assert keys.tolist() == [[0, 0, 0], [1, 0, 0], [1, 2, 4], [2, 2, 4]]
    # (0,0,0) voxel holds points 0 and 1 -> mean
    assert np.array_equal(cent[0], (p[0] + p[1]) / 2.0)
    with pytest.raises(RuntimeError, match="voxel_size <= 0"):
        O.voxel_down_sample(p, 0.0)
    with pytest.raises(RuntimeError, match="too small"):
        O.voxel_down_sample(np.array([[0, 0, 0], [1e10, 0, 0]]), 1e-3)


def test_voxel_normals_averaged_not_renormalised():
    # preprocess_fpfh's second voxel_down_sample (keyframe.py:202-203) of a cloud with normals:
    # AccumulatedPoint sums the non-NaN normals and divides by the member count
    v = 0.5
    p = np.array([[0.0, 0.0, 0.0], [0.1, 0.0, 0.0], [0.2, 0.0, 0.0], [2.0, 0.0, 0.0]])
    n = np.array([[0.0, 0.0, 1.0], [1.0, 0.0, 0.0], [np.nan, 0.0, 0.0], [0.0, 1.0, 0.0]])
    keys, cent, avg = O.voxel_down_sample(p, v, normals=n)
    assert keys.tolist() == [[0, 0, 0], [4, 0, 0]]
    assert np.array_equal(cent[0], ((p[0] + p[1]) + p[2]) / 3.0)
    assert np.array_equal(avg[0], np.array([1.0, 0.0, 1.0]) / 3.0)   # NaN member counted, not added
    assert np.array_equal(avg[1], [0.0, 1.0, 0.0])
    k2, c2 = O.voxel_down_sample(p, v)                                 # same points without normals
    assert np.array_equal(k2, keys) and np.array_equal(c2, cent)


def test_fast_eigen_matches_eigh():
    rng = np.random.default_rng(0)
    A = rng.normal(size=(500, 3, 3))
    C = A @ A.transpose(0, 2, 1)
    v = O.fast_eigen3x3(C)
    v /= np.linalg.norm(v, axis=1)[:, None]
    w, V = np.linalg.eigh(C)
    assert np.abs(np.abs(np.sum(v * V[:, :, 0], axis=1)) - 1).max() < 1e-9
    # degenerate / diagonal branches (Open3D: identity -> z, zero -> 0)
    assert O.fast_eigen3x3(np.eye(3)).tolist() == [0, 0, 1]
    assert O.fast_eigen3x3(np.diag([3.0, 1.0, 2.0])).tolist() == [0, 1, 0]
    assert O.fast_eigen3x3(np.zeros((3, 3))).tolist() == [0, 0, 0]


def test_planar_patch_normals():
    rng = np.random.default_rng(1)
    xy = rng.uniform(-1, 1, size=(3000, 2))
    p = np.column_stack([xy, np.full(len(xy), -0.69)])
    n = O.estimate_normals(p, radius=0.3, max_nn=300)
    assert np.allclose(np.abs(n[:, 2]), 1.0, atol=1e-12)


def test_ldlt_matches_solve_and_pseudo_inverse():
    rng = np.random.default_rng(2)
    for _ in range(50):
        J = rng.normal(size=(40, 6))
        A = J.T @ J
        b = rng.normal(size=6)
        assert np.allclose(O.ldlt_solve(A, b), np.linalg.solve(A, b), rtol=1e-9, atol=1e-9)
    # singular: zero pivots give zero components (Eigen's pseudo-inverse of D)
    A = np.diag([2.0, 0.0, 1.0, 0.0, 0.0, 4.0])
    assert O.ldlt_solve(A, np.ones(6)).tolist() == [0.5, 0, 1.0, 0, 0, 0.25]
    assert O.ldlt_solve(np.zeros((6, 6)), np.ones(6)).tolist() == [0.0] * 6


def test_vec6_convention():
    x = np.array([0.1, -0.2, 0.3, 1.0, 2.0, 3.0])
    T = O.vec6_to_mat4(x)
    Rz = synthetic.rot_xyz(0, 0, 0.3)
    Ry = synthetic.rot_xyz(0, -0.2, 0)
    Rx = synthetic.rot_xyz(0.1, 0, 0)
    assert np.allclose(T[:3, :3], Rz @ Ry @ Rx, atol=1e-15)
    assert T[:3, 3].tolist() == [1.0, 2.0, 3.0]


def test_umeyama_exact():
    rng = np.random.default_rng(3)
    src = rng.normal(size=(200, 3)) * 5
    D = synthetic.pose_from(0.4, -1.0, 0.2, 0.3, -0.2, 1.1)
    dst = O.transform_points(D, src)
    assert np.abs(O.umeyama(src, dst) - D).max() < 1e-12


@pytest.mark.parametrize("method", ["p2p", "p2plane"])
def test_icp_recovers_known_transform(method):
    seq = synthetic.make_sequence(1, seed=5, model=synthetic.VLP16_8K)
    tgt = O.filter_radius_height(seq.scans[0])
    D = synthetic.pose_from(0.2, -0.1, 0.03, 0.01, -0.015, 0.04)
    src = O.transform_points(np.linalg.inv(D), tgt)
    nrm = O.estimate_normals(tgt) if method == "p2plane" else None
    r = O.registration_icp(src, tgt, 1.0, np.eye(4), method, nrm, max_iteration=60)
    assert np.abs(r["transformation"] - D).max() < 1e-9
    assert r["fitness"] == 1.0 and r["inlier_rmse"] < 1e-9


def test_icp_errors_and_empty():
    p = np.zeros((10, 3))
    with pytest.raises(RuntimeError, match="max_correspondence_distance"):
        O.registration_icp(p, p, 0.0)
    with pytest.raises(RuntimeError, match="normal"):
        O.registration_icp(p, p, 1.0, method="p2plane", target_normals=None)
    far = np.full((5, 3), 100.0)
    r = O.registration_icp(far, p + 0.0, 1.0, method="p2p")
    assert r["fitness"] == 0.0 and r["inlier_rmse"] == 0.0
    assert np.array_equal(r["transformation"], np.eye(4))


def test_convergence_rule_counts_updates():
    # identical clouds with identity init: first update is ~identity, second pass converges
    seq = synthetic.make_sequence(1, seed=6, model=synthetic.VLP16_8K)
    p = O.filter_radius_height(seq.scans[0])
    r = O.registration_icp(p, p, 10.0, np.eye(4), "p2p")
    assert r["iterations"] == 1 and r["fitness"] == 1.0
    r0 = O.registration_icp(p, p, 10.0, np.eye(4), "p2p", max_iteration=0)
    assert r0["iterations"] == 0


def test_norm_formula_matches_numpy():
    rng = np.random.default_rng(7)
    for v in rng.normal(size=(2000, 3)) * 9:
        assert O._norm1(v) == np.linalg.norm(v)


# ------------------------------------------------------------------ icp2planes (§8f row 2)
def test_plane_sampler_matches_library():
    from lidar_slam_arvc_amd import _lib
    for seed, n in [(0, 3), (1, 10), (2**63 + 5, 100000)]:
        a = O.plane_samples(seed, n, 200)
        assert np.array_equal(a, _lib.plane_samples(seed, n, 200))
        assert all(len(set(r)) == 3 for r in a.tolist())
        assert a.min() >= 0 and a.max() < n


def test_ransac_recovers_plane():
    rng = np.random.default_rng(3)
    xy = rng.uniform(-10, 10, size=(3000, 2))
    z = 0.02 * xy[:, 0] - 0.01 * xy[:, 1] - 0.7 + rng.normal(scale=0.002, size=3000)
    P = np.column_stack([xy, z])
    P = np.vstack([P, rng.uniform(-10, 10, size=(500, 3))])        # outliers
    plane, inl = O.segment_plane_ransac(P, 0.01, 1000, seed=1)
    n = np.array([-0.02, 0.01, 1.0]) / np.linalg.norm([-0.02, 0.01, 1.0])
    s = np.sign(plane[2])
    assert np.abs(s * plane[:3] - n).max() < 1e-3
    assert abs(s * plane[3] - 0.7 * n[2]) < 5e-3
    assert len(inl) >= 2800
    g, r = O.segment_plane(P, plane, 0.4)
    assert len(g) + len(r) == len(P) and len(g) >= 3000


def test_ransac_too_few_points():
    with pytest.raises(RuntimeError, match="ransac_n"):
        O.segment_plane_ransac(np.zeros((2, 3)))
