"""CPU oracle for the ICP scan-matching hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import this package, and only as the checker / the timed CPU baseline. The product path
(``lidar_slam_arvc_amd``) never imports it and never falls back to it.

Two restatements: ``open3d_restated`` (NumPy/SciPy, the reference checker of the tests) and
``cpu_ref`` (ctypes over ``cpu/lsm_cpu.cpp``, C++/OpenMP f64 with an exact KD-tree: SURVEY.md
§8d's CPU baseline, timed by bench.py; tests/test_cpu_baseline.py checks it against the former).

Pinning status:
* loop-closure candidates / triplets / triangle acceptance, SE(3) host math, ``sample_times``
  and the EuRoC CSV schema: pinned bit-exactly against golden vectors captured by importing the
  NumPy-only reference modules in the build container (``tests/golden/make_golden.py``).
* filter_radius_height (keyframe.py:74-94): plain NumPy in the reference, but keyframe.py imports
  open3d at module level and cannot be imported here, so no vectors were captured from it; the
  restatement follows its mask line by line (strict inequalities, order kept) and is pinned by
  known-answer tests at the strict edges, NaN and inf (tests/test_oracle_kats.py).
* voxel down-sample, hybrid-kNN normals, ICP (P2P / P2Plane): the arithmetic lives in Open3D, which
  is un-vendored and absent here, so these are *parity unpinned* by reference
  fixtures. They are restated from Open3D's published algorithm and pinned by known-answer tests
  (recovery of known transforms, exact Umeyama, planar normals, hand-computed voxel keys).
"""
