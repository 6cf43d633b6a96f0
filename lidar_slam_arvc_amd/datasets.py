"""Write a synthetic sequence as an EuRoC/ASL-style dataset directory (the layout the reference
reads): robot0/lidar/data.csv + data/<t>.pcd, robot0/odom/data.csv (odometry =
ground truth composed with the noisy priors), robot0/scanmatcher_parameters.yaml."""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import yaml

from . import pcd, synthetic
from .se3 import HomogeneousMatrix


def write_euroc(directory, seq: synthetic.Sequence, t0_ns: int = 1_700_000_000_000_000_000,
                dt_ns: int = 500_000_000, method="icppointplane", voxel_size=None,
                pcd_mode="binary"):
    os.makedirs(os.path.join(directory, "robot0", "lidar", "data"), exist_ok=True)
    os.makedirs(os.path.join(directory, "robot0", "odom"), exist_ok=True)
    times = [t0_ns + k * dt_ns for k in range(len(seq.scans))]
    for t, scan in zip(times, seq.scans):
        pcd.write_pcd(os.path.join(directory, "robot0", "lidar", "data", f"{t}.pcd"), scan,
                      pcd_mode)
    pd.DataFrame({"#timestamp [ns]": times}).to_csv(
        os.path.join(directory, "robot0", "lidar", "data.csv"), index=False)
    # odometry poses: T_0 = I, T_{k+1} = T_k * prior_k (so relative odometry = the priors)
    T = np.eye(4)
    rows = []
    for k, t in enumerate(times):
        if k > 0:
            T = T @ seq.priors[k - 1]
        q = HomogeneousMatrix(T.copy()).Q()
        rows.append({"#timestamp [ns]": t, "x": T[0, 3], "y": T[1, 3], "z": T[2, 3],
                     "qx": q[1], "qy": q[2], "qz": q[3], "qw": q[0]})
    pd.DataFrame(rows).to_csv(os.path.join(directory, "robot0", "odom", "data.csv"), index=False)
    with open(os.path.join(directory, "robot0", "scanmatcher_parameters.yaml"), "w") as f:
        yaml.safe_dump({"start_index": 0, "delta_time": dt_ns / 1e9 * 0.99,
                        "voxel_size": voxel_size, "method": method}, f)
    return times
