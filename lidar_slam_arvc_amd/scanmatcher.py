"""Scan-matcher driver: the counterpart of the reference's run_scanmatcher.py on the MI355X path.

    python -m lidar_slam_arvc_amd.scanmatcher -i <euroc_directory> [--batch 128]

Same inputs and outputs as run_scanmatcher.scanmatcher (run_scanmatcher.py:128-237):
``robot0/scanmatcher_parameters.yaml`` (start_index, delta_time, voxel_size, method), LiDAR
times sampled with sample_times, odometry at the closest times, relative odometry priors,
ICP per consecutive pair seeded by the prior (:196-213), global transforms by the serial
product from T0 = I (:221), and the three CSVs lidar_times / scanmatcher_relative /
scanmatcher_global under ``robot0/scanmatcher/`` (:227-234).

The pair loop is batched: pairs (i, i+1) are independent given the odometry priors
(:203-206), so keyframes are pre-processed ``batch`` at a time in one device pass and their
pairs registered in one ICP batch; each batch keeps a one-keyframe halo so no keyframe is
loaded twice. Results are identical to the one-pair-at-a-time loop.
"""
from __future__ import annotations

import argparse
import time

import numpy as np
import yaml

from .eurocio import EurocReader, sample_times
from .keyframemanager import KeyFrameManager
from .se3 import (HomogeneousMatrix, compute_global_transformations,
                  compute_homogeneous_transforms, compute_relative_transformations)


def read_scanmatcher_parameters(directory):
    with open(directory + "/robot0/scanmatcher_parameters.yaml") as f:
        return yaml.safe_load(f)


def prepare_experiment_data(euroc_read, start_index=20, delta_time=1.0):
    df_lidar = euroc_read.read_csv(filename="/robot0/lidar/data.csv")
    scan_times = sample_times(df_lidar["#timestamp [ns]"].to_numpy(), start_index=start_index,
                              delta_time=delta_time * 1e9)
    df_odo = euroc_read.read_csv(filename="/robot0/odom/data.csv")
    odo_times = euroc_read.get_closest_times(scan_times, df_odo["#timestamp [ns]"].to_numpy())
    df_odo = euroc_read.get_df_at_times(df_odo, odo_times)
    try:
        df_gps = euroc_read.read_csv(filename="/robot0/gps0/data.csv")
        gps_times = euroc_read.get_closest_times(scan_times, df_gps["#timestamp [ns]"].to_numpy())
        df_gps = euroc_read.get_df_at_times(df_gps, gps_times)
    except FileNotFoundError:
        gps_times, df_gps = None, None
    return scan_times, odo_times, gps_times, df_odo, df_gps


def compute_relative_odometry_transformations(df_odo):
    return compute_relative_transformations(compute_homogeneous_transforms(df_odo))


def register_chain(kfm: KeyFrameManager, priors, batch: int = 128, verbose: bool = False):
    """ICP of every consecutive pair (i, i+1) of kfm's keyframes, seeded by priors[i]."""
    n = len(kfm.keyframes)
    out = []
    t0 = time.time()
    for a in range(0, n - 1, batch):
        b = min(a + batch, n - 1)              # pairs a .. b-1 need keyframes a .. b
        for k in range(a, b + 1):
            kfm.load_pointcloud(k)
        kfm.pre_process_batch(list(range(a, b + 1)))
        out += kfm.compute_transformations([(i, i + 1) for i in range(a, b)], priors[a:b])
        for k in range(a, b):                  # keep b: it is the next batch's first target
            kfm.unload_pointcloud(k)
        if verbose:
            print(f"pairs {a}..{b - 1}: {(time.time() - t0) / b * 1e3:.2f} ms/pair")
    return out


def scanmatcher(directory, batch: int = 128, verbose: bool = True):
    prm = read_scanmatcher_parameters(directory)
    start_index = prm.get("start_index", 0)
    delta_time = prm.get("delta_time", 0.5)
    voxel_size = prm.get("voxel_size", None)
    method = prm.get("method", "icppointplane")
    T0 = HomogeneousMatrix(np.eye(4))
    er = EurocReader(directory=directory)
    scan_times, _, _, df_odo, _ = prepare_experiment_data(er, start_index, delta_time)
    priors = compute_relative_odometry_transformations(df_odo)
    kfm = KeyFrameManager(directory=directory, scan_times=scan_times, voxel_size=voxel_size,
                          method=method)
    for i in range(len(scan_times)):
        kfm.add_keyframe(i)
    relative = register_chain(kfm, priors, batch=batch, verbose=verbose)
    kfm.unload_pointcloud(len(scan_times) - 1)
    glob = compute_global_transformations(relative, T0=T0, Trobot_gps=None)
    er.save_sensor_times_as_csv(scan_times, filename="/robot0/scanmatcher/lidar_times.csv")
    er.save_transforms_as_csv(scan_times, relative,
                              filename="/robot0/scanmatcher/scanmatcher_relative.csv")
    er.save_transforms_as_csv(scan_times, glob,
                              filename="/robot0/scanmatcher/scanmatcher_global.csv")
    return relative, glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-i", "--ifile", required=True, help="EuRoC-style dataset directory")
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    scanmatcher(a.ifile, batch=a.batch)


if __name__ == "__main__":
    main()
