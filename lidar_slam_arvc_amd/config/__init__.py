"""ICP_PARAMETERS: the reference's parameter singleton (config/config.py:6-34).

Loaded at import time from ``icp_parameters.yaml`` next to this file, or from the file named by
the environment variable ``LSM_ICP_PARAMETERS`` (e.g. a dataset's own copy). Same attribute
names as the reference: max_radius, min_radius, max_height, min_height, voxel_size, radius_gd,
max_nn_gd, radius_normals, max_nn, distance_threshold. As in the reference, KeyFrame uses the
hard-coded normal radius 0.3 (keyframe.py:33); ``radius_normals`` is read but unused.
"""
import os

import yaml


class IcpParameters:
    def __init__(self, path=None):
        path = path or os.environ.get("LSM_ICP_PARAMETERS") or os.path.join(
            os.path.dirname(os.path.abspath(__file__)), "icp_parameters.yaml")
        with open(path) as f:
            cfg = yaml.safe_load(f)
        self.max_radius = cfg["filter_by_radius"]["max_radius"]
        self.min_radius = cfg["filter_by_radius"]["min_radius"]
        self.max_height = cfg["filter_by_height"]["max_height"]
        self.min_height = cfg["filter_by_height"]["min_height"]
        self.voxel_size = cfg["down_sample"]["voxel_size"]
        self.radius_gd = cfg["filter_ground_plane"]["radius_normals"]
        self.max_nn_gd = cfg["filter_ground_plane"]["maximum_neighbors"]
        self.radius_normals = cfg["normals"]["radius_normals"]
        self.max_nn = cfg["normals"]["maximum_neighbors"]
        self.distance_threshold = cfg["icp"]["distance_threshold"]


ICP_PARAMETERS = IcpParameters()
