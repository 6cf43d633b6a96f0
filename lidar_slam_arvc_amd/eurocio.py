"""EuRoC/ASL-style dataset I/O around the scan-matching path.

Same directory layout and CSV schema as the reference's EurocReader (eurocreader/eurocreader.py)
so the CPU GTSAM back end and the viewers keep reading our outputs:

* ``<dir>/robot0/{lidar,odom,gps0}/data.csv`` with a ``#timestamp [ns]`` column;
* transforms written as ``,#timestamp [ns],x,y,z,qx,qy,qz,qw`` with the pandas index column
  (save_transforms_as_csv :46-64), quaternion from ``HomogeneousMatrix.Q()`` ([w,x,y,z] order);
* sensor times (:66-79) and loop closures (:81-97) likewise.

``sample_times`` follows tools/sampling.py:39-58 (keep times separated by >= delta_time, always
append the last one, unique).
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import yaml

from .se3 import HomogeneousMatrix


class EurocReader:
    def __init__(self, directory):
        self.directory = directory

    def _ensure_dir(self, filename):
        os.makedirs(os.path.dirname(os.path.abspath(self.directory + filename)), exist_ok=True)

    def read_csv(self, filename):
        return pd.read_csv(self.directory + filename)

    def save_csv(self, df, filename):
        df.to_csv(self.directory + filename)

    def read_transform(self, sensor):
        path = self.directory + "/robot0/" + sensor + "/transform.yaml"
        with open(path) as f:
            cfg = yaml.safe_load(f)
        return HomogeneousMatrix(cfg["transform"])

    def read_utm_ref(self, gpsname):
        with open(self.directory + "/robot0/" + gpsname + "/reference.yaml") as f:
            return yaml.safe_load(f)

    def save_transforms_as_csv(self, sensor_times, transforms, filename):
        self._ensure_dir(filename)
        rows = []
        for t, T in zip(sensor_times, transforms):
            p, q = T.pos(), T.Q()
            rows.append({"#timestamp [ns]": t, "x": p[0], "y": p[1], "z": p[2],
                         "qx": q[1], "qy": q[2], "qz": q[3], "qw": q[0]})
        df = pd.DataFrame(rows)
        df.to_csv(self.directory + filename)
        return df

    def save_sensor_times_as_csv(self, sensor_times, filename):
        self._ensure_dir(filename)
        df = pd.DataFrame([{"#timestamp [ns]": t} for t in sensor_times])
        df.to_csv(self.directory + filename)
        return df

    def save_loop_closures_as_csv(self, loop_closures, filename):
        self._ensure_dir(filename)
        rows = [{"i": p[0], "j": p[1]} for lc in loop_closures if lc is not None for p in lc]
        df = pd.DataFrame(rows)
        df.to_csv(self.directory + filename)
        return df

    def get_closest_times(self, master_sensor_times, sensor_times, warning_max_time_dif_s=0.5e9):
        st = np.asarray(sensor_times)
        out = []
        for ts in master_sensor_times:
            d = np.abs(st - ts)
            k = int(np.argmin(d))
            if d[k] > warning_max_time_dif_s:
                print("CAUTION!!! Found time difference (s): ", d[k] / 1e9)
            out.append(st[k])
        return np.array(out)

    def get_df_at_times(self, df_data, time_list):
        parts = [df_data.loc[df_data["#timestamp [ns]"] == t] for t in time_list]
        cols = ["#timestamp [ns]", "x", "y", "z", "qx", "qy", "qz", "qw"]
        if not parts:
            return pd.DataFrame(columns=cols)
        return pd.concat(parts, ignore_index=True)


def sample_times(sensor_times, start_index=10, delta_time=1e9):
    """Times at least delta_time apart from start_index on, plus the last one, unique."""
    cur = sensor_times[start_index]
    t = cur
    out = [cur]
    for i in range(start_index, len(sensor_times)):
        cur = sensor_times[i]
        if float(np.abs(cur - t)) >= delta_time:
            out.append(cur)
            t = cur
    out.append(cur)
    return np.unique(np.array(out))
