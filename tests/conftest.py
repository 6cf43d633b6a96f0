import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def dev():
    from lidar_slam_arvc_amd import _lib
    return _lib.device(0)
