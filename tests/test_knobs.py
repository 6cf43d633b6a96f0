"""The library's test knobs (api.cpp kKnobs: the only environment it reads) are each documented in
DESIGN.md's knob table and exercised by a GPU test that proves the selected path exact."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _knobs():
    src = open(os.path.join(ROOT, "lidar_slam_arvc_amd", "csrc", "api.cpp")).read()
    body = re.search(r"kKnobs\[\]\s*=\s*\{(.*?)\};", src, re.S).group(1)
    return re.findall(r'"(LSM_[A-Z0-9_]+)"', body)


def test_knob_list_parsed():
    k = _knobs()
    assert len(k) == len(set(k)) and "LSM_NN_NOCERT" in k and "LSM_FB_GL" in k


def test_every_knob_documented_and_tested():
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    table = [ln for ln in design.splitlines() if ln.startswith("| `LSM_")]
    documented = set(re.findall(r"`(LSM_[A-Z0-9_]+)`", "\n".join(table)))
    tests = ""
    for f in sorted(os.listdir(os.path.join(ROOT, "tests"))):
        if f.startswith("test_gpu") and f.endswith(".py"):
            tests += open(os.path.join(ROOT, "tests", f)).read()
    for k in _knobs():
        assert k in documented, f"{k} missing from DESIGN.md's knob table"
        assert f'"{k}"' in tests, f"{k} not exercised by a GPU test"
