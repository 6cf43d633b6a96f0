"""CPU checks of the committed measurement records (no GPU): the headline parity summary that
tools/bench_parity.py wrote on the MI355X (profiles/bench_parity.json, the latest run; the
driver-run suite repeats the comparison in test_headline_full_sequence_vs_cpp_oracle) must
report every pair of the bench's 1999-pair batch within north_star's bar, on the sequence whose
SHA-256 the C++ oracle fixture carries."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_headline_parity_record():
    with open(os.path.join(ROOT, "profiles", "bench_parity.json")) as f:
        j = json.load(f)
    fx = np.load(os.path.join(ROOT, "tests", "golden", "seed3_seq_cpu_oracle.npz"))
    assert j["sequence_sha256"] == str(fx["sha256"])
    assert j["pairs"] == 1999
    assert j["tolerance"] == {"R_abs": 1e-4, "t_abs_m": 1e-3}
    assert j["within_tolerance"] == 1999, j.get("outside_tolerance_converged")
    assert j["outside_tolerance_converged"] == []
    assert j["nonconverged"]["gpu_hit_max_iteration"] == j["nonconverged"]["cpu_hit_max_iteration"]
