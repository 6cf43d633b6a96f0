"""The RCCL leg of the N-GPU path on the MI355X: bench.py at N > 1 runs distributed.py's two
device all-gathers (compose_global_sharded: the chunks' pose totals; gather_pair_results: the
loop-closure batch's per-pair results) over the "nccl" backend, which is RCCL on
ROCm. A one-GPU box cannot hold two RCCL ranks, so this runs them in a world-1 process group on
cuda:0: the collectives execute through RCCL on the device and must return exactly what the
no-collective path returns. (World sizes 2 and 3 run over gloo on the CPU, test_host.py; more
than one GPU is the driver's SCALE run.)

It runs in a child interpreter that imports torch before anything loads liblidarsm, as bench.py
does: torch ships its own HIP runtime beside the system one the library links, and a torch
imported after the library's runtime has initialised the device finds no GPU."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import socket, sys
import torch
import torch.distributed as dist
import numpy as np
sys.path.insert(0, sys.argv[1])
from lidar_slam_arvc_amd.distributed import compose_global_sharded, gather_pair_results

def random_se3(rng, n):
    out = np.tile(np.eye(4), (n, 1, 1))
    for k in range(n):
        q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
        out[k, :3, :3] = q * np.sign(np.linalg.det(q))
        out[k, :3, 3] = rng.uniform(-2.0, 2.0, 3)
    return out

rng = np.random.default_rng(21)
rel = random_se3(rng, 37)
T0 = random_se3(rng, 1)[0]
perm = rng.permutation(37)
want_T = compose_global_sharded(rel, T0)                 # no process group: no collective
want_g = gather_pair_results(rel[perm], perm, 37)
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
cuda = torch.device("cuda", 0)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                        device_id=cuda)
try:
    assert dist.get_backend() == "nccl"
    got_T = compose_global_sharded(rel, T0, group=dist.group.WORLD, device=cuda)
    got_g = gather_pair_results(rel[perm], perm, 37, group=dist.group.WORLD, device=cuda)
    torch.cuda.synchronize()
finally:
    dist.destroy_process_group()
assert np.array_equal(got_T, want_T), "compose_global_sharded"
assert np.array_equal(got_g, want_g) and np.array_equal(got_g, rel), "gather_pair_results"
print("rccl world-1 all-gathers: exact")
"""


def test_rccl_all_gathers_world1():
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "exact" in r.stdout
