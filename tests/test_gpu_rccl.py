"""The RCCL leg of the N-GPU path on the MI355X: bench.py at N > 1 runs distributed.py's two
device all-gathers (compose_global_sharded: the chunks' pose totals; gather_pair_results: the
loop-closure batch's per-pair results) over the "nccl" backend, which is RCCL on
ROCm. A one-GPU box cannot hold two RCCL ranks, so this runs them in a world-1 process group on
cuda:0: the collectives execute through RCCL on the device and must return exactly what the
no-collective path returns. (World sizes 2 and 3 run over gloo on the CPU, test_host.py; more
than one GPU is the driver's SCALE run.)"""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _random_se3(rng, n):
    out = np.tile(np.eye(4), (n, 1, 1))
    for k in range(n):
        q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
        out[k, :3, :3] = q * np.sign(np.linalg.det(q))
        out[k, :3, 3] = rng.uniform(-2.0, 2.0, 3)
    return out


def test_rccl_all_gathers_world1():
    import torch
    import torch.distributed as dist

    from lidar_slam_arvc_amd.distributed import compose_global_sharded, gather_pair_results

    rng = np.random.default_rng(21)
    rel = _random_se3(rng, 37)
    T0 = _random_se3(rng, 1)[0]
    perm = rng.permutation(37)
    assert not dist.is_initialized()
    want_T = compose_global_sharded(rel, T0)
    want_g = gather_pair_results(rel[perm], perm, 37)
    cuda = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=cuda)
    try:
        assert dist.get_backend() == "nccl"
        got_T = compose_global_sharded(rel, T0, group=dist.group.WORLD, device=cuda)
        got_g = gather_pair_results(rel[perm], perm, 37, group=dist.group.WORLD, device=cuda)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert np.array_equal(got_T, want_T)
    assert np.array_equal(got_g, want_g) and np.array_equal(got_g, rel)
