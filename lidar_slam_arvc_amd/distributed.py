"""Sequence-level sharding across GPUs.

Pairs (i, i+1) of the scan-matcher chain are independent given the odometry priors
(run_scanmatcher.py:203-206), so rank r owns a contiguous run of pairs and pre-processes the
keyframes they touch (one keyframe of halo shared with rank r+1: no point-cloud traffic). The
only exchange is the pose prefix product of compute_global_transformations
(artelib/homogeneousmatrix.py:184-205): each rank composes its chunk locally, all ranks
all-gather the 4x4 chunk totals (RCCL over xGMI on GPUs, gloo on CPU), and every rank
left-multiplies its exclusive prefix. That is 128 bytes per rank -- latency-bound, one collective.

Relative transforms are bit-identical to a single-GPU run (the ICP path is deterministic); the
composed global poses differ from the serial product only by floating-point association.
"""
from __future__ import annotations

import numpy as np


def shard_pairs(n_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous pair range [a, b) of `rank`; keyframes a .. b (inclusive) are needed."""
    base, rem = divmod(n_pairs, world)
    a = rank * base + min(rank, rem)
    b = a + base + (1 if rank < rem else 0)
    return a, b


def local_prefix(relative: np.ndarray) -> np.ndarray:
    """G[k] = R_0 R_1 ... R_k for the chunk (k = 0 .. n-1); identity-first convention below.
    The serial 4 x 4 products run in the library's host code (a NumPy loop costs ~3 us a pair)."""
    from . import _lib
    return _lib.se3_prefix(relative)


def compose_global_sharded(relative: np.ndarray, T0=None, group=None, device=None) -> np.ndarray:
    """Global poses of this rank's keyframes a .. b given its relative transforms R_a .. R_{b-1}.

    Returns (b - a + 1) x 4 x 4 poses T0 * R_0 * ... * R_{k-1} for k = a .. b (the first one is
    the pose of keyframe a). With no process group it degenerates to the serial product.
    """
    import torch
    import torch.distributed as dist

    rel = np.asarray(relative, dtype=np.float64).reshape(-1, 4, 4)
    loc = local_prefix(rel)
    T0 = np.eye(4) if T0 is None else np.asarray(T0, dtype=np.float64)
    if group is None and not (dist.is_available() and dist.is_initialized()):
        return T0 @ loc
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else "cpu"
    mine = torch.as_tensor(loc[-1].reshape(16), dtype=torch.float64, device=dev)
    allt = torch.empty(world * 16, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allt, mine, group=group)
    totals = allt.cpu().numpy().reshape(world, 4, 4)
    prefix = T0.copy()
    for r in range(rank):
        prefix = prefix @ totals[r]
    return prefix @ loc
