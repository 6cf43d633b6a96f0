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


def balance_pairs(costs, world: int) -> list:
    """Cost-balanced packing of independent pairs over `world` ranks:
    longest-processing-time greedy -- pairs by decreasing cost (ties by index), each to the rank
    with the smallest load so far (ties to the lowest rank). Deterministic, so every rank
    computes the same assignment from the same costs; every pair lands on exactly one rank.
    Returns one ascending index array per rank.

    The cost of a registration is its source size times its correspondence passes (an ICP pass
    is one search per source point): the caller passes e.g. N_src * iterations from an earlier
    batch of the same keyframes (loop-closure candidates recur, loopclosing.py:80-99), or N_src
    alone when no iteration counts are known."""
    c = np.asarray(costs, dtype=np.float64).reshape(-1)
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(c)), key=lambda k: (-c[k], k))
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for k in order:
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(k)
        load[r] += c[k]
    return [np.asarray(sorted(v), dtype=np.int64) for v in out]


def balance_contiguous(costs, world: int) -> list:
    """Cost-balanced CONTIGUOUS split of independent pairs over `world` ranks: rank r gets the
    pair range [cut[r], cut[r + 1]), the cuts chosen so every prefix of ranks carries its share of
    the total cost as closely as whole pairs allow (cut[r] = the first pair whose cost prefix
    reaches r / world of the total). Unlike balance_pairs it keeps each rank's pairs adjacent, so
    re-balancing a contiguous sharding only moves the pairs next to the shard boundaries between
    neighbouring ranks. Deterministic; returns [a, b) per rank."""
    c = np.asarray(costs, dtype=np.float64).reshape(-1)
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(c)
    pre = np.concatenate([[0.0], np.cumsum(c)])
    tot = pre[-1]
    cuts = [0]
    for r in range(1, world):
        k = int(np.searchsorted(pre, tot * r / world, side="left"))
        # the nearer of the two cuts around the target, never behind the previous cut
        if k > 0 and abs(pre[k - 1] - tot * r / world) <= abs(pre[min(k, n)] - tot * r / world):
            k -= 1
        cuts.append(min(max(k, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def gather_pair_results(mine: np.ndarray, index: np.ndarray, n_total: int, group=None,
                        device=None) -> np.ndarray:
    """The sequence-level exchange of a sharded batch: every rank contributes
    its pairs' results (rows of `mine`, float64, pair order `index`) and receives all
    `n_total` rows in global pair order. One all-gather of fixed-size buffers (RCCL over xGMI
    on GPUs, gloo on CPU); ranks with fewer pairs pad. Without a process group it returns
    `mine` scattered into global order."""
    import torch
    import torch.distributed as dist

    mine = np.asarray(mine, dtype=np.float64)
    width = int(np.prod(mine.shape[1:])) if mine.ndim > 1 else 1
    rows = mine.reshape(len(index), width)
    if group is None and not (dist.is_available() and dist.is_initialized()):
        out = np.zeros((n_total, width))
        out[np.asarray(index, dtype=np.int64)] = rows
        return out.reshape((n_total,) + mine.shape[1:])
    world = dist.get_world_size(group)
    dev = device if device is not None else "cpu"
    cap = -(-n_total // world) if n_total else 0
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, torch.tensor([len(index)], dtype=torch.int64, device=dev),
                                group=group)
    cap = max(cap, int(counts.max().item()))
    buf = torch.zeros((cap, width + 1), dtype=torch.float64, device=dev)
    buf[:len(index), 0] = torch.as_tensor(np.asarray(index, dtype=np.float64), device=dev)
    buf[:len(index), 1:] = torch.as_tensor(rows, device=dev)
    allb = torch.empty((world * cap, width + 1), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allb, buf, group=group)
    allb = allb.cpu().numpy().reshape(world, cap, width + 1)
    out = np.zeros((n_total, width))
    seen = np.zeros(n_total, dtype=bool)
    for r in range(world):
        n = int(counts[r].item())
        idx = allb[r, :n, 0].astype(np.int64)
        if seen[idx].any():
            raise RuntimeError("a pair was registered by two ranks")
        seen[idx] = True
        out[idx] = allb[r, :n, 1:]
    if not seen.all():
        raise RuntimeError("some pairs were registered by no rank")
    return out.reshape((n_total,) + mine.shape[1:])


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
