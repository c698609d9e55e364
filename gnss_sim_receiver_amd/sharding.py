"""Channel sharding across GPUs: one process per GPU, the IF sample block broadcast
from rank 0 (RCCL over xGMI when the torch.distributed backend is "nccl"), channels dealt
round-robin so that every rank correlates a disjoint channel set of the same block.

The GNU Radio reference connects the same conditioner output to every channel
(gnss_flowgraph.cc:1127-1136); here that fan-out is the broadcast, and the per-channel blocks are
the ranks' channel shards.  No collective is needed on the tracking outputs (each rank owns its
channels); acquisition maxima are gathered with one small all_gather.
"""
from __future__ import annotations

import os

import numpy as np


def dist_env():
    """(rank, world_size, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0)))


def shard_channels(n_channels: int, world: int, rank: int) -> list:
    """Round-robin channel → rank assignment (balanced to ±1 channel)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world size")
    return list(range(rank, n_channels, world))


def weak_channels(per_rank: int, rank: int) -> list:
    """Weak scaling: rank r owns global channels [r·per_rank, (r+1)·per_rank)."""
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def broadcast_block(block, src: int = 0, group=None, async_op: bool = False):
    """Broadcast the raw IF block (a torch tensor, any dtype) from `src` to every rank."""
    import torch.distributed as dist
    flat = block.view(-1)
    if flat.dtype.is_complex:
        flat = torch_view_real(flat)
    return dist.broadcast(flat, src=src, group=group, async_op=async_op)


def torch_view_real(t):
    import torch
    return torch.view_as_real(t).view(-1)


def gather_acq_maxima(local: np.ndarray, group=None) -> np.ndarray:
    """All-gather per-rank acquisition result rows (float64 [n_prn_local, k]) → rank-ordered stack."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.from_numpy(np.ascontiguousarray(local, np.float64))
    n = torch.tensor([t.shape[0]], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx, t.shape[1]), dtype=torch.float64)
    pad[: t.shape[0]] = t
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return np.concatenate([o[: int(s.item())].numpy() for o, s in zip(outs, sizes)], axis=0)


def max_over_ranks(x: float, group=None) -> float:
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.cpu().item())
