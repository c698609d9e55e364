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


def shard_prns(n_prns: int, world: int, rank: int) -> list:
    """Acquisition cells sharded by PRN slot (round-robin): a rank searches every Doppler bin of its
    PRNs, so each per-PRN statistic — first-vs-second peak in the peak's row, or the CFAR input power
    of the row opposite the peak bin ((idx + nb/2) % nb, pcps_acquisition.cc:496-528) — is complete
    on one rank and only the per-PRN results travel (one all-gather).  Sharding the bins instead
    would need a second exchange for the opposite-row power."""
    return shard_channels(n_prns, world, rank)


ACQ_ROW_FIELDS = ("prn_slot", "doppler_index", "code_index", "doppler_hz", "peak", "input_power", "test_statistic", "acq_delay_samples")


def acq_rows(results, slots) -> np.ndarray:
    """Per-PRN acquisition results (gnsship_acq_result-like objects) → float64 rows (ACQ_ROW_FIELDS)."""
    rows = np.zeros((len(slots), len(ACQ_ROW_FIELDS)), np.float64)
    for i, (r, s) in enumerate(zip(results, slots)):
        rows[i] = (s, r.doppler_index, r.code_index, r.doppler_hz, r.peak, r.input_power, r.test_statistic, r.acq_delay_samples)
    return rows


def pad_rows(rows: np.ndarray, n: int) -> np.ndarray:
    """Fixed-size all-gather payload: `n` rows, unused ones with prn_slot = -1."""
    out = np.zeros((n, rows.shape[1]), np.float64)
    out[:, 0] = -1
    out[: len(rows)] = rows
    return out


def merge_acq_rows(gathered: np.ndarray) -> dict:
    """Rank-ordered gathered rows → {prn_slot: row}, padding dropped (each slot on exactly one rank)."""
    out = {}
    for row in np.asarray(gathered).reshape(-1, len(ACQ_ROW_FIELDS)):
        if row[0] >= 0:
            slot = int(row[0])
            if slot in out:
                raise ValueError(f"PRN slot {slot} reported by two ranks")
            out[slot] = row
    return out


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
