"""Multi-GPU sharding of independent walks / disturbance scenarios.

The batch shards embarrassingly: one process per GPU (``torch.distributed``; backend "nccl"
is RCCL on ROCm), each rank rolls out a contiguous block of walks on its own device with no
communication on the data path.  The only collective is the optional all-gather that
reassembles full CoM trajectories on every rank at the end (RCCL over xGMI).
"""

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int):
    """Contiguous block [start, stop) of `total` walks for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return start, stop


def allgather_walks(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """Reassemble per-rank blocks [b_r, ...] (from shard_range) into [total, ...] everywhere.

    Shards are padded to the largest block so every rank sends the same byte count (ring
    collectives over point-to-point xGMI links move equal chunks), then trimmed.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_range(total, world, r) for r in range(world)]
    cap = max(b - a for a, b in sizes)
    a, b = sizes[rank]
    if local.shape[0] != b - a:
        raise ValueError(f"rank {rank} holds {local.shape[0]} walks, its shard is {b - a}")
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: b - a] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([bufs[r][: sizes[r][1] - sizes[r][0]] for r in range(world)], 0)
