"""Multi-GPU plumbing: one process per GPU, independent streams sharded by rank, the weight arena
broadcast once from rank 0 (RCCL over xGMI on MI355X, gloo in CPU tests), max-over-ranks timing.
There is no per-step collective: streams never exchange data."""
from __future__ import annotations


def shard_streams(n_streams: int, world: int, rank: int):
    """stream s -> rank s // ceil(n/world) (contiguous blocks, SURVEY §8e round-robin alternative is equivalent)."""
    per = (n_streams + world - 1) // world
    return list(range(rank * per, min(n_streams, (rank + 1) * per)))


def broadcast_arena(tensor, src: int = 0):
    """Broadcast the weight arena (a uint8 tensor aliasing libwmx's device allocation on GPU; a host tensor under
    gloo) from `src`.  The only data-path collective of the job, paid once at start-up."""
    import torch.distributed as dist
    dist.broadcast(tensor, src=src)
    return tensor


def max_over_ranks(value: float, device="cpu") -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device="cpu") -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
