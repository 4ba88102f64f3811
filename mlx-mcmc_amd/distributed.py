"""Chain sharding over GPUs (one process per GPU, torch.distributed over RCCL).

Independent chains shard embarrassingly: global chains
[0, C) are split into contiguous blocks, rank r runs chains
[offset_r, offset_r + count_r) with ``chain_offset = offset_r``.  Every draw
is keyed by the *global* chain id, so the samples of a chain do not depend on
how many GPUs run the job.  There is no exchange during sampling; the only
collective is the final gather of the samples to rank 0 (``gather_to_root``),
plus a max-reduction of wall times and sums of per-rank counts for reporting.  With the gloo backend (a
CPU rehearsal of the RCCL path, e.g. several ranks sharing one GPU) the
collectives run on host copies.
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def shard(total_chains: int, world: int, rank: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous block; the first C % world ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(int(total_chains), world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def gather_to_root(t, group=None) -> Optional[object]:
    """Gather every rank's [count_r, ...] tensor on rank 0, concatenated in rank
    (= global chain) order; other ranks get None.  Ranks may hold different
    counts (the leading dimension)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return t
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        out = gather_to_root(t.cpu(), group)
        return None if out is None else out.to(t.device)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    cmax = max(counts)
    pad = t
    if t.shape[0] < cmax:
        pad = torch.cat([t, t.new_zeros((cmax - t.shape[0],) + tuple(t.shape[1:]))])
    bufs: Optional[List] = ([torch.empty_like(pad) for _ in range(world)] if rank == 0
                            else None)
    dist.gather(pad.contiguous(), gather_list=bufs, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def _reduce_scalar(x: float, op, device=None, group=None) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op, group=group)
    return float(t.item())


def max_over_ranks(x: float, device=None, group=None) -> float:
    import torch.distributed as dist

    return _reduce_scalar(x, dist.ReduceOp.MAX, device, group)


def sum_over_ranks(x: float, device=None, group=None) -> float:
    """Sum of a per-rank count (exact in f64 below 2**53)."""
    import torch.distributed as dist

    return _reduce_scalar(x, dist.ReduceOp.SUM, device, group)
