"""Board sharding over ranks (one process per GPU) and the episode-stats gather.

Boards are independent: rank r of a world of size W steps the
contiguous block [r * B, (r + 1) * B) of the global batch, and board i's seeds are
``base + i`` for its global index i, so a board's trajectory is the same whatever
the number of GPUs.  Nothing is exchanged on the data path; the only collectives
are the timing MAX and the gather of per-rank episode statistics, which run over
RCCL (``nccl`` backend) on GPUs and over gloo in the CPU tests.
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_range(rank, boards_per_rank):
    """Global board indices [lo, hi) owned by ``rank``."""
    return rank * boards_per_rank, (rank + 1) * boards_per_rank


def shard_seeds(base, rank, boards_per_rank):
    """Seeds of the rank's boards: ``base`` + global board index."""
    lo, hi = shard_range(rank, boards_per_rank)
    return np.arange(lo, hi, dtype=np.int64) + int(base)


def episode_stats(done, ep_return):
    """(finished episodes, sum of their returns) of one step's outputs, as f64 [2]."""
    d = done.to(torch.bool)
    n = d.sum().to(torch.float64)
    s = torch.where(d, ep_return.to(torch.float64), torch.zeros((), dtype=torch.float64, device=ep_return.device)).sum()
    return torch.stack([n, s])


def _group():
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(t):
    """In-place MAX over ranks (no-op without a process group; a group of one still runs
    the collective, so the RCCL path is exercised at world size 1 too)."""
    if _group():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def gather_stats(stats, dst=0):
    """Gather every rank's stats tensor on ``dst``; returns [W, ...] there, None elsewhere."""
    if not _group():
        return stats.unsqueeze(0)
    rank, world = dist.get_rank(), dist.get_world_size()
    out = [torch.zeros_like(stats) for _ in range(world)] if rank == dst else None
    dist.gather(stats, out, dst=dst)
    return torch.stack(out) if rank == dst else None


def pack_episode_records(ret, length, win):
    """(return f64, length i32, win i32) per board -> [B, 16] uint8 (td_episode_record)."""
    B = ret.shape[0]
    raw = torch.empty((B, 16), dtype=torch.uint8, device=ret.device)
    raw[:, :8] = ret.to(torch.float64).contiguous().reshape(B, 1).view(torch.uint8)
    raw[:, 8:12] = length.to(torch.int32).contiguous().reshape(B, 1).view(torch.uint8)
    raw[:, 12:] = win.to(torch.int32).contiguous().reshape(B, 1).view(torch.uint8)
    return raw


def unpack_episode_records(raw):
    ints = raw[:, 8:].contiguous().view(torch.int32)
    return raw[:, :8].contiguous().view(torch.float64).reshape(-1), ints[:, 0], ints[:, 1]


def gather_episode_records(ret, length, win, dst=0):
    """Gather every rank's per-board last-episode records on ``dst`` -- 16 B per board
    (return f64, length i32, win i32), the per-board payload of SURVEY.md 8(e), once per
    reporting interval -- as [world * B] tensors in global board order.  None elsewhere."""
    raw = pack_episode_records(ret, length, win)
    if not _group():
        return unpack_episode_records(raw)
    rank, world = dist.get_rank(), dist.get_world_size()
    out = [torch.zeros_like(raw) for _ in range(world)] if rank == dst else None
    dist.gather(raw, out, dst=dst)
    return unpack_episode_records(torch.cat(out)) if rank == dst else None
