"""Multi-GPU plumbing: one process per GPU, envs sharded in contiguous blocks with no
data-path collective; the only exchanges are the timing reduction of a benchmark and the gather of
per-env episode statistics (trainers/rollout_worker.py:122-129 stats, gathered for the trainer on rank 0).

Works with any torch.distributed backend: "nccl" (RCCL over xGMI) on the GPU box, "gloo" in the CPU tests.
"""

from __future__ import annotations

import os


def rank_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seeds(rank: int, envs_per_rank: int, base_seed: int = 0) -> list[int]:
    """Seeds of this rank's contiguous env block: env k of rank r is global env r*B + k."""
    return [base_seed + rank * envs_per_rank + i for i in range(envs_per_rank)]


def reduce_timing(stats, world: int):
    """stats = [elapsed, then additive counters...] (1-D float64 tensor). Returns the job-wide view:
    max elapsed over ranks (the slowest rank bounds the job), counters summed."""
    if world <= 1:
        return stats
    import torch
    import torch.distributed as dist

    tmax = stats[0:1].clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    rest = stats[1:].clone()
    dist.all_reduce(rest, op=dist.ReduceOp.SUM)
    return torch.cat([tmax, rest])


def gather_env_stats(local, world: int):
    """all_gather of a per-env statistics tensor [B_local, k] (same B on every rank); returns the global
    [world * B_local, k] tensor in global env order on every rank."""
    if world <= 1:
        return local
    import torch
    import torch.distributed as dist

    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous())
    return torch.cat(parts, dim=0)


def split_rows(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of `total` rows for `rank` (the first total % world ranks get one more)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_var(t, world: int, rank: int, dst: int = 0):
    """gather to rank `dst` of tensors whose first dimension differs across ranks (sizes all-gathered, payload
    padded to the max and gathered to `dst` only). Returns the per-rank tensors in rank order on `dst`, None
    elsewhere. bool tensors travel as uint8."""
    if world <= 1:
        return [t]
    import torch
    import torch.distributed as dist

    is_bool = t.dtype == torch.bool
    x = t.to(torch.uint8) if is_bool else t
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    sizes = [int(v.item()) for v in ns]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad.contiguous(), parts, dst=dst)
    if rank != dst:
        return None
    out = [p[:k] for p, k in zip(parts, sizes)]
    return [o.bool() for o in out] if is_bool else out


def all_gather_var(t, world: int) -> list:
    """all_gather of tensors whose first dimension differs across ranks (padded to the max, then trimmed).
    Returns the per-rank tensors in rank order. bool tensors travel as uint8 (gloo has no bool)."""
    if world <= 1:
        return [t]
    import torch
    import torch.distributed as dist

    is_bool = t.dtype == torch.bool
    x = t.to(torch.uint8) if is_bool else t
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    sizes = [int(v.item()) for v in ns]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous())
    out = [p[:k] for p, k in zip(parts, sizes)]
    return [o.bool() for o in out] if is_bool else out
