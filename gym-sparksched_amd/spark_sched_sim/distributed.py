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
