"""Host heuristic schedulers over the facade's observation dicts (reference `schedulers/heuristics/`).

These are the policy plugins `examples.py` and the rollout workers call: `schedule(obs) -> (action, info)` on
the single-env obs dict that `SparkSchedSimEnv` returns (`GraphInstance` nodes/edge_links, `dag_ptr`,
`exec_supplies`, `source_job_idx`, `num_committable_execs`). They are pure functions of the observation (plus,
for the random scheduler, a legacy `RandomState` stream), so the actions they return are the reference's for
the same observation. The batched device equivalents used by the vector env live in `csrc/policy.h`.
"""

from __future__ import annotations

import math
from abc import ABC, abstractmethod
from typing import Any

import numpy as np


class Scheduler(ABC):
    """Scheduler interface (schedulers/scheduler.py:10-18)."""

    name: str
    env_wrapper_cls: type | None = None

    @abstractmethod
    def schedule(self, obs: dict) -> tuple[dict, dict]:
        ...


def preprocess_obs(obs: dict[str, Any]) -> None:
    """Adds `frontier_stages` (node rows with no incoming active edge) and `schedulable_stages`
    (node row -> rank among the schedulable rows, i.e. the action's stage_idx) to `obs`
    (heuristics/utils.py:5-17)."""
    graph = obs["dag_batch"]
    n = graph.nodes.shape[0]
    has_parent = np.zeros(n, dtype=bool)
    links = np.asarray(graph.edge_links).reshape(-1, 2)
    if links.shape[0]:
        has_parent[links[:, 1]] = True
    rows = np.flatnonzero(graph.nodes[:, 2].astype(bool))
    obs["frontier_stages"] = set(np.flatnonzero(~has_parent).tolist())
    obs["schedulable_stages"] = {int(r): k for k, r in enumerate(rows.tolist())}


def find_stage(obs: dict[str, Any], job_idx: int) -> int:
    """Action stage_idx of a schedulable stage of job `job_idx`: its first frontier one in node order, else its
    first schedulable one, else -1 (heuristics/utils.py:20-37)."""
    sched = obs["schedulable_stages"]
    frontier = obs["frontier_stages"]
    fallback = -1
    for row in range(int(obs["dag_ptr"][job_idx]), int(obs["dag_ptr"][job_idx + 1])):
        k = sched.get(row)
        if k is None:
            continue
        if row in frontier:
            return k
        if fallback < 0:
            fallback = k
    return fallback


class RoundRobinScheduler(Scheduler):
    """Fair (dynamic_partition) / FIFO scheduler (heuristics/round_robin.py:7-49)."""

    def __init__(self, num_executors: int, dynamic_partition: bool = True, **kwargs):
        self.name = "Fair" if dynamic_partition else "FIFO"
        self.num_executors = num_executors
        self.dynamic_partition = dynamic_partition
        self.env_wrapper_cls = None

    def schedule(self, obs: dict) -> tuple[dict, dict]:
        preprocess_obs(obs)
        supplies = obs["exec_supplies"]
        n_jobs = len(supplies)
        committable = obs["num_committable_execs"]
        cap = math.ceil(self.num_executors / max(1, n_jobs)) if self.dynamic_partition else self.num_executors
        src = obs["source_job_idx"]
        if src < n_jobs:  # the job releasing executors keeps all of them if it can use them
            k = find_stage(obs, src)
            if k != -1:
                return {"stage_idx": k, "num_exec": committable}, {}
        for j in range(n_jobs):  # arrival order, below the cap
            if j == src or supplies[j] >= cap:
                continue
            k = find_stage(obs, j)
            if k != -1:
                return {"stage_idx": k, "num_exec": min(committable, cap - supplies[j])}, {}
        return {"stage_idx": -1, "num_exec": committable}, {}


class RandomScheduler(Scheduler):
    """Uniform job, its find_stage pick, uniform executor count (heuristics/random_scheduler.py:7-32).
    Draws from `np.random.RandomState(seed)` in the reference's order: `choice` over the remaining job
    indices until one has a schedulable stage, then `randint(1, committable + 1)`."""

    def __init__(self, seed: int = 42, **kwargs):
        self.name = "Random"
        self.env_wrapper_cls = None
        self.set_seed(seed)

    def set_seed(self, seed: int) -> None:
        self.np_random = np.random.RandomState(seed)

    def schedule(self, obs: dict) -> tuple[dict, dict]:
        preprocess_obs(obs)
        candidates = list(range(len(obs["exec_supplies"])))
        k = -1
        while candidates:
            j = self.np_random.choice(candidates)
            k = find_stage(obs, j)
            if k != -1:
                break
            candidates.remove(j)
        num_exec = self.np_random.randint(1, obs["num_committable_execs"] + 1)
        return {"stage_idx": k, "num_exec": num_exec}, {}
