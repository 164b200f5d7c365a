"""Heuristic policies restated from the reference — TEST INFRASTRUCTURE ONLY (see oracle/restatement.py).

  * ``FairPolicy``    — schedulers/heuristics/round_robin.py:7-49 (RoundRobinScheduler, dynamic partition)
  * ``RandomPolicy``  — schedulers/heuristics/random_scheduler.py:7-32 (legacy MT19937 RandomState)
  * ``mark_obs`` / ``pick_stage`` — schedulers/heuristics/utils.py:5-37
They act on the observation dicts returned by ``SparkSchedOracle`` (same layout as the reference env).
"""

from __future__ import annotations

import numpy as np


def mark_obs(obs: dict) -> None:
    """utils.py:5-15 — frontier = nodes with no incoming active edge; schedulable index = rank among flagged."""
    nodes = obs["dag_batch"].nodes
    frontier = np.ones(nodes.shape[0], dtype=bool)
    frontier[obs["dag_batch"].edge_links[:, 1]] = False
    flagged = nodes[:, 2].astype(bool)
    obs["frontier_stages"] = set(frontier.nonzero()[0])
    obs["schedulable_stages"] = dict(zip(flagged.nonzero()[0], np.arange(flagged.sum())))


def pick_stage(obs: dict, job_idx: int) -> int:
    """utils.py:17-37 — first schedulable frontier node of the job, else its first schedulable node."""
    fallback = -1
    for node in range(obs["dag_ptr"][job_idx], obs["dag_ptr"][job_idx + 1]):
        if node not in obs["schedulable_stages"]:
            continue
        i = obs["schedulable_stages"][node]
        if node in obs["frontier_stages"]:
            return i
        if fallback == -1:
            fallback = i
    return fallback


class FairPolicy:
    name = "Fair"

    def __init__(self, num_executors: int, dynamic_partition: bool = True):
        self.num_executors = num_executors
        self.dynamic = dynamic_partition

    def schedule(self, obs: dict):  # round_robin.py:14-49
        mark_obs(obs)
        n_jobs = len(obs["exec_supplies"])
        cap = int(np.ceil(self.num_executors / max(1, n_jobs))) if self.dynamic else self.num_executors
        src = obs["source_job_idx"]
        if src < n_jobs:
            i = pick_stage(obs, src)
            if i != -1:
                return {"stage_idx": i, "num_exec": obs["num_committable_execs"]}, {}
        for j in range(n_jobs):
            if obs["exec_supplies"][j] >= cap or j == src:
                continue
            i = pick_stage(obs, j)
            if i == -1:
                continue
            n = min(obs["num_committable_execs"], cap - obs["exec_supplies"][j])
            return {"stage_idx": i, "num_exec": n}, {}
        return {"stage_idx": -1, "num_exec": obs["num_committable_execs"]}, {}


class RandomPolicy:
    name = "Random"

    def __init__(self, seed: int = 42):
        self.rng = np.random.RandomState(seed)

    def schedule(self, obs: dict):  # random_scheduler.py:16-32
        mark_obs(obs)
        candidates = list(range(len(obs["exec_supplies"])))
        i = -1
        while candidates:
            j = self.rng.choice(candidates)
            i = pick_stage(obs, j)
            if i != -1:
                break
            candidates.remove(j)
        return {"stage_idx": i, "num_exec": self.rng.randint(1, obs["num_committable_execs"] + 1)}, {}


def run_episode(env, policy, seed: int = 1234, max_steps: int | None = None, record=None):
    """examples.py:84-102 — one episode; returns (avg job duration in s, number of decisions)."""
    obs, _ = env.reset(seed=seed)
    done = False
    steps = 0
    while not done:
        action, _ = policy.schedule(obs)
        if record is not None:
            record.append((int(action["stage_idx"]), int(action["num_exec"])))
        obs, _, done, _, _ = env.step(action)
        steps += 1
        if max_steps is not None and steps >= max_steps:
            break
    return steps
