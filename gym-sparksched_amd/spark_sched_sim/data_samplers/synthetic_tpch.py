"""Seeded synthetic dataset in the TPC-H on-disk *format* used by the reference sampler.

The reference downloads its TPC-H traces (`spark_sched_sim/data_samplers/tpch.py:13,48-49,109-115`),
which is impossible offline, so every benchmark and parity test here runs on this generator's output.
It reproduces the structure the sampler reads:

* 22 queries x 7 sizes (`tpch.py:14-15`), query DAG = square 0/1 adjacency matrix, `adj[u, v] != 0`
  means u -> v (u is a parent of v; networkx `from_numpy_array`, `tpch.py:199`);
* per stage a dict `{"fresh_durations"|"first_wave"|"rest_wave": {exec_key: [ms, ...]}}` with
  exec keys drawn from {5,10,20,40,50,60,80,100} (`tpch.py:238`).

Deliberate irregularities so that every fallback in `TPCHDataSampler.task_duration` (`tpch.py:75-106`)
and the preprocessing (`tpch.py:135-159`) is exercised: missing keys (KeyError path), empty lists
(ValueError path), fresh durations duplicated inside `first_wave` (multiset cleaning), cleaned
first-wave lists that become empty (nearest-neighbour fill), shuffled key insertion order
(`next(iter(first_wave))` and `max(first_wave)`), and non-topological stage labels.

Invariants the reference needs to run at all (violations would crash it, not exercise it):
``rest_wave`` holds the first ``first_wave`` key (`tpch.py:185-187`), ``fresh_durations`` holds every
``first_wave`` key (`tpch.py:142`), every stage has >=1 task, every DAG has >=1 edge
(`spark_sched_sim.py:254`), and ``fresh_durations[k]`` is non-empty for every first-wave key so that
the last fallback in `task_duration` can always draw.
"""

from __future__ import annotations

import numpy as np

QUERY_SIZES = ["2g", "5g", "10g", "20g", "50g", "80g", "100g"]
NUM_QUERIES = 22
EXEC_LEVELS = [5, 10, 20, 40, 50, 60, 80, 100]

# work multiplier per data size (task count and duration grow with the scale factor)
_SIZE_TASK_SCALE = [0.35, 0.5, 0.7, 1.0, 1.5, 2.0, 2.5]
_SIZE_DUR_SCALE = [0.6, 0.75, 0.9, 1.0, 1.2, 1.35, 1.5]


def _random_dag(rng: np.random.Generator, n: int) -> np.ndarray:
    """Spark-like query DAG: each non-source stage consumes 1-2 earlier stages (joins have 2).
    Labels are permuted so the adjacency matrix is not upper triangular."""
    adj = np.zeros((n, n), dtype=np.int64)
    order = rng.permutation(n)
    for pos in range(1, n):
        child = order[pos]
        num_parents = 1 if (pos < 2 or rng.random() < 0.65) else 2
        parents = rng.choice(pos, size=min(num_parents, pos), replace=False)
        for p in parents:
            adj[order[p], child] = 1
    # occasionally add a shortcut edge (u earlier than v in topo order)
    if n >= 4 and rng.random() < 0.5:
        a, b = sorted(rng.choice(n, size=2, replace=False))
        adj[order[a], order[b]] = 1
    assert adj.sum() >= 1
    return adj


def _stage_durations(rng, num_tasks, dur_scale):
    """One stage's duration dict in the reference's 3-wave format."""
    keys = [k for k in EXEC_LEVELS if rng.random() < 0.7]
    if not keys:
        keys = [EXEC_LEVELS[int(rng.integers(len(EXEC_LEVELS)))]]
    if rng.random() < 0.3:
        rng.shuffle(keys)  # insertion order matters for next(iter(first_wave))
    base = float(rng.uniform(150.0, 1500.0)) * dur_scale
    fresh, first, rest = {}, {}, {}
    for k in keys:
        n_first = min(k, num_tasks)
        n_rest = num_tasks - n_first
        fw = list(np.round(rng.gamma(4.0, base / 4.0, size=n_first) + 50.0, 2))
        rw = list(np.round(rng.gamma(5.0, 0.8 * base / 5.0, size=n_rest) + 40.0, 2))
        # fresh executors run the first tasks: some of their durations also sit in first_wave
        n_dup = int(rng.integers(0, min(3, len(fw)) + 1))
        dups = [fw[int(i)] for i in rng.choice(len(fw), size=n_dup, replace=False)] if n_dup else []
        extra = list(np.round(rng.gamma(4.0, 1.3 * base / 4.0, size=int(rng.integers(1, 4))) + 300.0, 2))
        fresh[k] = dups + extra
        if k != keys[0] and rng.random() < 0.08:
            fw = list(dups)  # cleaning empties this list -> nearest-neighbour fill
        first[k] = fw
        r = rng.random()
        if k == keys[0]:
            rest[k] = rw  # needed by the num_tasks computation (tpch.py:185-187)
        elif r < 0.12:
            pass  # missing key -> KeyError fallback
        elif r < 0.2:
            rest[k] = []  # empty list -> ValueError fallback
        else:
            rest[k] = rw
    # num_tasks must come out of the first key exactly as the sampler recomputes it
    k0 = keys[0]
    assert len(first[k0]) + len(rest[k0]) == num_tasks
    return {"fresh_durations": fresh, "first_wave": first, "rest_wave": rest}


def generate(seed: int = 0) -> dict:
    """Return ``{(query_num, size_str): (adj_matrix, task_duration_dict)}`` for 22 x 7 queries."""
    rng = np.random.Generator(np.random.PCG64(seed))
    data = {}
    for q in range(1, NUM_QUERIES + 1):
        n_stages = int(rng.integers(2, 19))
        adj = _random_dag(rng, n_stages)
        base_tasks = rng.integers(1, 24, size=n_stages)
        for si, size in enumerate(QUERY_SIZES):
            srng = np.random.Generator(np.random.PCG64([seed, q, si]))
            stages = {}
            for s in range(n_stages):
                nt = max(1, int(round(base_tasks[s] * _SIZE_TASK_SCALE[si] * srng.uniform(0.8, 1.25))))
                stages[s] = _stage_durations(srng, nt, _SIZE_DUR_SCALE[si])
            data[(q, size)] = (adj.copy(), stages)
    return data
