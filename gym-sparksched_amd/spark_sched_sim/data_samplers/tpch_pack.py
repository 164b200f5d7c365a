"""Packs a TPC-H-format dataset into the flat arrays the device sampler reads (ssim_dataset).

Everything the reference recomputes per job at reset time is deterministic per (query, size) and is
precomputed here once (SURVEY.md Appendix A "Durations"):
  * num_tasks from the *uncleaned* first first_wave key            (tpch.py:185-187)
  * first_wave cleaned of fresh durations (multiset) + nearest fill (tpch.py:135-159)
  * rough duration = np.mean(fresh + cleaned first + rest)          (tpch.py:162-174)
  * DAG children/parents CSR from the adjacency matrix, row-major   (tpch.py:199, networkx order)
  * executor_intervals table for N executors                        (tpch.py:237-262)
Template id = (query_num - 1) * 7 + size_index.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass

import numpy as np

from .synthetic_tpch import EXEC_LEVELS, NUM_QUERIES, QUERY_SIZES

WAVES = ("fresh_durations", "first_wave", "rest_wave")


def clean_first_wave(td: dict) -> None:
    """tpch.py:135-159 (in place)."""
    out = {}
    for key, durations in td["first_wave"].items():
        budget = {}
        for d in td["fresh_durations"][key]:
            budget[d] = budget.get(d, 0) + 1
        keep = []
        for d in durations:
            if budget.get(d, 0) > 0:
                budget[d] -= 1
            else:
                keep.append(d)
        out[key] = keep
    prev = []
    for key in sorted(out):
        if len(out[key]) == 0:
            out[key] = prev
        prev = out[key]
    td["first_wave"] = out


def executor_intervals(num_executors: int) -> np.ndarray:
    """tpch.py:237-262: (left, right) executor-count data points per local-executor count, float64."""
    table = np.zeros((num_executors + 1, 2))
    table[: EXEC_LEVELS[0] + 1] = EXEC_LEVELS[0]
    for a, b in zip(EXEC_LEVELS[:-1], EXEC_LEVELS[1:]):
        table[a + 1: b] = (a, b)
        if b > num_executors:
            break
        table[b] = b
    if num_executors > EXEC_LEVELS[-1]:
        table[EXEC_LEVELS[-1] + 1: num_executors] = EXEC_LEVELS[-1]
    return table


@dataclass
class PackedDataset:
    num_templates: int
    num_template_stages: int
    max_stages: int
    max_edges: int
    tpl_stage_base: np.ndarray
    ts_num_tasks: np.ndarray
    ts_rough: np.ndarray
    ts_child_base: np.ndarray
    ts_children: np.ndarray
    ts_parent_base: np.ndarray
    ts_parents: np.ndarray
    ts_fw_keymask: np.ndarray
    ts_fw_maxlevel: np.ndarray
    dur_off: np.ndarray
    dur_len: np.ndarray
    durations: np.ndarray
    intervals: np.ndarray
    ts_topo: np.ndarray  # uint64 [TS]: parent bits 0-31, child bits 32-63 (zeros if a template has > 32 stages)

    def arrays(self) -> list[np.ndarray]:
        from .._abi import DATASET_ARRAYS

        return [getattr(self, n) for n in DATASET_ARRAYS]

    def with_executors(self, num_executors: int) -> "PackedDataset":
        out = copy.copy(self)
        out.intervals = np.ascontiguousarray(executor_intervals(num_executors).reshape(-1))
        return out


def template_id(query_num: int, size: str) -> int:
    return (query_num - 1) * len(QUERY_SIZES) + QUERY_SIZES.index(size)


def pack(raw: dict, num_executors: int) -> PackedDataset:
    """raw: {(query_num, size): (adj, {stage_id: {wave: {exec_key: [ms]}}})}"""
    level_of = {k: i for i, k in enumerate(EXEC_LEVELS)}
    n_tpl = NUM_QUERIES * len(QUERY_SIZES)
    stage_base = [0]
    num_tasks, rough, keymask, maxlevel = [], [], [], []
    child_base, children, parent_base, parents = [0], [], [0], []
    dur_off, dur_len, durations = [], [], []
    topo = []
    max_stages = max_edges = 0
    for tid in range(n_tpl):
        q, si = tid // len(QUERY_SIZES) + 1, tid % len(QUERY_SIZES)
        adj, tds = raw[(q, QUERY_SIZES[si])]
        n = adj.shape[0]
        rows, cols = np.nonzero(adj)
        max_stages = max(max_stages, n)
        max_edges = max(max_edges, len(rows))
        kids = [[] for _ in range(n)]
        pars = [[] for _ in range(n)]
        for u, v in zip(rows.tolist(), cols.tolist()):
            kids[u].append(v)
            pars[v].append(u)
        for sid in range(n):
            td = copy.deepcopy(tds[sid])
            k0 = next(iter(td["first_wave"]))
            num_tasks.append(len(td["first_wave"][k0]) + len(td["rest_wave"][k0]))
            clean_first_wave(td)
            flat = [d for w in WAVES for lst in td[w].values() for d in lst]
            rough.append(np.mean(flat))
            mask = 0
            for key in td["first_wave"]:
                if key not in level_of:
                    raise ValueError(f"exec key {key} is not one of {EXEC_LEVELS}")
                mask |= 1 << level_of[key]
            keymask.append(mask)
            maxlevel.append(level_of[max(td["first_wave"])])
            for w in WAVES:
                for lvl, key in enumerate(EXEC_LEVELS):
                    if key in td[w]:
                        lst = td[w][key]
                        dur_off.append(len(durations))
                        dur_len.append(len(lst))
                        durations.extend(float(d) for d in lst)
                    else:
                        dur_off.append(0)
                        dur_len.append(-1)
            children.extend(kids[sid])
            child_base.append(len(children))
            parents.extend(pars[sid])
            parent_base.append(len(parents))
            if n <= 32:
                topo.append(sum(1 << p for p in pars[sid]) | (sum(1 << c for c in kids[sid]) << 32))
            else:
                topo.append(0)
        stage_base.append(stage_base[-1] + n)
    i32 = lambda x: np.ascontiguousarray(np.asarray(x, dtype=np.int32))  # noqa: E731
    return PackedDataset(
        num_templates=n_tpl,
        num_template_stages=stage_base[-1],
        max_stages=max_stages,
        max_edges=max_edges,
        tpl_stage_base=i32(stage_base),
        ts_num_tasks=i32(num_tasks),
        ts_rough=np.ascontiguousarray(np.asarray(rough, dtype=np.float64)),
        ts_child_base=i32(child_base),
        ts_children=i32(children if children else [0]),
        ts_parent_base=i32(parent_base),
        ts_parents=i32(parents if parents else [0]),
        ts_fw_keymask=i32(keymask),
        ts_fw_maxlevel=i32(maxlevel),
        dur_off=i32(dur_off),
        dur_len=i32(dur_len),
        durations=np.ascontiguousarray(np.asarray(durations if durations else [0.0], dtype=np.float64)),
        intervals=np.ascontiguousarray(executor_intervals(num_executors).reshape(-1)),
        ts_topo=np.ascontiguousarray(np.asarray(topo if max_stages <= 32 else [0] * len(topo), dtype=np.uint64)),
    )
