"""TPC-H data sampler plugin (reference spark_sched_sim/data_samplers/tpch.py, data_sampler.py).

The reference's sampler does three things: reads the per-query tables from `data/tpch/{size}/adj_mat_{q}.npy`
and `task_duration_{q}.npy` (tpch.py:118-132), draws job sequences at reset (tpch.py:54-73) and task
durations at step time (tpch.py:75-106). Here the tables are read once and packed (tpch_pack.pack: the
reference's per-job preprocessing, precomputed) for the device, which draws the task durations in the step
kernel (csrc/engine.h task_duration) from the same numpy PCG64 stream; job sequences are drawn either on the
host (`job_sequence`, the same numpy Generator calls) or in the reset kernel (ssim_reset_sampled).

`data_dir` layout (unchanged from the reference): `{data_dir}/{size}/adj_mat_{q}.npy` (square 0/1 matrix,
adj[u, v] != 0 means u -> v) and `{data_dir}/{size}/task_duration_{q}.npy` (pickled dict
`{stage_id: {"fresh_durations"|"first_wave"|"rest_wave": {exec_key: [ms, ...]}}}`), q in 1..22, size in
QUERY_SIZES. The pickled dict is read by an allow-list unpickler (safe_npy.py), never a plain np.load.
The reference downloads the data when `data/tpch` is missing (tpch.py:48-49, 109-115); there is no network
here, so a missing directory is an error when it was asked for explicitly and otherwise falls back (with a
warning) to the seeded synthetic set in the same format (synthetic_tpch.py).
"""

from __future__ import annotations

import os
import warnings
from abc import ABC, abstractmethod

import numpy as np

from . import job_sequence as js
from .safe_npy import load_npy, save_object_npy
from .synthetic_tpch import NUM_QUERIES, QUERY_SIZES
from .tpch_pack import PackedDataset, pack

DEFAULT_DATA_DIR = os.path.join("data", "tpch")  # relative to the working directory, as tpch.py:48,120


class DataSampler(ABC):
    """data_sampler.py:9-23. A sampler that runs on the device supplies TPC-H-format tables through
    `packed(num_executors)`; the env asks for nothing else at step time."""

    np_random: np.random.Generator | None = None

    def reset(self, np_random: np.random.Generator) -> None:
        self.np_random = np_random

    @abstractmethod
    def job_sequence(self, max_time: float):
        """[(t_arrival, job spec)] of one episode (reset time)."""

    def task_duration(self, job, stage, task, executor) -> float:
        raise NotImplementedError("task durations are drawn on the device (csrc/engine.h task_duration, "
                                  "restating tpch.py:75-106); there is no host step path")

    @abstractmethod
    def packed(self, num_executors: int) -> PackedDataset:
        """The dataset tables in the device layout (include/sparksched.h ssim_dataset)."""


def load_query(data_dir: str, query_num: int, query_size: str):
    """tpch.py:118-132 (`_load_query`): (adjacency matrix, task-duration dict) of one query."""
    path = os.path.join(data_dir, str(query_size))
    adj = np.asarray(load_npy(os.path.join(path, f"adj_mat_{query_num}.npy")))
    tds = load_npy(os.path.join(path, f"task_duration_{query_num}.npy"))
    tds = tds.item() if isinstance(tds, np.ndarray) and tds.shape == () else tds
    if adj.ndim != 2 or adj.shape[0] != adj.shape[1]:
        raise ValueError(f"{path}/adj_mat_{query_num}.npy is not a square matrix")
    if adj.shape[0] != len(tds):
        raise ValueError(f"query {query_num} ({query_size}): {adj.shape[0]} stages in the DAG but {len(tds)} "
                         "in the duration table")
    return adj, tds


def load_tpch(data_dir: str = DEFAULT_DATA_DIR) -> dict:
    """Every query of the on-disk dataset: {(query_num, size): (adj, task_duration_dict)}."""
    if not os.path.isdir(data_dir):
        raise FileNotFoundError(f"TPC-H data directory {data_dir!r} not found (the reference downloads it from "
                                "https://bit.ly/3F1Go8t; place the unzipped data/tpch tree there)")
    return {(q, size): load_query(data_dir, q, size) for q in range(1, NUM_QUERIES + 1) for size in QUERY_SIZES}


def save_tpch(raw: dict, data_dir: str) -> None:
    """Write a {(query_num, size): (adj, task_duration_dict)} dataset in the reference's on-disk layout."""
    for (q, size), (adj, tds) in raw.items():
        path = os.path.join(data_dir, str(size))
        os.makedirs(path, exist_ok=True)
        np.save(os.path.join(path, f"adj_mat_{q}.npy"), np.asarray(adj), allow_pickle=False)
        save_object_npy(os.path.join(path, f"task_duration_{q}.npy"), tds)


class JobSpec(tuple):
    """(query_num, query_size, template_id) of a sampled job (the reference builds a Job object here)."""

    __slots__ = ()

    def __new__(cls, query_num: int, query_size: str):
        tid = (query_num - 1) * len(QUERY_SIZES) + QUERY_SIZES.index(query_size)
        return super().__new__(cls, (query_num, query_size, tid))

    query_num = property(lambda self: self[0])
    query_size = property(lambda self: self[1])
    template_id = property(lambda self: self[2])


class TPCHDataSampler(DataSampler):
    """tpch.py:18-49. Same constructor keys (job_arrival_rate, job_arrival_cap, num_executors, warmup_delay);
    `data_dir` (default data/tpch) or in-memory `tables` ({(q, size): (adj, tds)}) select the tables. (The
    reference's config also carries `dataset: 'tpch'`, config/decima_tpch.yaml:87; like the reference, unknown
    keys are ignored.)"""

    def __init__(self, job_arrival_rate: float, job_arrival_cap: int | None, num_executors: int,
                 warmup_delay: float, data_dir: str | None = None, tables: dict | None = None, **kwargs):
        self.job_arrival_cap = job_arrival_cap
        self.job_arrival_rate = job_arrival_rate
        self.mean_interarrival_time = 1 / job_arrival_rate
        self.warmup_delay = warmup_delay
        self.num_executors = num_executors
        self.np_random = None
        self._raw = tables
        self._packed: PackedDataset | None = None
        self.source = "in-memory" if tables is not None else None
        if tables is None:
            d = data_dir or DEFAULT_DATA_DIR
            if os.path.isdir(d):
                self._raw = load_tpch(d)
                self.source = os.path.abspath(d)
            elif data_dir is not None:
                raise FileNotFoundError(f"TPC-H data directory {data_dir!r} not found")
            else:
                from .synthetic_tpch import generate

                warnings.warn(f"{DEFAULT_DATA_DIR!r} not found and no dataset given: using the seeded synthetic "
                              "TPC-H-format set (synthetic_tpch.generate(0)); the reference would download the "
                              "real traces here", stacklevel=2)
                self._raw = generate(0)
                self.source = "synthetic_tpch.generate(0)"

    @property
    def raw(self) -> dict:
        return self._raw

    def packed(self, num_executors: int | None = None) -> PackedDataset:
        n = num_executors or self.num_executors
        if self._packed is None:
            self._packed = pack(self._raw, n)
        return self._packed.with_executors(n)

    def job_sequence(self, max_time: float):
        """tpch.py:54-73 on the sampler's Generator: [(t_arrival, JobSpec)]."""
        assert self.np_random is not None
        tpl, arr = js.sample_jobs(self.np_random, self.job_arrival_cap, self.job_arrival_rate, max_time)
        return [(float(t), JobSpec(int(k) // len(QUERY_SIZES) + 1, QUERY_SIZES[int(k) % len(QUERY_SIZES)]))
                for t, k in zip(arr, tpl)]


class SyntheticTPCHDataSampler(TPCHDataSampler):
    """The seeded synthetic set in the TPC-H format (synthetic_tpch.py), selected by name."""

    def __init__(self, job_arrival_rate: float, job_arrival_cap: int | None, num_executors: int,
                 warmup_delay: float, dataset_seed: int = 0, **kwargs):
        from .synthetic_tpch import generate

        kwargs.pop("data_dir", None)
        kwargs.pop("tables", None)
        super().__init__(job_arrival_rate, job_arrival_cap, num_executors, warmup_delay,
                         tables=generate(dataset_seed), **kwargs)
        self.source = f"synthetic_tpch.generate({dataset_seed})"
