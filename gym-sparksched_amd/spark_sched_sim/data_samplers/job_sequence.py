"""Host-side reset sampling: the job sequence of each episode (reset-time, not on the step hot path).

Restates TPCHDataSampler.job_sequence / _sample_job's RNG consumption (tpch.py:54-73, 176-178) on a
gymnasium-seeded numpy Generator (spark_sched_sim.py:130: Generator(PCG64(SeedSequence(seed)))):
per job `integers(22)`, `choice(QUERY_SIZES)` (consumes exactly like `integers(0, 7)`, pinned in
tests/test_kats.py), then `exponential(1/rate)` after every job, while t < time_limit and under the cap.
The Generator state after sampling is handed to the device, which continues the same stream at step time
(task durations, tpch.py:75-106).
"""

from __future__ import annotations

import math

import numpy as np

from .synthetic_tpch import NUM_QUERIES, QUERY_SIZES

_MASK64 = (1 << 64) - 1


def make_rng(seed: int | None) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def sample_jobs(rng: np.random.Generator, job_arrival_cap, job_arrival_rate: float, time_limit: float):
    """Returns (template ids int32[n], arrival times float64[n]); advances `rng` like the reference."""
    mean_gap = 1 / job_arrival_rate
    tpl, arr = [], []
    t, k = 0, 0
    integers, exponential = rng.integers, rng.exponential
    while t < time_limit and (not job_arrival_cap or k < job_arrival_cap):
        q = 1 + integers(NUM_QUERIES)
        s = integers(0, len(QUERY_SIZES))
        tpl.append((int(q) - 1) * len(QUERY_SIZES) + int(s))
        arr.append(float(t))
        t += exponential(mean_gap)
        k += 1
    return np.asarray(tpl, dtype=np.int32), np.asarray(arr, dtype=np.float64)


def rng_words(rng: np.random.Generator):
    """numpy PCG64 state -> (state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger)."""
    st = rng.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    return (s >> 64) & _MASK64, s & _MASK64, (inc >> 64) & _MASK64, inc & _MASK64, int(st["has_uint32"]), int(
        st["uinteger"]) & 0xFFFFFFFF


def write_reset_record(buf: np.ndarray, offset: int, job_cap: int, tpl: np.ndarray, arr: np.ndarray, words,
                       time_limit: float) -> None:
    """Pack one env's reset record (include/sparksched.h ssim_reset_record + t_arrival[] + tpl[])."""
    from .._abi import RESET_HEAD_BYTES

    n = len(tpl)
    if n > job_cap:
        raise ValueError(f"episode has {n} jobs but job_cap is {job_cap}")
    head = np.zeros(8, dtype=np.uint64)
    head[0:4] = words[0:4]
    head[4] = np.uint64(words[4] | (words[5] << 32))
    head[5] = np.uint64(np.uint32(n)) & np.uint64(0xFFFFFFFF)
    head[6] = np.frombuffer(np.float64(time_limit).tobytes(), dtype=np.uint64)[0]
    view = buf[offset: offset + RESET_HEAD_BYTES + 12 * job_cap]
    view[:RESET_HEAD_BYTES] = head.view(np.uint8)[:RESET_HEAD_BYTES]
    t_view = view[RESET_HEAD_BYTES: RESET_HEAD_BYTES + 8 * job_cap].view(np.float64)
    i_view = view[RESET_HEAD_BYTES + 8 * job_cap: RESET_HEAD_BYTES + 12 * job_cap].view(np.int32)
    t_view[:] = 0.0
    i_view[:] = 0
    t_view[:n] = arr
    i_view[:n] = tpl


def time_limit_or_inf(options) -> float:
    if options is None:
        return math.inf
    return options.get("time_limit", math.inf)
