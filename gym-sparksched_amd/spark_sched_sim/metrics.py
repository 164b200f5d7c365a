"""Episode metrics (reference spark_sched_sim/metrics.py:4-23) computed from the device job tables."""

from __future__ import annotations

import numpy as np


def job_durations(env) -> list[float]:
    """Durations of active and completed jobs; active jobs are measured up to the current wall time."""
    env = getattr(env, "unwrapped", env)
    ta, tc, st, _ = env.job_times()
    out = []
    for j in np.nonzero(st > 0)[0]:
        t_end = min(tc[j], env.wall_time)
        out.append(float(t_end - ta[j]))
    return out


def avg_job_duration(env) -> float:
    return np.mean(job_durations(env))


def avg_num_jobs(env) -> float:
    env_u = getattr(env, "unwrapped", env)
    return sum(job_durations(env)) / env_u.wall_time


def job_duration_percentiles(env):
    return np.percentile(job_durations(env), [25, 50, 75, 100])
