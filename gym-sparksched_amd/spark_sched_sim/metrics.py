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


class RowStats:
    """rollout_worker.py:122-129 `collect_stats` for every row of a batched engine (a row = one reference worker
    whose env persists across resets):
      avg_job_duration  env.avg_job_duration: mean of the last 200 job durations over ALL of the row's episodes
                        (one deque(maxlen=200), spark_sched_sim.py:83,243-245,697), in seconds;
      avg_num_jobs      metrics.avg_num_jobs of the current episode (durations of active and completed jobs up
                        to the wall time, / wall time);
      num_completed_jobs, num_job_arrivals of the current episode: the reference's num_job_arrivals is
                        num_completed_jobs + num_active_jobs (rollout_worker.py:126-127), i.e. the arrived jobs
                        (state 1 or 2 here) -- not the completed count.
    Call `flush(rows, engine)` before an engine resets `rows` (their finished episode's completions enter the
    windows); `stats(engine)` -> float64 [B, 4]. Completions enter a window in completion-time order (stable in
    job id for equal times)."""

    def __init__(self, num_rows: int, cap: int = 200):
        from collections import deque

        self.windows = [deque(maxlen=cap) for _ in range(num_rows)]
        self.started = np.zeros(num_rows, dtype=bool)

    @staticmethod
    def _completed(ta, tc, st, e):
        done = np.nonzero(st[e] == 2)[0]
        order = done[np.argsort(tc[e, done], kind="stable")]
        return (tc[e, order] - ta[e, order]).tolist()

    def flush(self, rows, engine) -> None:
        rows = [int(r) for r in rows]
        if not any(self.started[r] for r in rows):
            self.started[rows] = True
            return
        ta, tc, st = (np.asarray(x) for x in engine.job_times_np())
        for e in rows:
            if self.started[e]:
                self.windows[e].extend(self._completed(ta, tc, st, e))
        self.started[rows] = True

    def stats(self, engine) -> np.ndarray:
        from collections import deque

        ta, tc, st = (np.asarray(x) for x in engine.job_times_np())
        wall = np.asarray(engine.host_views()["wall_time"], dtype=np.float64)
        B = ta.shape[0]
        out = np.zeros((B, 4))
        for e in range(B):
            w = deque(self.windows[e], maxlen=self.windows[e].maxlen)
            w.extend(self._completed(ta, tc, st, e))
            out[e, 0] = (np.mean(w) if len(w) else np.nan) * 1e-3
            arrived = st[e] > 0
            dur = np.minimum(tc[e, arrived], wall[e]) - ta[e, arrived]
            out[e, 1] = dur.sum() / wall[e] if wall[e] > 0 else np.nan
            out[e, 2] = float((st[e] == 2).sum())
            out[e, 3] = float(arrived.sum())
        return out
