"""Single-env drop-in for spark_sched_sim.SparkSchedSimEnv (reference spark_sched_sim/spark_sched_sim.py:29-245).

Same constructor config keys, `reset(seed, options) -> (obs, info)`, `step(action) -> (obs, reward,
terminated, truncated, info)`, observation dicts (GraphInstance(nodes f32[S,3], edges i64[E], edge_links
i64[E,2]), dag_ptr, num_committable_execs, source_job_idx, exec_supplies), action-space bookkeeping and
exception types (ValueError / KeyError / AssertionError). The state machine runs on the GPU (one
wavefront); this class only marshals one env's slice of the obs arena to numpy.
"""

from __future__ import annotations

import math
from collections import deque
from typing import Any

import numpy as np

from . import _abi
from .engine import DeviceEngine, decode_trace, executor_histories, obs_dict
from .spaces import action_space, observation_space

NUM_NODE_FEATURES = 3

try:  # a gymnasium.Env subclass when gymnasium is importable (gym.make / wrappers then work unchanged)
    from gymnasium import Env as _EnvBase  # type: ignore
except Exception:  # noqa: BLE001 - gymnasium is not installed in this image

    class _EnvBase:  # the attributes of gymnasium.Env the reference's callers touch
        metadata: dict = {}
        render_mode = None
        spec = None

        @property
        def unwrapped(self):
            return self

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            self.close()
            return False


def resolve_dataset(env_cfg: dict, dataset=None):
    """The tables the device samples from: an explicit `dataset` (raw {(q, size): (adj, tds)} dict or
    PackedDataset) wins; otherwise the config's data sampler plugin (make_data_sampler, defaulting to
    TPCHDataSampler over data/tpch, spark_sched_sim.py:54 / data_samplers/__init__.py:9-15)."""
    if dataset is not None:
        return dataset
    from .data_samplers import make_data_sampler

    return make_data_sampler(env_cfg).packed(env_cfg["num_executors"])


def _raise_for(err: int, action) -> None:
    if err & _abi.SSIM_ERR_SPACE:
        raise ValueError("invalid action: does not belong to the action space")
    if err & _abi.SSIM_ERR_KEY:
        raise KeyError(action["stage_idx"])
    if err & _abi.SSIM_ERR_TOO_MANY:
        raise ValueError("invalid action: too many executors requested")
    if err & _abi.SSIM_ERR_SAMPLER:
        raise ValueError("task_duration: no duration data for the sampled executor key")
    if err & _abi.SSIM_ERR_INVARIANT:
        raise AssertionError("simulator invariant violated (reference `assert`)")
    if err & (_abi.SSIM_ERR_CAPACITY | _abi.SSIM_ERR_RESET):
        raise RuntimeError(f"device capacity/reset error {err:#x}")
    if err & _abi.SSIM_ERR_PENDING:
        # a step preempted by a budget launch (SSIM_ROLLOUT_PREEMPT) was completed instead: this action, chosen on
        # the observation before that step, was NOT applied
        raise RuntimeError("a preempted step was completed by this call; the action was not applied")


class SparkSchedSimEnv(_EnvBase):
    """A Gymnasium environment that simulates DAG job scheduling in Spark, stepped on the GPU."""

    metadata = {"render_modes": ["human"], "render_fps": 30}

    def __init__(self, env_cfg: dict[str, Any], dataset=None, device="cuda", job_cap: int | None = None,
                 history_cap: int = 0, _engine_factory=None):
        self.num_executors: int = env_cfg["num_executors"]
        self.moving_delay = env_cfg["moving_delay"]
        self.beta = env_cfg.get("beta", 0)
        self.job_arrival_cap = env_cfg.get("job_arrival_cap")
        self.render_mode = env_cfg.get("render_mode")
        if self.render_mode == "human":
            raise ValueError("pygame is unavailable")  # rendering is out of scope (no renderer is built)
        dataset = resolve_dataset(env_cfg, dataset)
        # history_cap > 0 records the per-episode event trace (that many records) for render_data()
        self.history_cap = int(history_cap)
        factory = _engine_factory or (lambda cfg, ds: DeviceEngine(cfg, 1, ds, device=device, job_cap=job_cap,
                                                                   trace_cap=self.history_cap))
        self._eng = factory(dict(env_cfg), dataset)
        self.action_space = action_space(self.num_executors)
        self.observation_space = observation_space(self.num_executors)
        self.job_duration_buff: deque = deque(maxlen=200)
        self.wall_time = 0.0
        self._obs = None
        self._have_episode = False

    # -- gym API ------------------------------------------------------------------------------------
    def reset(self, seed: int | None = None, options: dict | None = None):
        if self._have_episode:
            self._flush_durations()
        self._eng.reset(seeds=[seed] if seed is not None else None, options=options)
        self._have_episode = True
        v = self._eng.host_views()
        err = int(v["counts"][0][_abi.OC_ERR])
        if err:
            _raise_for(err, {"stage_idx": None})
        self.job_arrival_cap = self._eng.sampler.arrival_cap[0]
        self.observation_space["source_job_idx"].n = self.job_arrival_cap + 1  # :157
        return self._observe(v), self.info

    def step(self, action: dict):
        if not self.action_space.contains(action):
            raise ValueError("invalid action: does not belong to the action space")
        self._eng.step([int(action["stage_idx"])], [int(action["num_exec"])])
        v = self._eng.host_views()
        c = v["counts"][0]
        err = int(c[_abi.OC_ERR])
        if err:
            _raise_for(err, action)
        obs = self._observe(v)
        return obs, float(v["reward"][0]), bool(c[_abi.OC_TERMINATED]), False, self.info

    def close(self) -> None:
        self._eng.close()

    # -- reference properties (spark_sched_sim.py:227-245) ------------------------------------------
    @property
    def unwrapped(self) -> "SparkSchedSimEnv":
        return self

    @property
    def info(self) -> dict:
        return {"wall_time": self.wall_time}

    @property
    def all_jobs_complete(self) -> bool:
        c = self._counts()
        return int(c[_abi.OC_NUM_COMPLETED]) == self.job_arrival_cap

    @property
    def num_completed_jobs(self) -> int:
        return int(self._counts()[_abi.OC_NUM_COMPLETED])

    @property
    def num_active_jobs(self) -> int:
        return int(self._counts()[_abi.OC_NUM_JOBS])

    @property
    def avg_job_duration(self) -> float:
        """Mean of the last 200 job durations over all episodes (spark_sched_sim.py:83,243-245,697: one
        deque(maxlen=200) that survives resets). The current episode's completions are appended in completion
        order to the finished episodes' buffer, then the window is cut to 200."""
        window = deque(self.job_duration_buff, maxlen=200)
        window.extend(self._episode_durations())
        return np.mean(window).item() * 1e-3

    def job_times(self):
        """(t_arrival, t_completed, state) numpy arrays of this episode's jobs."""
        ta, tc, st = self._eng.job_times_np()
        n = int(self._counts()[_abi.OC_NUM_ARRIVED]) if self._have_episode else 0
        total = self.job_arrival_cap or 0
        return ta[0][:total], tc[0][:total], st[0][:total], n

    # -- render data (spark_sched_sim.py:408-426 `_render_frame`; drawing itself needs pygame) ---------
    def _trace(self) -> list:
        if self.history_cap <= 0:
            raise ValueError("render data needs SparkSchedSimEnv(..., history_cap=N)")
        v = self._eng.host_views()
        n = int(v["counts"][0][_abi.OC_TRACE_LEN])
        if n > self.history_cap:
            raise RuntimeError(f"event trace overflowed history_cap={self.history_cap} ({n} records)")
        return decode_trace(np.asarray(v["trace"][0]), n)

    def executor_histories(self) -> list[list[list]]:
        """Executor.history of every executor for the current episode (executor.py:22-44)."""
        return executor_histories(self._trace(), self.num_executors)

    def render_data(self) -> dict:
        """The arguments `_render_frame` (spark_sched_sim.py:408-424) hands to the renderer: executor
        histories, completion times of the completed jobs (in the reference's set order), wall time, average job
        duration (int seconds, metrics.avg_job_duration * 1e-3), active and completed job counts."""
        from . import metrics

        recs = self._trace()
        # the reference iterates its `completed_job_ids` set: a set built by the same add() sequence (completion
        # order, no removals within an episode) iterates in the same order
        t_done, completed = {}, set()
        for t, kind, _e, j, _s, _q in recs:
            if kind == _abi.TR_JOB_DONE:
                t_done[j] = t
                completed.add(j)
        return {"executor_histories": executor_histories(recs, self.num_executors),
                "job_completion_times": [t_done[j] for j in completed],
                "wall_time": self.wall_time,
                "average_job_duration": int(metrics.avg_job_duration(self) * 1e-3),
                "num_active_jobs": self.num_active_jobs,
                "num_jobs_completed": self.num_completed_jobs}

    # -- internals ----------------------------------------------------------------------------------
    def _counts(self):
        return self._eng.host_views()["counts"][0]

    def _observe(self, v):
        obs = obs_dict(v, 0)
        self.wall_time = float(v["wall_time"][0])
        n = obs["dag_batch"].nodes.shape[0] + 1
        self.action_space["stage_idx"].n = n  # :403-404
        self.observation_space["dag_ptr"].feature_space.n = n
        return obs

    def _episode_durations(self):
        ta, tc, st, _ = self.job_times()
        done = np.nonzero(st == 2)[0]
        order = done[np.argsort(tc[done], kind="stable")]
        return [float(tc[j] - ta[j]) for j in order]

    def _flush_durations(self):
        for d in self._episode_durations():
            self.job_duration_buff.append(d)


def make(env_cfg: dict, **kw) -> SparkSchedSimEnv:
    """gym.make("spark_sched_sim:SparkSchedSimEnv-v0", env_cfg=...) equivalent (spark_sched_sim/__init__.py:6)."""
    return SparkSchedSimEnv(env_cfg, **kw)


def time_limit_from(options) -> float:
    return math.inf if not options else options.get("time_limit", math.inf)
