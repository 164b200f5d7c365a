"""StochasticTimeLimit (reference spark_sched_sim/wrappers/stochastic_time_limit.py:5-31).

Per reset the time limit is drawn from a legacy MT19937 RandomState(seed or 42).exponential(mean), the env
is reset with options={"time_limit": limit}, and `truncated` becomes True once wall_time >= limit.
"""

from __future__ import annotations

import numpy as np


class StochasticTimeLimit:
    def __init__(self, env, mean_time_limit: float, seed: int = 42):
        self.env = env
        self.mean_time_limit = mean_time_limit
        self.np_random = np.random.RandomState(seed)
        self.time_limit = None

    def reset(self, seed=None, options=None):
        if seed:
            self.np_random = np.random.RandomState(seed)
        self.time_limit = self.np_random.exponential(self.mean_time_limit)
        options = dict(options) if options else {}
        options["time_limit"] = self.time_limit
        return self.env.reset(seed=seed, options=options)

    def step(self, act):
        obs, rew, term, trunc, info = self.env.step(act)
        if info["wall_time"] >= self.time_limit:
            trunc = True
        return obs, rew, term, trunc, info

    def __getattr__(self, name):
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return getattr(self.env, "unwrapped", self.env)


class StochasticTimeLimitSampler:
    """Per-env time limits for the vector env with the wrapper's seeding semantics."""

    def __init__(self, mean: float, num_envs: int, seed: int = 42):
        self.mean = mean
        self.rngs = [np.random.RandomState(seed) for _ in range(num_envs)]

    def sample(self, env: int, seed=None) -> float:
        if seed:
            self.rngs[env] = np.random.RandomState(seed)
        return float(self.rngs[env].exponential(self.mean))
