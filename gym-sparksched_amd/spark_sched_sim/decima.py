"""Drop-in for schedulers/decima/env_wrapper.py (DecimaEnvWrapper, DecimaActWrapper, DecimaObsWrapper).

Same wrapping order and observation dict ("dag_batch" GraphInstance with 5 node features, "dag_ptr",
"stage_mask", "exec_mask", "edge_masks") and the same action conversion (num_exec = 1 + act["num_exec"]),
but the features and the topological DAG-layer edge masks are computed on the GPU by
ssim_decima_features (csrc/decima.h) from the obs arena the step kernel just wrote; this module only
unpacks env 0's slice to numpy. Batched consumers use SparkSchedSimVecEnv.decima_features() (device tensors).
"""

from __future__ import annotations

from typing import Any

from .engine import decima_obs_dict

NUM_NODE_FEATURES = 5  # env_wrapper.py:9


class _Wrapper:
    def __init__(self, env):
        self.env = env

    @property
    def unwrapped(self):
        return getattr(self.env, "unwrapped", self.env)

    def __getattr__(self, name):  # forward everything else (num_executors, job_duration_buff, ...)
        return getattr(self.env, name)

    def reset(self, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        return self.env.step(action)

    def close(self):
        return self.env.close()


class DecimaActWrapper(_Wrapper):
    """converts Decima's actions to the environment's format (env_wrapper.py:19-34)"""

    def action(self, act: dict[str, Any]) -> dict[str, Any]:
        return {"stage_idx": act["stage_idx"], "num_exec": 1 + act["num_exec"]}

    def step(self, action):
        return self.env.step(self.action(action))


class DecimaObsWrapper(_Wrapper):
    """transforms environment observations into Decima's format (env_wrapper.py:37-161), on device"""

    def __init__(self, env, num_tasks_scale: int = 200, work_scale: float = 1e5) -> None:
        super().__init__(env)
        self.num_tasks_scale = num_tasks_scale
        self.work_scale = work_scale
        self.num_executors = self.unwrapped.num_executors

    def observation(self, obs: dict[str, Any]) -> dict[str, Any]:
        eng = self.unwrapped._eng
        dec = {k: (x.cpu().numpy() if hasattr(x, "cpu") else x)
               for k, x in eng.decima_features_np(self.num_tasks_scale, self.work_scale).items()}
        return decima_obs_dict(eng.host_views(), dec, 0, self.num_executors)

    def reset(self, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        return self.observation(obs), reward, terminated, truncated, info


class DecimaEnvWrapper(_Wrapper):
    """DecimaObsWrapper(DecimaActWrapper(env)) (env_wrapper.py:12-16)"""

    def __init__(self, env):
        super().__init__(DecimaObsWrapper(DecimaActWrapper(env)))
