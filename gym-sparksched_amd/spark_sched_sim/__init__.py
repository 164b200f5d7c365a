"""MI355X-native batched Spark scheduling simulator (drop-in for spark_sched_sim's hot path).

Public surface:
  * ``SparkSchedSimVecEnv`` — B envs on one GPU, torch device tensors (vec_env.py)
  * ``SparkSchedSimEnv``    — single-env facade with the reference's reset/step/obs dicts (env.py)
  * ``DeviceEngine``        — the C-ABI engine wrapper (engine.py)
Everything per step runs in the gfx950 kernels of ``build/libsparksched.so``; there is no CPU fallback.
"""

__all__ = ["DeviceEngine", "SparkSchedSimEnv"]

from .engine import DeviceEngine  # noqa: E402
from .env import SparkSchedSimEnv  # noqa: E402

try:  # reference-compatible registration (spark_sched_sim/__init__.py:6) when gymnasium is available
    from gymnasium.envs.registration import register

    register(id="SparkSchedSimEnv-v0", entry_point="spark_sched_sim.env:SparkSchedSimEnv")
except Exception:  # gymnasium is not installed in this image
    pass
