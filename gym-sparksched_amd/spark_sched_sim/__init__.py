"""MI355X-native batched Spark scheduling simulator (drop-in for spark_sched_sim's hot path).

Public surface:
  * ``SparkSchedSimVecEnv`` — B envs on one GPU, torch device tensors (vec_env.py)
  * ``SparkSchedSimEnv``    — single-env facade with the reference's reset/step/obs dicts (env.py)
  * ``DeviceEngine``        — the C-ABI engine wrapper (engine.py)
Everything per step runs in the gfx950 kernels of ``build/libsparksched.so``; there is no CPU fallback.
"""

__all__ = ["DeviceEngine"]

from .engine import DeviceEngine  # noqa: E402
