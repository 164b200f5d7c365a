"""GPU-resident training around the batched simulator: rollouts collected on the
device vector env with the batched Decima policy, returns/baselines on device, PPO with data-parallel
replicas (one process per GPU, gradients all-reduced over RCCL) and the episode-statistics gather.
Restates trainers/{trainer,ppo,rollout_worker}.py and trainers/utils/{returns_calculator,baselines}.py."""

from .ppo import DECIMA_TPCH, PPO, make_trainer  # noqa: F401
from .returns import Baseline, ReturnsCalculator  # noqa: F401
from .rollouts import (AsyncRolloutCollector, ArenaRolloutBuffer, DecimaSampleArena, DeviceRolloutCollector,  # noqa: F401
                       GpuRolloutBuffer, RolloutCollector)
