"""Scheduler plugins (reference `schedulers/__init__.py`): host heuristics over the facade's obs dicts, the
batched Decima GNN over device observations, and `make_scheduler` by class name. The batched device action
drivers (fair / FIFO / random) used inside the rollout kernels are in csrc/policy.h."""

__all__ = ["Scheduler", "DecimaScheduler", "RandomScheduler", "RoundRobinScheduler", "make_scheduler",
           "preprocess_obs", "find_stage"]

from copy import deepcopy

from .heuristics import RandomScheduler, RoundRobinScheduler, Scheduler, find_stage, preprocess_obs


def __getattr__(name):  # torch is imported only when the GNN is asked for
    if name == "DecimaScheduler":
        from .decima import DecimaScheduler

        return DecimaScheduler
    raise AttributeError(name)


def make_scheduler(agent_cfg: dict):
    """Instantiate `agent_cfg["agent_cls"]` with the whole config as keyword arguments
    (schedulers/__init__.py:16-20)."""
    cls = agent_cfg["agent_cls"]
    if cls not in __all__[:4]:
        raise AssertionError(f"'{cls}' is not a valid scheduler.")
    return (globals().get(cls) or __getattr__(cls))(**deepcopy(agent_cfg))
