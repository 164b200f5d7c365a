"""Data sampler plugins (reference spark_sched_sim/data_samplers/__init__.py:1-15).

`make_data_sampler(cfg)` instantiates the class named by `cfg["data_sampler_cls"]` with the whole config as
keyword arguments, as the reference does. The registry starts with the reference's TPCHDataSampler and the
synthetic TPC-H-format sampler; `register_data_sampler` adds user classes (they must implement
`DataSampler.packed`, i.e. provide TPC-H-format tables, since durations are drawn on the device).
"""

from __future__ import annotations

from copy import deepcopy

from .tpch import DataSampler, SyntheticTPCHDataSampler, TPCHDataSampler, load_tpch, save_tpch

__all__ = ["DataSampler", "TPCHDataSampler", "SyntheticTPCHDataSampler", "make_data_sampler",
           "register_data_sampler", "check_device_sampler", "load_tpch", "save_tpch"]

_REGISTRY: dict[str, type] = {"TPCHDataSampler": TPCHDataSampler,
                              "SyntheticTPCHDataSampler": SyntheticTPCHDataSampler}


def check_device_sampler(cls: type) -> None:
    """The contract a sampler class must meet to drive the device engine (INTEGRATION.md "Data samplers"):
    task durations are drawn in the step kernel from TPC-H-format tables (csrc/engine.h task_duration, restating
    tpch.py:75-106), so the class supplies those tables through `packed(num_executors)` and must not rely on its
    own per-task `task_duration` hook (data_sampler.py:19-23), which the device would never call. Raises TypeError
    naming what is wrong, at registration / construction time instead of at the first step."""
    if not (isinstance(cls, type) and issubclass(cls, DataSampler)):
        raise TypeError(f"{cls!r} is not a DataSampler subclass")
    if cls.task_duration is not DataSampler.task_duration:
        raise TypeError(f"{cls.__name__} overrides task_duration(); the device engine draws task durations itself "
                        "from the TPC-H-format tables the sampler returns from packed(num_executors) (tpch.py:75-106 "
                        "semantics) and never calls a per-task hook. Express the durations as such tables "
                        "(tpch_pack.pack of a {(query, size): (adj, task_duration_dict)} dict) instead.")
    missing = sorted(getattr(cls, "__abstractmethods__", ()))
    if missing:
        raise TypeError(f"{cls.__name__} does not implement {', '.join(missing)}: a device sampler provides "
                        "job_sequence(max_time) and packed(num_executors)")


def register_data_sampler(cls: type) -> type:
    check_device_sampler(cls)
    _REGISTRY[cls.__name__] = cls
    return cls


def make_data_sampler(data_sampler_cfg: dict) -> DataSampler:
    """data_samplers/__init__.py:9-15. config/decima_tpch.yaml names no data_sampler_cls (the reference then
    raises KeyError); it defaults to TPCHDataSampler here."""
    name = data_sampler_cfg.get("data_sampler_cls", "TPCHDataSampler")
    assert name in _REGISTRY, f"'{name}' is not a valid data sampler."
    check_device_sampler(_REGISTRY[name])
    return _REGISTRY[name](**deepcopy(data_sampler_cfg))
