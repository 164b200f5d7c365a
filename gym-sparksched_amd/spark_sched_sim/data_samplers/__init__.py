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
           "register_data_sampler", "load_tpch", "save_tpch"]

_REGISTRY: dict[str, type] = {"TPCHDataSampler": TPCHDataSampler,
                              "SyntheticTPCHDataSampler": SyntheticTPCHDataSampler}


def register_data_sampler(cls: type) -> type:
    if not (isinstance(cls, type) and issubclass(cls, DataSampler)):
        raise TypeError(f"{cls!r} is not a DataSampler subclass")
    _REGISTRY[cls.__name__] = cls
    return cls


def make_data_sampler(data_sampler_cfg: dict) -> DataSampler:
    """data_samplers/__init__.py:9-15. config/decima_tpch.yaml names no data_sampler_cls (the reference then
    raises KeyError); it defaults to TPCHDataSampler here."""
    name = data_sampler_cfg.get("data_sampler_cls", "TPCHDataSampler")
    assert name in _REGISTRY, f"'{name}' is not a valid data sampler."
    return _REGISTRY[name](**deepcopy(data_sampler_cfg))
