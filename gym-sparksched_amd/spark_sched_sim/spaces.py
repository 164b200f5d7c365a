"""Minimal gymnasium-compatible spaces for the env's dynamic action space (gymnasium is not installed here).

Mirrors gymnasium 0.29.1 `Discrete(n, start).contains` and `Dict.contains` exactly as the reference uses them
(spark_sched_sim.py:85-94, 276-277, 403-404): {"stage_idx": Discrete(S_act + 1, start=-1),
"num_exec": Discrete(N, start=1)}; python ints and numpy integer scalars are members, anything else is not.
"""

from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int, start: int = 0):
        self.n, self.start = int(n), int(start)

    def contains(self, x) -> bool:
        if isinstance(x, int):
            v = int(x)
        elif isinstance(x, (np.generic, np.ndarray)) and np.issubdtype(x.dtype, np.integer) and x.shape == ():
            v = int(x)
        else:
            return False
        return self.start <= v < self.start + self.n

    __contains__ = contains

    def __repr__(self):
        return f"Discrete({self.n}, start={self.start})"


class ActionSpace(dict):
    def __init__(self, num_executors: int):
        super().__init__(stage_idx=Discrete(1, start=-1), num_exec=Discrete(num_executors, start=1))

    def contains(self, action) -> bool:
        if not isinstance(action, dict) or action.keys() != self.keys():
            return False
        return all(self[k].contains(action[k]) for k in self)
