"""The env's action and observation spaces (spark_sched_sim.py:85-125, updated at :157 and :403-404).

With gymnasium installed these are gymnasium.spaces objects, exactly as the reference builds them. Without it
(this image), minimal stand-ins mirror the parts of gymnasium 0.29.1 the reference and its callers use:
`Discrete(n, start).contains` (python ints and numpy integer scalars are members), `Dict.contains`,
`Box(low, high, shape)`, `Graph(node_space, edge_space)` and `Sequence(space, stack)`, each with a `contains`
that accepts the env's observations, and the mutable `n` / `feature_space.n` the env updates per step.
"""

from __future__ import annotations

import numpy as np

NUM_NODE_FEATURES = 3  # spark_sched_sim.py:25

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium import spaces as _gs

    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    _gs = None
    HAVE_GYMNASIUM = False


def _as_int(x):
    if isinstance(x, (bool, np.bool_)):
        return None
    if isinstance(x, int):
        return int(x)
    if isinstance(x, (np.generic, np.ndarray)) and np.issubdtype(x.dtype, np.integer) and x.shape == ():
        return int(x)
    return None


class Discrete:
    def __init__(self, n: int, start: int = 0):
        self.n, self.start = int(n), int(start)

    def contains(self, x) -> bool:
        v = _as_int(x)
        return v is not None and self.start <= v < self.start + self.n

    __contains__ = contains

    def __repr__(self):
        return f"Discrete({self.n}, start={self.start})" if self.start else f"Discrete({self.n})"


class Box:
    def __init__(self, low, high, shape):
        self.low, self.high, self.shape = low, high, tuple(shape)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    __contains__ = contains

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, float32)"


class Graph:
    """gymnasium.spaces.Graph: node features in `node_space` (per node), edge features in `edge_space`."""

    def __init__(self, node_space: Box, edge_space: Discrete):
        self.node_space, self.edge_space = node_space, edge_space

    def contains(self, g) -> bool:
        try:
            nodes, edges, links = np.asarray(g.nodes), np.asarray(g.edges), np.asarray(g.edge_links)
        except AttributeError:
            return False
        if nodes.ndim != 2 or nodes.shape[1:] != self.node_space.shape:
            return False
        if not all(self.node_space.contains(r) for r in nodes):
            return False
        if edges.shape[0] != links.shape[0] or not all(self.edge_space.contains(e) for e in edges):
            return False
        return links.size == 0 or (links.ndim == 2 and links.shape[1] == 2 and bool(np.all(links >= 0))
                                   and bool(np.all(links < nodes.shape[0])))

    __contains__ = contains

    def __repr__(self):
        return f"Graph({self.node_space!r}, {self.edge_space!r})"


class Sequence:
    def __init__(self, space, stack: bool = False):
        self.feature_space, self.stack = space, stack

    def contains(self, xs) -> bool:
        try:
            return all(self.feature_space.contains(x) for x in xs)
        except TypeError:
            return False

    __contains__ = contains

    def __repr__(self):
        return f"Sequence({self.feature_space!r}, stack={self.stack})"


class Dict(dict):
    def contains(self, x) -> bool:
        if not isinstance(x, dict) or x.keys() != self.keys():
            return False
        return all(self[k].contains(x[k]) for k in self)

    __contains__ = contains


def action_space(num_executors: int):
    """spark_sched_sim.py:85-94."""
    S = _gs if HAVE_GYMNASIUM else None
    if S is not None:  # pragma: no cover
        return S.Dict({"stage_idx": S.Discrete(1, start=-1), "num_exec": S.Discrete(num_executors, start=1)})
    return Dict(stage_idx=Discrete(1, start=-1), num_exec=Discrete(num_executors, start=1))


def observation_space(num_executors: int):
    """spark_sched_sim.py:96-125: dag_batch Graph(Box(0, inf, (3,)), Discrete(1)), dag_ptr
    Sequence(Discrete(1)) (n = active stages + 1 after each observation), num_committable_execs Discrete(N+1),
    source_job_idx Discrete(1) (n = job count + 1 after reset), exec_supplies Sequence(Discrete(2N))."""
    if HAVE_GYMNASIUM:  # pragma: no cover
        S = _gs
        return S.Dict({
            "dag_batch": S.Graph(node_space=S.Box(0, np.inf, (NUM_NODE_FEATURES,)), edge_space=S.Discrete(1)),
            "dag_ptr": S.Sequence(S.Discrete(1), stack=True),
            "num_committable_execs": S.Discrete(num_executors + 1),
            "source_job_idx": S.Discrete(1),
            "exec_supplies": S.Sequence(S.Discrete(2 * num_executors), stack=True),
        })
    return Dict(
        dag_batch=Graph(node_space=Box(0, np.inf, (NUM_NODE_FEATURES,)), edge_space=Discrete(1)),
        dag_ptr=Sequence(Discrete(1), stack=True),
        num_committable_execs=Discrete(num_executors + 1),
        source_job_idx=Discrete(1),
        exec_supplies=Sequence(Discrete(2 * num_executors), stack=True),
    )


class ActionSpace(Dict):
    """Back-compat name: the env's action space (`action_space(num_executors)` without gymnasium)."""

    def __init__(self, num_executors: int):
        super().__init__(stage_idx=Discrete(1, start=-1), num_exec=Discrete(num_executors, start=1))
