"""A `.npy` reader for the TPC-H dataset files that executes nothing from the file.

The reference stores each query's stage durations as a pickled 0-d object array holding a dict
(`task_duration_{q}.npy`, read with `np.load(..., allow_pickle=True).item()` at tpch.py:126-128). A plain
unpickler runs whatever callables the stream names. This reader parses the `.npy` header with numpy's own
format module and, for object arrays, unpickles with an allow-list: only the constructors numpy itself emits
for arrays, dtypes and scalars (plus the pickle protocol's native dict / list / tuple / int / float / str
opcodes, which construct data without calling anything) may appear. Anything else raises
`pickle.UnpicklingError` before it is called. Numeric arrays (`adj_mat_{q}.npy`) take the
`allow_pickle=False` path of np.load.
"""

from __future__ import annotations

import importlib
import pickle

import numpy as np
from numpy.lib import format as npy_format

# (module, name) pairs numpy's pickling of ndarray / dtype / numpy scalars refers to (numpy 1.x wrote
# numpy.core.*, numpy 2.x writes numpy._core.*); the 1.x names resolve to the 2.x objects
_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"): ("numpy._core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"): ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"): ("numpy", "ndarray"),
    ("numpy", "dtype"): ("numpy", "dtype"),
}


class _AllowListUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str):
        target = _ALLOWED.get((module, name))
        if target is None:
            raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")
        mod, attr = target
        try:
            return getattr(importlib.import_module(mod), attr)
        except (ImportError, AttributeError):  # numpy 1.x runtime
            return getattr(importlib.import_module(mod.replace("numpy._core", "numpy.core")), attr)


def load_npy(path: str):
    """np.load(path, allow_pickle=True) for numeric and object arrays, without executing file content."""
    with open(path, "rb") as f:
        version = npy_format.read_magic(f)
        if version == (1, 0):
            shape, fortran, dtype = npy_format.read_array_header_1_0(f)
        else:
            shape, fortran, dtype = npy_format.read_array_header_2_0(f)
        if not dtype.hasobject:
            return np.load(path, allow_pickle=False)
        arr = _AllowListUnpickler(f).load()
    if not isinstance(arr, np.ndarray):
        raise pickle.UnpicklingError(f"{path}: object payload is not an ndarray")
    return arr


def save_object_npy(path: str, obj) -> None:
    """Write `obj` as a pickled 0-d object array (the reference dataset's task_duration_{q}.npy format)."""
    a = np.empty((), dtype=object)
    a[()] = obj
    np.save(path, a, allow_pickle=True)
