"""The GPU suite must test the library built from THIS tree.

The box runs the in-tree `build/libsparksched.so` pushed with the snapshot (it does not rebuild). A stale or foreign
library would make every parity claim below refer to other code, so the library's own build identity (ssim_build_id,
compiled in as -DSSIM_BUILD_ID) must equal the hash of the sources and headers that sit next to it
(__graft_entry__.source_hash). smoke() makes the same check.
"""

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


@pytest.mark.gpu
def test_loaded_library_is_this_trees_build():
    import __graft_entry__ as ge
    from spark_sched_sim import native

    assert os.path.realpath(native.LIB_PATH) == os.path.realpath(ge.LIB), "SSIM_LIB points at another library"
    assert native.build_id() == ge.source_hash(), (
        f"loaded {native.LIB_PATH} reports build {native.build_id()}, the tree's sources hash to {ge.source_hash()}: "
        "rebuild with `python __graft_entry__.py build` before pushing")
