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


def test_library_loads_after_torch():
    """native.lib() imports torch before it dlopens the HIP library: the library's libamdhip64 dependency must resolve
    to the HIP runtime torch loaded (loaded the other way round, torch's device init fails with "no ROCm-capable
    device" and ssim_create cannot copy to the device; scripts/diag_init_order.py is the GPU check)."""
    import subprocess

    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from spark_sched_sim import native\n"
            "assert 'torch' not in sys.modules\n"
            "native.lib()\n"
            "assert 'torch' in sys.modules\n") % (REPO, os.path.join(REPO, "gym-sparksched_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
