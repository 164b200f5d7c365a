"""Loader for the in-tree gfx950 library (libsparksched.so). Fails loudly: there is no CPU fallback."""

from __future__ import annotations

import ctypes as ct
import os

from ._abi import SsimConfig, SsimDataset, SsimLayout

_HERE = os.path.dirname(os.path.abspath(__file__))
# SSIM_LIB overrides the path (development A/B runs of alternative builds of the same sources)
LIB_PATH = os.environ.get("SSIM_LIB") or os.path.join(os.path.dirname(_HERE), "build", "libsparksched.so")

_lib = None


class NativeError(RuntimeError):
    pass


def lib() -> ct.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # torch first: its HIP runtime must be the process's (the library's libamdhip64 dependency then resolves to the copy
    # torch loaded). Loaded the other way round, torch's device init later fails ("no ROCm-capable device").
    import torch  # noqa: F401

    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"libsparksched.so not found at {LIB_PATH}; build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). The simulator has no CPU fallback.")
    L = ct.CDLL(LIB_PATH)
    vp, i32, u64 = ct.c_void_p, ct.c_int32, ct.c_uint64
    L.ssim_layout_for.argtypes = [ct.POINTER(SsimConfig), ct.POINTER(SsimLayout)]
    L.ssim_create.argtypes = [ct.POINTER(SsimConfig), ct.POINTER(SsimDataset), vp, vp, vp, ct.POINTER(vp)]
    L.ssim_destroy.argtypes = [vp]
    L.ssim_reset.argtypes = [vp, vp]
    L.ssim_step.argtypes = [vp, vp, vp, vp]
    L.ssim_policy.argtypes = [vp, i32, u64, u64, vp, vp, vp]
    L.ssim_rollout.argtypes = [vp, i32, u64, i32, vp, vp]
    L.ssim_rollout_ex.argtypes = [vp, i32, u64, i32, i32, vp, vp, vp]
    L.ssim_rollout_budget.argtypes = [vp, i32, u64, i32, ct.c_int64, i32, vp, vp, vp]
    L.ssim_rollout_steps.argtypes = [vp, i32, u64, vp, i32, i32, vp, vp, vp]
    L.ssim_reset_sampled.argtypes = [vp, vp, vp, vp, vp]
    L.ssim_decima_policy.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                     vp]
    L.ssim_job_times.argtypes = [vp, vp, vp, vp, vp]
    L.ssim_decima_features.argtypes = [vp, ct.c_float, ct.c_float, vp, vp, vp, vp, vp]
    L.ssim_decima_workspace_bytes.argtypes = [vp]
    L.ssim_decima_workspace_bytes.restype = ct.c_int64
    L.ssim_decima_rollout_lds_bytes.argtypes = [vp]
    L.ssim_decima_rollout_lds_bytes.restype = ct.c_int64
    L.ssim_decima_rollout.argtypes = [vp, vp, i32, ct.c_float, ct.c_float, u64, u64, i32, ct.c_int64, i32, vp, vp,
                                      ct.c_int64, vp, vp, vp]
    L.ssim_last_error.restype = ct.c_char_p
    L.ssim_build_id.restype = ct.c_char_p
    L.ssim_debug_set_trace.argtypes = [vp, vp, i32, i32, vp, vp]
    L.ssim_debug_set_trace.restype = ct.c_int
    L.ssim_debug_set_trace_ex.argtypes = [vp, vp, i32, i32, vp, i32, vp]
    L.ssim_debug_set_trace_ex.restype = ct.c_int
    L.ssim_debug_kernel_name.argtypes = [vp, i32]
    L.ssim_debug_kernel_name.restype = ct.c_char_p
    L.ssim_linear_fwd.argtypes = [vp, vp, vp, vp, ct.c_int64, i32, i32, i32, vp]
    L.ssim_linear_fwd.restype = ct.c_int
    L.ssim_linear_wgrad_parts.argtypes = [ct.c_int64]
    L.ssim_linear_wgrad_parts.restype = i32
    L.ssim_linear_wgrad.argtypes = [vp, vp, vp, vp, ct.c_int64, i32, i32, vp, i32, vp]
    L.ssim_linear_wgrad.restype = ct.c_int
    L.ssim_mlp3_supported.argtypes = [i32, i32, i32, i32, i32]
    L.ssim_mlp3_supported.restype = i32
    L.ssim_mlp3_fwd.argtypes = [vp, vp, i32] + [vp] * 9 + [ct.c_int64, i32, i32, i32, i32, i32, ct.c_float, vp]
    L.ssim_mlp3_fwd.restype = ct.c_int
    L.ssim_mlp3_parts.argtypes = [ct.c_int64]
    L.ssim_mlp3_parts.restype = i32
    L.ssim_mlp3_partial_floats.argtypes = [ct.c_int64, i32, i32, i32, i32]
    L.ssim_mlp3_partial_floats.restype = ct.c_int64
    L.ssim_mlp3_bwd.argtypes = [vp, vp, vp, i32] + [vp] * 14 + [ct.c_int64, i32, i32, i32, i32, i32, ct.c_float, vp,
                                                                 i32, vp]
    L.ssim_mlp3_bwd.restype = ct.c_int
    L.ssim_discounted_returns.argtypes = [vp, vp, vp, ct.c_int64, ct.c_int64, i32, vp]
    L.ssim_discounted_returns.restype = ct.c_int
    for name in ("ssim_layout_for", "ssim_create", "ssim_destroy", "ssim_reset", "ssim_step", "ssim_policy",
                 "ssim_rollout", "ssim_rollout_ex", "ssim_rollout_budget", "ssim_rollout_steps", "ssim_reset_sampled",
                 "ssim_job_times", "ssim_decima_features", "ssim_decima_policy", "ssim_decima_rollout"):
        getattr(L, name).restype = ct.c_int
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise NativeError(f"{what} failed ({rc}): {lib().ssim_last_error().decode(errors='replace')}")


EXPORTED_SYMBOLS = ["ssim_layout_for", "ssim_create", "ssim_destroy", "ssim_reset", "ssim_step", "ssim_policy",
                    "ssim_rollout", "ssim_rollout_ex", "ssim_rollout_budget", "ssim_rollout_steps", "ssim_reset_sampled",
                    "ssim_job_times",
                    "ssim_decima_features", "ssim_decima_policy", "ssim_decima_workspace_bytes", "ssim_decima_rollout",
                    "ssim_decima_rollout_lds_bytes",
                    "ssim_last_error", "ssim_build_id", "ssim_debug_set_trace", "ssim_debug_set_trace_ex",
                    "ssim_debug_kernel_name", "ssim_linear_fwd",
                    "ssim_linear_wgrad_parts", "ssim_linear_wgrad", "ssim_mlp3_supported", "ssim_mlp3_fwd",
                    "ssim_mlp3_parts", "ssim_mlp3_partial_floats", "ssim_mlp3_bwd", "ssim_discounted_returns"]


def build_id() -> str:
    """The loaded library's build identity (source + definition hash, __graft_entry__.source_hash)."""
    return lib().ssim_build_id().decode()
