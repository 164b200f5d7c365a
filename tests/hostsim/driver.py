"""Python driver for the TEST-ONLY host build of the engine (hostsim.cpp). Mirrors DeviceEngine's API with
numpy arrays over host memory so the same parity harness drives both."""

from __future__ import annotations

import ctypes as ct
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))

from spark_sched_sim import _abi  # noqa: E402
from spark_sched_sim._abi import SsimConfig, SsimDataset, SsimLayout  # noqa: E402
from spark_sched_sim.data_samplers.tpch_pack import PackedDataset, pack  # noqa: E402
from spark_sched_sim.engine import _ResetSampler, arena_views, make_config  # noqa: E402

# HOSTSIM_SO / HOSTSIM_FLAGS: a variant build (e.g. scripts/hostsim_sanitize.sh: -DSSIM_PROFILE under ASan/UBSan)
SO_PATH = os.environ.get("HOSTSIM_SO") or os.path.join(HERE, "_hostsim.so")
ENV_FLAGS = os.environ.get("HOSTSIM_FLAGS", "").split()
SOURCES = [os.path.join(HERE, "hostsim.cpp")] + [
    os.path.join(REPO, "gym-sparksched_amd", "csrc", f) for f in ("engine.h", "policy.h", "pyset.h", "pcg64.h", "decima.h", "fdlibm.h", "ziggurat.h",
                                                                  "layout.h", "rollout.h")] + [
    os.path.join(REPO, "include", "sparksched.h")]

_lib = None


def build(force: bool = False, extra_flags=()) -> str:
    """Builds _hostsim.so if stale. Safe under parallel test workers (pytest -n): one builder at a time holds
    an flock, and each writes its own temporary before the atomic rename."""
    import fcntl

    def stale():
        newest = max(os.path.getmtime(p) for p in SOURCES)
        return not os.path.exists(SO_PATH) or os.path.getmtime(SO_PATH) < newest

    if not force and not stale():
        return SO_PATH
    with open(SO_PATH + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if force or stale():
            tmp = f"{SO_PATH}.{os.getpid()}.tmp"
            cmd = ["g++", "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
                   "-Wno-unused-function", f"-I{os.path.join(REPO, 'include')}",
                   f"-I{os.path.join(REPO, 'gym-sparksched_amd', 'csrc')}", SOURCES[0], "-o", tmp, *extra_flags, *ENV_FLAGS]
            subprocess.run(cmd, check=True)
            os.replace(tmp, SO_PATH)
    return SO_PATH


def lib():
    global _lib
    if _lib is None:
        L = ct.CDLL(build())
        vp = ct.c_void_p
        L.hs_create.argtypes = [ct.POINTER(SsimConfig), ct.POINTER(SsimDataset), ct.POINTER(vp),
                                ct.POINTER(SsimLayout)]
        L.hs_destroy.argtypes = [vp]
        L.hs_set_resident.argtypes = [vp, ct.c_int]
        for n in ("hs_obs", "hs_reset_arena", "hs_state"):
            getattr(L, n).argtypes = [vp]
            getattr(L, n).restype = ct.POINTER(ct.c_uint8)
        L.hs_reset.argtypes = [vp]
        L.hs_step.argtypes = [vp, vp, vp]
        L.hs_policy.argtypes = [vp, ct.c_int, ct.c_uint64, ct.c_uint64, vp, vp]
        L.hs_rollout.argtypes = [vp, ct.c_int, ct.c_uint64, ct.c_int, vp]
        L.hs_pcg_run.argtypes = [vp, vp, ct.c_int, vp]
        L.hs_job_times.argtypes = [vp, vp, vp, vp]
        L.hs_pyset_trace.argtypes = [vp, ct.c_int, ct.c_int, vp]
        L.hs_decima.argtypes = [vp, ct.c_float, ct.c_float, vp, vp, vp, vp]
        L.hs_reset_sampled.argtypes = [vp, vp, vp, vp]
        L.hs_rollout_ex.argtypes = [vp, ct.c_int, ct.c_uint64, ct.c_int, ct.c_int, vp, vp]
        L.hs_rollout_steps.argtypes = [vp, ct.c_int, ct.c_uint64, vp, ct.c_int, ct.c_int, vp, vp]
        L.hs_seed_words.argtypes = [ct.c_uint64, vp]
        L.hs_std_exponential.argtypes = [vp, ct.c_int, vp]
        L.hs_log1p.argtypes = [vp, ct.c_int, vp]
        _lib = L
    return _lib


class HostEngine:
    def __init__(self, env_cfg: dict, num_envs: int, dataset, job_cap=None, trace_cap: int = 0, resident=False):
        N = env_cfg["num_executors"]
        packed = dataset if isinstance(dataset, PackedDataset) else pack(dataset, N)
        self.packed = packed.with_executors(N)
        self.cfg = make_config(env_cfg, num_envs, self.packed, job_cap, trace_cap)
        self.num_envs = num_envs
        self._arrays = [np.ascontiguousarray(a) for a in self.packed.arrays()]
        self.ds = SsimDataset(self.packed.num_templates, self.packed.num_template_stages,
                              *[a.ctypes.data for a in self._arrays])
        self.layout = SsimLayout()
        h = ct.c_void_p()
        rc = lib().hs_create(ct.byref(self.cfg), ct.byref(self.ds), ct.byref(h), ct.byref(self.layout))
        assert rc == 0
        self.handle = h
        # emulate the device's LDS residency (poisoned working copy of the hot block, the engine's own
        # load_hot / save_hot around every step and rollout)
        lib().hs_set_resident(h, 1 if resident else 0)
        L = self.layout
        self.obs = np.ctypeslib.as_array(lib().hs_obs(h), shape=(L.obs_bytes,))
        self.reset_buf = np.ctypeslib.as_array(lib().hs_reset_arena(h), shape=(L.reset_bytes,))
        self.state = np.ctypeslib.as_array(lib().hs_state(h), shape=(L.state_bytes,))
        self.views = arena_views(self.obs, L)
        self.sampler = _ResetSampler(dict(env_cfg), self.cfg.job_cap, num_envs)
        self.actions = np.zeros((2, num_envs), dtype=np.int32)

    def _rng_words(self, env):
        off = 4096 + env * self.layout.env_bytes + 16
        raw = self.state[off: off + 40]
        w = raw[:32].view(np.uint64)
        u = raw[32:40].view(np.uint32)
        return int(w[0]), int(w[1]), int(w[2]), int(w[3]), int(u[0]), int(u[1])

    def reset(self, seeds=None, options=None, env_ids=None):
        ids = range(self.num_envs) if env_ids is None else list(env_ids)
        self.reset_buf[:] = 0
        for k, e in enumerate(ids):
            if seeds is None:
                s = None
            elif np.isscalar(seeds):
                s = int(seeds) + e
            else:
                s = int(seeds[k])
            opt = options[k] if isinstance(options, (list, tuple)) else options
            self.sampler.fill(self.reset_buf, self.layout.reset_stride, e, s, opt, self._rng_words)
        lib().hs_reset(self.handle)

    def step(self, stage_idx, num_exec):
        si = np.ascontiguousarray(np.asarray(stage_idx, dtype=np.int32).reshape(self.num_envs))
        ne = np.ascontiguousarray(np.asarray(num_exec, dtype=np.int32).reshape(self.num_envs))
        lib().hs_step(self.handle, si.ctypes.data, ne.ctypes.data)

    def policy(self, kind, seed=0, counter=0):
        a = self.actions
        lib().hs_policy(self.handle, kind, seed, counter, a[0].ctypes.data, a[1].ctypes.data)
        return a[0].copy(), a[1].copy()

    def reset_sampled(self, mode, seeds=None, time_limits=None):
        """Device-style reset (job sequences sampled by the engine): mode uint8 [B], seeds uint64 [B]."""
        m = np.ascontiguousarray(np.broadcast_to(np.asarray(mode, dtype=np.uint8), (self.num_envs,)))
        sd = None if seeds is None else np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))
        tl = None if time_limits is None else np.ascontiguousarray(np.asarray(time_limits, dtype=np.float64))
        self._keep = (m, sd, tl)
        lib().hs_reset_sampled(self.handle, m.ctypes.data, None if sd is None else sd.ctypes.data,
                               None if tl is None else tl.ctypes.data)

    def rollout(self, kind, seed, num_steps, action_log=None, flags=0, time_limits=None):
        ptr = action_log.ctypes.data if action_log is not None else None
        tl = None if time_limits is None else np.ascontiguousarray(np.asarray(time_limits, dtype=np.float64))
        self._keep_tl = tl
        rc = lib().hs_rollout_ex(self.handle, kind, seed, num_steps, flags, None if tl is None else tl.ctypes.data,
                                 ptr)
        assert rc == 0, "hostsim rollout: the hot-block policy view disagreed with the obs-arena view" if rc == -5 \
            else f"hostsim rollout rc={rc}"

    def rollout_steps(self, kind, seed, env_steps, max_steps, action_log=None, flags=0, time_limits=None):
        st = np.ascontiguousarray(np.asarray(env_steps, dtype=np.int32).reshape(self.num_envs))
        ptr = action_log.ctypes.data if action_log is not None else None
        tl = None if time_limits is None else np.ascontiguousarray(np.asarray(time_limits, dtype=np.float64))
        self._keep_tl = (st, tl)
        rc = lib().hs_rollout_steps(self.handle, kind, seed, st.ctypes.data, max_steps, flags,
                                    None if tl is None else tl.ctypes.data, ptr)
        assert rc == 0, f"hostsim rollout_steps rc={rc}"

    def host_views(self):
        return self.views

    def decima_features_np(self, num_tasks_scale: float = 200.0, work_scale: float = 1e5) -> dict:
        L = self.layout
        d = {"node_feats": np.zeros((L.num_envs, L.stage_cap, 5), dtype=np.float32),
             "commit_cap": np.zeros((L.num_envs, L.job_cap), dtype=np.int32),
             "edge_mask": np.zeros((L.num_envs, L.edge_cap), dtype=np.int32),
             "depth": np.zeros((L.num_envs,), dtype=np.int32)}
        lib().hs_decima(self.handle, num_tasks_scale, work_scale, *[d[k].ctypes.data for k in
                                                                     ("node_feats", "commit_cap", "edge_mask",
                                                                      "depth")])
        return d

    def job_times_np(self):
        B, J = self.num_envs, self.cfg.job_cap
        ta, tc = np.zeros((B, J)), np.zeros((B, J))
        st = np.zeros((B, J), dtype=np.int32)
        lib().hs_job_times(self.handle, ta.ctypes.data, tc.ctypes.data, st.ctypes.data)
        return ta, tc, st

    def alloc_action_log(self, num_steps):
        return np.zeros((num_steps, self.num_envs, 2), dtype=np.int32)

    @staticmethod
    def to_numpy(x):
        return x

    def snapshot_obs(self):
        return self.obs.copy()

    def close(self):
        if self.handle is not None:
            lib().hs_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["HostEngine", "build", "lib", "_abi"]
