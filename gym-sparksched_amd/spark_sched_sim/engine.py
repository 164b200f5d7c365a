"""Batched engine: device arenas + the C ABI (include/sparksched.h) behind a small Python surface.

``DeviceEngine`` owns three caller-allocated device arenas (torch uint8 tensors on the GPU): the state
arena (per-env SoA state in HBM), the obs arena (zero-copy observation tensors) and the reset staging
arena, plus the packed dataset blob. Reset-time job sequences are sampled on the host with numpy's
Generator (exactly the reference's reset-time RNG consumption) and uploaded; everything per step runs in
the gfx950 kernels.
"""

from __future__ import annotations

import ctypes as ct
import math

import numpy as np

from . import _abi
from ._abi import SsimConfig, SsimDataset, SsimLayout
from .data_samplers import job_sequence as js
from .data_samplers.tpch_pack import PackedDataset, pack

HEADER_RNG_OFFSET = 16  # EnvHeader: wall, time_limit, then the PCG64 words (layout.h)
PARAMS_RESERVE = 4096   # engine.h kParamsReserve


def make_config(env_cfg: dict, num_envs: int, packed: PackedDataset, job_cap: int | None, trace_cap: int,
                flags: int = 0):
    cap = job_cap if job_cap is not None else env_cfg.get("job_arrival_cap")
    if not cap:
        raise ValueError("job_cap is required when the env config has no job_arrival_cap")
    return SsimConfig(
        num_envs=num_envs,
        num_executors=env_cfg["num_executors"],
        job_cap=int(cap),
        max_stages=packed.max_stages,
        max_edges=packed.max_edges,
        trace_cap=trace_cap,
        moving_delay=float(env_cfg["moving_delay"]),
        warmup_delay=float(env_cfg["warmup_delay"]),
        beta=float(env_cfg.get("beta", 0.0)),
        job_arrival_gap=(1 / env_cfg["job_arrival_rate"]) if env_cfg.get("job_arrival_rate") else 0.0,
        job_arrival_cap=int(env_cfg.get("job_arrival_cap") or 0),
        flags=flags,
    )


def arena_views(arena, L: SsimLayout) -> dict:
    """Typed views over an obs arena (numpy uint8 array or torch uint8 tensor); zero-copy."""
    B, S, E, J, T = L.num_envs, L.stage_cap, L.edge_cap, L.job_cap, L.trace_cap

    def sl(off, nbytes, dtype, shape):
        return arena[off: off + nbytes].view(dtype).reshape(shape)

    if isinstance(arena, np.ndarray):
        f32, i64, i32, u8, f64 = np.float32, np.int64, np.int32, np.uint8, np.float64
    else:
        import torch

        f32, i64, i32, u8, f64 = torch.float32, torch.int64, torch.int32, torch.uint8, torch.float64
    v = {
        "nodes": sl(L.ob_nodes, B * S * 12, f32, (B, S, 3)),
        "edge_links": sl(L.ob_edge_links, B * E * 16, i64, (B, E, 2)),
        "dag_ptr": sl(L.ob_dag_ptr, B * (J + 1) * 4, i32, (B, J + 1)),
        "exec_supplies": sl(L.ob_supplies, B * J * 4, i32, (B, J)),
        "frontier": sl(L.ob_frontier, B * S, u8, (B, S)),
        "sched_rank": sl(L.ob_sched_rank, B * S * 4, i32, (B, S)),
        "counts": sl(L.ob_counts, B * _abi.NUM_COUNTS * 4, i32, (B, _abi.NUM_COUNTS)),
        "reward": sl(L.ob_reward, B * 8, f64, (B,)),
        "wall_time": sl(L.ob_wall_time, B * 8, f64, (B,)),
        "acc": sl(L.ob_acc, B * 8 * _abi.NUM_ACC, i64, (B, _abi.NUM_ACC)),
    }
    if T > 0:
        v["trace"] = arena[L.ob_trace: L.ob_trace + B * T * _abi.TRACE_BYTES].reshape(B, T, _abi.TRACE_BYTES)
    return v


def decode_trace(raw_u8: np.ndarray, n: int):
    """[T, 32] uint8 records -> list of (t, kind, exec, job, stage, seq)."""
    n = min(n, raw_u8.shape[0])
    rec = np.ascontiguousarray(raw_u8[:n])
    t = rec[:, 0:8].copy().view(np.float64).reshape(-1)
    ints = rec[:, 8:32].copy().view(np.int32).reshape(n, 6)
    return [(float(t[i]), int(ints[i, 0]), int(ints[i, 1]), int(ints[i, 2]), int(ints[i, 3]), int(ints[i, 4]))
            for i in range(n)]


def executor_histories(records, num_executors: int) -> list[list[list]]:
    """Executor.history (executor.py:22-44) rebuilt from one episode's trace records: an EXECUTOR_READY
    event attaches the executor to its job (spark_sched_sim.py:445), a TO_COMMON record releases it to the
    common pool (:782). Each history is [[t_release, job_id], ...] starting from [None, -1], the last entry
    open (t = None) -- the renderer's input (spark_sched_sim.py:411, renderer.py:84-95)."""
    hist = [[[None, -1]] for _ in range(num_executors)]
    for t, kind, e, j, _s, _q in records:
        if kind == _abi.TR_READY:
            job = j
        elif kind == _abi.TR_TO_COMMON:
            job = -1
        else:
            continue
        h = hist[e]
        h[-1][0] = t
        h.append([None, job])
    return hist


def obs_dict(v: dict, env: int) -> dict:
    """Reference-format observation of one env (spark_sched_sim.py:393-399) from host (numpy) views."""
    from collections import namedtuple

    c = v["counts"][env]
    n, ne, nj = int(c[_abi.OC_NUM_NODES]), int(c[_abi.OC_NUM_EDGES]), int(c[_abi.OC_NUM_JOBS])
    links = np.array(v["edge_links"][env, :ne], dtype=np.int64).reshape(ne, 2)
    return {
        "dag_batch": GraphInstance(np.array(v["nodes"][env, :n], dtype=np.float32).reshape(n, 3),
                                   np.zeros(ne, dtype=np.int64), links),
        "dag_ptr": [int(x) for x in v["dag_ptr"][env, : nj + 1]],
        "num_committable_execs": int(c[_abi.OC_COMMITTABLE]),
        "source_job_idx": int(c[_abi.OC_SOURCE_JOB_IDX]),
        "exec_supplies": [int(x) for x in v["exec_supplies"][env, :nj]],
    }


def decima_obs_dict(v: dict, dec: dict, env: int, num_executors: int) -> dict:
    """Reference-format Decima observation of one env (schedulers/decima/env_wrapper.py:98-104) from host
    obs views `v` and host copies `dec` of the ssim_decima_features outputs. Edge masks are the bit planes
    of the per-edge mask words: edge_masks[l, e] = bit l of edge_mask[e], l < depth - 1."""
    c = v["counts"][env]
    n, ne, nj = int(c[_abi.OC_NUM_NODES]), int(c[_abi.OC_NUM_EDGES]), int(c[_abi.OC_NUM_JOBS])
    links = np.array(v["edge_links"][env, :ne], dtype=np.int64).reshape(ne, 2)
    caps = np.asarray(dec["commit_cap"][env, :nj], dtype=np.int64)
    depth = int(dec["depth"][env])
    if depth < 0:
        raise ValueError("DAG depth exceeds the 32-level edge-mask word")
    words = np.asarray(dec["edge_mask"][env, :ne]).astype(np.uint32)
    levels = np.arange(max(depth - 1, 0), dtype=np.uint32)
    return {
        "dag_batch": GraphInstance(np.array(dec["node_feats"][env, :n], dtype=np.float32).reshape(n, 5),
                                   np.zeros(ne, dtype=np.int64), links),
        "dag_ptr": [int(x) for x in v["dag_ptr"][env, : nj + 1]],
        "stage_mask": np.array(v["nodes"][env, :n, 2]).astype(bool),
        "exec_mask": np.arange(num_executors)[None, :] < caps[:, None],
        "edge_masks": ((words[None, :] >> levels[:, None]) & 1).astype(bool),
    }


try:  # gymnasium is optional; mirror its GraphInstance when absent
    from gymnasium.spaces import GraphInstance  # type: ignore
except Exception:  # pragma: no cover - gymnasium not installed in this image
    from collections import namedtuple

    GraphInstance = namedtuple("GraphInstance", ["nodes", "edges", "edge_links"])


class _ResetSampler:
    """Per-env host RNGs + reset-record packing (gymnasium seeding semantics, spark_sched_sim.py:130)."""

    def __init__(self, env_cfg: dict, job_cap: int, num_envs: int):
        self.env_cfg = env_cfg
        self.job_cap = job_cap
        self.rngs = [None] * num_envs
        self.arrival_cap = [env_cfg.get("job_arrival_cap")] * num_envs  # env-level cap, overwritten by reset

    def fill(self, buf: np.ndarray, stride: int, env: int, seed, options, rng_words_fn):
        limit = js.time_limit_or_inf(options)
        if limit == math.inf and not self.arrival_cap[env]:
            raise ValueError("must either have a limit on job arrivals or time.")
        if seed is not None:
            self.rngs[env] = js.make_rng(seed)
        elif self.rngs[env] is None:
            self.rngs[env] = js.make_rng(None)
        else:  # continue the env's stream where the device left it
            words = rng_words_fn(env)
            st = self.rngs[env].bit_generator.state
            st["state"]["state"] = (int(words[0]) << 64) | int(words[1])
            st["state"]["inc"] = (int(words[2]) << 64) | int(words[3])
            st["has_uint32"], st["uinteger"] = int(words[4]), int(words[5])
            self.rngs[env].bit_generator.state = st
        rng = self.rngs[env]
        tpl, arr = js.sample_jobs(rng, self.env_cfg.get("job_arrival_cap"), self.env_cfg["job_arrival_rate"], limit)
        if len(tpl) == 0 or arr[0] != 0:
            raise AssertionError("first job must arrive at t=0")
        self.arrival_cap[env] = len(tpl)
        js.write_reset_record(buf, env * stride, self.job_cap, tpl, arr, js.rng_words(rng), limit)
        return len(tpl)


class DeviceEngine:
    """B independent envs on one GPU. All tensors live on `device`; nothing is copied per step."""

    def __init__(self, env_cfg: dict, num_envs: int, dataset, device="cuda", job_cap=None, trace_cap: int = 0,
                 config_flags: int = 0):
        """config_flags: ssim_config.flags (SSIM_CFG_FORCE_HBM: hot blocks in HBM whatever their size, test use)."""
        import torch

        from . import native

        self.torch = torch
        self.device = torch.device(device)
        self.env_cfg = dict(env_cfg)
        N = env_cfg["num_executors"]
        packed = dataset if isinstance(dataset, PackedDataset) else pack(dataset, N)
        self.packed = packed.with_executors(N)
        self.cfg = make_config(env_cfg, num_envs, self.packed, job_cap, trace_cap, config_flags)
        self.num_envs = num_envs
        # the library sizes LDS residency from the CURRENT device's compute units (ssim_layout.chip_cus): make it this
        # engine's device for the layout query and ssim_create
        import contextlib

        on_dev = torch.cuda.device(self.device) if self.device.type == "cuda" else contextlib.nullcontext()
        L = SsimLayout()
        with on_dev:
            native.check(native.lib().ssim_layout_for(ct.byref(self.cfg), ct.byref(L)), "ssim_layout_for")
        self.layout = L
        # dataset blob
        arrays = self.packed.arrays()
        offs, total = [], 0
        for a in arrays:
            offs.append(total)
            total += (a.nbytes + 255) // 256 * 256
        blob = np.zeros(total, dtype=np.uint8)
        for a, o in zip(arrays, offs):
            blob[o: o + a.nbytes] = np.frombuffer(a.tobytes(), dtype=np.uint8)
        self.dataset_dev = torch.from_numpy(blob).to(self.device)
        base = self.dataset_dev.data_ptr()
        self.ds = SsimDataset(self.packed.num_templates, self.packed.num_template_stages,
                              *[base + o for o in offs])
        self.state = torch.zeros(L.state_bytes, dtype=torch.uint8, device=self.device)
        self.obs = torch.zeros(L.obs_bytes, dtype=torch.uint8, device=self.device)
        self.reset_dev = torch.zeros(L.reset_bytes, dtype=torch.uint8, device=self.device)
        self.reset_host = np.zeros(L.reset_bytes, dtype=np.uint8)
        self.actions = torch.zeros((2, num_envs), dtype=torch.int32, device=self.device)
        h = ct.c_void_p()
        with on_dev:
            native.check(native.lib().ssim_create(ct.byref(self.cfg), ct.byref(self.ds), self.state.data_ptr(),
                                                  self.obs.data_ptr(), self.reset_dev.data_ptr(), ct.byref(h)),
                         "ssim_create")
        self.handle = h
        self.views = arena_views(self.obs, L)
        self.sampler = _ResetSampler(self.env_cfg, self.cfg.job_cap, num_envs)
        self._native = native

    def _stream(self):
        return ct.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _rng_words(self, env: int):
        off = PARAMS_RESERVE + env * self.layout.env_bytes + HEADER_RNG_OFFSET
        raw = self.state[off: off + 40].cpu().numpy()
        w = raw[:32].view(np.uint64)
        u = raw[32:40].view(np.uint32)
        return int(w[0]), int(w[1]), int(w[2]), int(w[3]), int(u[0]), int(u[1])

    def reset(self, seeds=None, options=None, env_ids=None):
        """Reset `env_ids` (default: all). seeds: int base, sequence of per-env seeds, or None."""
        ids = range(self.num_envs) if env_ids is None else list(env_ids)
        buf = self.reset_host
        stride = self.layout.reset_stride
        buf[:] = 0
        for k, e in enumerate(ids):
            if seeds is None:
                s = None
            elif np.isscalar(seeds):
                s = int(seeds) + e
            else:
                s = int(seeds[k])
            opt = options[k] if isinstance(options, (list, tuple)) else options
            self.sampler.fill(buf, stride, e, s, opt, self._rng_words)
        self.reset_dev.copy_(self.torch.from_numpy(buf), non_blocking=False)
        self._native.check(self._native.lib().ssim_reset(self.handle, self._stream()), "ssim_reset")

    def step(self, stage_idx, num_exec):
        """stage_idx/num_exec: device int32 tensors [num_envs] (or anything torch can turn into one)."""
        t = self.torch
        si = t.as_tensor(stage_idx, dtype=t.int32, device=self.device).contiguous()
        ne = t.as_tensor(num_exec, dtype=t.int32, device=self.device).contiguous()
        self._keep = (si, ne)
        self._native.check(self._native.lib().ssim_step(self.handle, si.data_ptr(), ne.data_ptr(), self._stream()),
                           "ssim_step")

    def policy(self, kind: int, seed: int = 0, counter: int = 0):
        a = self.actions
        self._native.check(self._native.lib().ssim_policy(self.handle, kind, seed, counter, a[0].data_ptr(),
                                                          a[1].data_ptr(), self._stream()), "ssim_policy")
        return a[0], a[1]

    def reset_sampled(self, mode, seeds=None, time_limits=None):
        """Device-side reset (ssim_reset_sampled): job sequences sampled by the kernel from each env's
        Generator stream. mode: uint8 [B] of _abi.SSIM_RESET_* (or one value for all envs); seeds: uint64 [B]
        for SSIM_RESET_SEED envs; time_limits: float64 [B] (None = +inf)."""
        t, B = self.torch, self.num_envs
        if isinstance(mode, t.Tensor):  # device tensors are used in place (no host round trip)
            m = mode.to(device=self.device, dtype=t.uint8).contiguous()
        else:
            m = t.as_tensor(np.broadcast_to(np.asarray(mode, dtype=np.uint8), (B,)).copy(), device=self.device)
        sd = None
        if isinstance(seeds, t.Tensor):
            sd = seeds.to(device=self.device, dtype=t.int64).contiguous()
        elif seeds is not None:
            sd = t.as_tensor(np.asarray(seeds, dtype=np.uint64).view(np.int64).reshape(B), device=self.device)
        tl = None
        if isinstance(time_limits, t.Tensor):
            tl = time_limits.to(device=self.device, dtype=t.float64).contiguous()
        elif time_limits is not None:
            tl = t.as_tensor(np.asarray(time_limits, dtype=np.float64).reshape(B), device=self.device)
        self._keep = (m, sd, tl)
        self._native.check(self._native.lib().ssim_reset_sampled(
            self.handle, m.data_ptr(), None if sd is None else sd.data_ptr(), None if tl is None else tl.data_ptr(),
            self._stream()), "ssim_reset_sampled")

    def rollout(self, kind: int, seed: int, num_steps: int, action_log=None, flags: int = 0, time_limits=None):
        """`num_steps` fused policy+step launches' worth of decisions in ONE kernel launch. flags:
        _abi.SSIM_ROLLOUT_AUTORESET resets finished episodes in place (limits from `time_limits`)."""
        ptr = action_log.data_ptr() if action_log is not None else None
        tl = None
        if time_limits is not None:
            tl = self.torch.as_tensor(np.asarray(time_limits, dtype=np.float64).reshape(self.num_envs),
                                      device=self.device) if not hasattr(time_limits, "data_ptr") else time_limits
        self._keep_tl = tl
        self._native.check(self._native.lib().ssim_rollout_ex(
            self.handle, kind, seed, num_steps, flags, None if tl is None else tl.data_ptr(), ptr, self._stream()),
            "ssim_rollout")

    def rollout_budget(self, kind: int, seed: int, max_steps: int, total_decisions: int, action_log=None,
                       flags: int = 0, time_limits=None):
        """Work-conserving rollout (ssim_rollout_budget): `total_decisions` decisions shared by all envs, each
        env at most `max_steps`; each env's decisions equal those of `rollout`, only their number differs."""
        ptr = action_log.data_ptr() if action_log is not None else None
        tl = None
        if time_limits is not None:
            tl = self.torch.as_tensor(np.asarray(time_limits, dtype=np.float64).reshape(self.num_envs),
                                      device=self.device) if not hasattr(time_limits, "data_ptr") else time_limits
        self._keep_tl = tl
        self._native.check(self._native.lib().ssim_rollout_budget(
            self.handle, kind, seed, max_steps, total_decisions, flags, None if tl is None else tl.data_ptr(), ptr,
            self._stream()), "ssim_rollout_budget")

    def rollout_steps(self, kind: int, seed: int, env_steps, max_steps: int, action_log=None, flags: int = 0,
                      time_limits=None):
        """ssim_rollout_steps: env i takes min(env_steps[i], max_steps) fused policy+step decisions in one
        launch (env_steps: int32 [num_envs], host or device)."""
        t = self.torch
        st = t.as_tensor(np.asarray(env_steps, dtype=np.int32).reshape(self.num_envs), device=self.device) \
            if not isinstance(env_steps, t.Tensor) else env_steps.to(device=self.device, dtype=t.int32).contiguous()
        ptr = action_log.data_ptr() if action_log is not None else None
        tl = None
        if time_limits is not None:
            tl = t.as_tensor(np.asarray(time_limits, dtype=np.float64).reshape(self.num_envs),
                             device=self.device) if not hasattr(time_limits, "data_ptr") else time_limits
        self._keep_tl = (st, tl)
        self._native.check(self._native.lib().ssim_rollout_steps(
            self.handle, kind, seed, st.data_ptr(), max_steps, flags, None if tl is None else tl.data_ptr(), ptr,
            self._stream()), "ssim_rollout_steps")

    def host_views(self) -> dict:
        return arena_views(self.obs.cpu().numpy(), self.layout)

    def job_times(self):
        t = self.torch
        B, J = self.num_envs, self.cfg.job_cap
        ta = t.empty((B, J), dtype=t.float64, device=self.device)
        tc = t.empty((B, J), dtype=t.float64, device=self.device)
        st = t.empty((B, J), dtype=t.int32, device=self.device)
        self._native.check(self._native.lib().ssim_job_times(self.handle, ta.data_ptr(), tc.data_ptr(), st.data_ptr(),
                                                             self._stream()), "ssim_job_times")
        return ta, tc, st

    def decima_features(self, num_tasks_scale: float = 200.0, work_scale: float = 1e5) -> dict:
        """Decima featurisation of the current obs on device (ssim_decima_features); device tensors,
        overwritten by the next call: node_feats f32 [B,S,5], commit_cap i32 [B,J], edge_mask i32 [B,E]
        (uint32 bit planes stored as int32), depth i32 [B]."""
        t = self.torch
        L = self.layout
        if getattr(self, "_dec", None) is None:
            self._dec = {
                "node_feats": t.zeros((L.num_envs, L.stage_cap, 5), dtype=t.float32, device=self.device),
                "commit_cap": t.zeros((L.num_envs, L.job_cap), dtype=t.int32, device=self.device),
                "edge_mask": t.zeros((L.num_envs, L.edge_cap), dtype=t.int32, device=self.device),
                "depth": t.zeros((L.num_envs,), dtype=t.int32, device=self.device),
            }
        d = self._dec
        self._native.check(self._native.lib().ssim_decima_features(
            self.handle, float(num_tasks_scale), float(work_scale), d["node_feats"].data_ptr(),
            d["commit_cap"].data_ptr(), d["edge_mask"].data_ptr(), d["depth"].data_ptr(), self._stream()),
            "ssim_decima_features")
        return d

    def decima_workspace(self):
        """The persistent Decima rollout's per-env workspace (ssim_decima_workspace_bytes), allocated once."""
        if getattr(self, "_dws", None) is None:
            n = int(self._native.lib().ssim_decima_workspace_bytes(self.handle))
            if n <= 0:
                self._native.check(-1, "ssim_decima_workspace_bytes")
            self._dws = self.torch.zeros(n, dtype=self.torch.uint8, device=self.device)
        return self._dws

    def decima_rollout(self, params, seed: int, counter: int, max_steps: int, total_decisions: int = 0,
                       flags: int = 0, time_limits=None, samples=None, action_log=None,
                       num_tasks_scale: float = 200.0, work_scale: float = 1e5):
        """ssim_decima_rollout: Decima features + fused policy + step per env and decision, in ONE launch.
        params: DecimaScheduler.packed_params() (fp32 device tensor). samples: a DecimaSampleArena (or None).
        flags: 0 = collect until each env's episode ends; _abi.SSIM_ROLLOUT_AUTORESET / PREEMPT (with
        total_decisions) / WARMUP as ssim_rollout_budget."""
        ws = self.decima_workspace()
        tl = None
        if time_limits is not None:
            tl = self.torch.as_tensor(np.asarray(time_limits, dtype=np.float64).reshape(self.num_envs),
                                      device=self.device) if not hasattr(time_limits, "data_ptr") else time_limits
        st = samples.struct() if samples is not None else None
        self._keep_dr = (params, tl, st)
        self._native.check(self._native.lib().ssim_decima_rollout(
            self.handle, params.data_ptr(), params.numel(), float(num_tasks_scale), float(work_scale),
            int(seed) & (2**64 - 1), int(counter) & (2**64 - 1), int(max_steps), int(total_decisions), int(flags),
            None if tl is None else tl.data_ptr(), ws.data_ptr(), ws.numel(),
            None if st is None else ct.byref(st), None if action_log is None else action_log.data_ptr(),
            self._stream()), "ssim_decima_rollout")

    def decima_features_np(self, num_tasks_scale: float = 200.0, work_scale: float = 1e5) -> dict:
        return {k: x.cpu().numpy() for k, x in self.decima_features(num_tasks_scale, work_scale).items()}

    def job_times_np(self):
        return tuple(x.cpu().numpy() for x in self.job_times())

    def alloc_action_log(self, num_steps: int):
        return self.torch.zeros((num_steps, self.num_envs, 2), dtype=self.torch.int32, device=self.device)

    @staticmethod
    def to_numpy(x):
        return x.cpu().numpy()

    def snapshot_obs(self) -> np.ndarray:
        return self.obs.cpu().numpy().copy()

    def close(self):
        if self.handle is not None:
            self._native.lib().ssim_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
