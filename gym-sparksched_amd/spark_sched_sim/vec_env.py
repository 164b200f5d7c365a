"""Batched env: B independent SparkSchedSimEnv instances on one GPU with torch device tensors.

Observations are zero-copy views of the obs arena (padded per env; `num_nodes`/`num_edges`/`num_jobs`
give the valid prefix). They are overwritten by the next step — consumers that keep observations (rollout
storage) copy them. Actions are device int32 tensors `stage_idx[B]`, `num_exec[B]` with the reference's
meaning (spark_sched_sim.py:275-315). Per-env errors are reported in `info["err"]` (SSIM_ERR_* bits);
a frozen env (sticky error) stops advancing until its next reset.
"""

from __future__ import annotations

import numpy as np

from . import _abi
from .engine import DeviceEngine
from .wrappers import StochasticTimeLimitSampler


DEVICE_RESET_MIN_ENVS = 1024  # reset() samples job sequences in the reset kernel from this batch size up


class SparkSchedSimVecEnv:
    """`device_reset`: None = job sequences drawn by the reset kernel (ssim_reset_sampled) when num_envs >=
    DEVICE_RESET_MIN_ENVS, else on the host with numpy (ssim_reset); True / False force one path. Both give
    the same episodes bit for bit (tests/cases.py case_sampled_reset)."""

    def __init__(self, env_cfg: dict, num_envs: int, dataset=None, device="cuda", job_cap=None,
                 mean_time_limit: float | None = None, time_limit_seed: int = 42, trace_cap: int = 0,
                 device_reset: bool | None = None):
        from .env import resolve_dataset

        dataset = resolve_dataset(env_cfg, dataset)
        self.num_envs = num_envs
        self.device_reset = (num_envs >= DEVICE_RESET_MIN_ENVS) if device_reset is None else bool(device_reset)
        self._ever_reset = np.zeros(num_envs, dtype=bool)
        from .metrics import RowStats

        self.stats = RowStats(num_envs)
        self.num_executors = env_cfg["num_executors"]
        self.engine = DeviceEngine(env_cfg, num_envs, dataset, device=device, job_cap=job_cap, trace_cap=trace_cap)
        self.device = self.engine.device
        self.layout = self.engine.layout
        self._limits = (StochasticTimeLimitSampler(mean_time_limit, num_envs, time_limit_seed)
                        if mean_time_limit else None)
        v = self.engine.views
        c = v["counts"]
        self.obs = {
            "nodes": v["nodes"], "edge_links": v["edge_links"], "dag_ptr": v["dag_ptr"],
            "exec_supplies": v["exec_supplies"], "frontier": v["frontier"], "sched_rank": v["sched_rank"],
            "num_nodes": c[:, _abi.OC_NUM_NODES], "num_edges": c[:, _abi.OC_NUM_EDGES],
            "num_jobs": c[:, _abi.OC_NUM_JOBS], "num_committable_execs": c[:, _abi.OC_COMMITTABLE],
            "source_job_idx": c[:, _abi.OC_SOURCE_JOB_IDX], "num_schedulable": c[:, _abi.OC_NUM_SCHEDULABLE],
        }

    def reset(self, seed=None, options=None, env_ids=None):
        """reset(seed, options) of the envs `env_ids` (default all). seed: None (continue each env's stream, or
        fresh entropy for an env never reset), an int base (env i gets base + i) or one seed per listed env.
        options: {"time_limit": t} for all, or a list of per-env option dicts."""
        ids = list(range(self.num_envs)) if env_ids is None else list(env_ids)
        seeds = None if seed is None else ([seed + i for i in ids] if np.isscalar(seed) else list(seed))
        if self._limits is not None:
            options = [{"time_limit": self._limits.sample(i, None if seeds is None else seeds[k])}
                       for k, i in enumerate(ids)]
        self.stats.flush(ids, self.engine)  # finished episodes' completions enter the duration windows
        if self.device_reset:
            self._reset_on_device(ids, seeds, options)
        else:
            self.engine.reset(seeds=seed, options=options, env_ids=env_ids)
        self._ever_reset[ids] = True
        return self.obs, self._info()

    def _reset_on_device(self, ids, seeds, options):
        """One ssim_reset_sampled launch: the reset kernel draws each listed env's job sequence from its
        Generator stream (tpch.py:54-73) and resets it; the other envs are left as they are."""
        from .data_samplers.job_sequence import time_limit_or_inf

        B = self.num_envs
        mode = np.full(B, _abi.SSIM_RESET_SKIP, dtype=np.uint8)
        sd = np.zeros(B, dtype=np.uint64)
        lim = np.full(B, np.inf)
        fresh = np.random.SeedSequence().generate_state(len(ids), dtype=np.uint64) if seeds is None else None
        for k, i in enumerate(ids):
            if seeds is not None:
                mode[i], sd[i] = _abi.SSIM_RESET_SEED, np.uint64(int(seeds[k]) & 0xFFFFFFFFFFFFFFFF)
            elif self._ever_reset[i]:
                mode[i] = _abi.SSIM_RESET_CONTINUE
            else:  # gymnasium seeds a never-reset env from OS entropy
                mode[i], sd[i] = _abi.SSIM_RESET_SEED, fresh[k]
            opt = options[k] if isinstance(options, (list, tuple)) else options
            lim[i] = time_limit_or_inf(opt)
        if np.isinf(lim[mode != _abi.SSIM_RESET_SKIP]).any() and not self.engine.cfg.job_arrival_cap:
            raise ValueError("must either have a limit on job arrivals or time.")
        self.engine.reset_sampled(mode, seeds=sd, time_limits=lim)

    def step(self, stage_idx, num_exec):
        self.engine.step(stage_idx, num_exec)
        c = self.engine.views["counts"]
        term = c[:, _abi.OC_TERMINATED] != 0
        trunc = c[:, _abi.OC_TRUNCATED] != 0
        return self.obs, self.engine.views["reward"], term, trunc, self._info()

    def policy(self, kind: int = _abi.SSIM_POLICY_FAIR, seed: int = 0, counter: int = 0):
        """On-device action driver (fair / FIFO / random); returns (stage_idx, num_exec) tensors."""
        return self.engine.policy(kind, seed, counter)

    def rollout(self, kind: int, seed: int, num_steps: int, action_log=None):
        """`num_steps` device-policy decisions per env fused into one launch."""
        self.engine.rollout(kind, seed, num_steps, action_log)

    def decima_features(self, num_tasks_scale: float = 200.0, work_scale: float = 1e5) -> dict:
        """Decima featurisation of every env's current obs, on device (schedulers/decima/env_wrapper.py:69-161):
        node_feats f32 [B,S,5], commit_cap i32 [B,J] (exec_mask = arange(N) < cap), edge_mask [B,E] (bit l =
        DAG-layer mask l), depth [B]. Padded rows beyond the per-env counts are unspecified."""
        return self.engine.decima_features(num_tasks_scale, work_scale)

    def _info(self):
        c = self.engine.views["counts"]
        err = c[:, _abi.OC_ERR]
        # action_dropped: envs whose step call completed a step a budget launch had preempted
        # (SSIM_ROLLOUT_PREEMPT) instead of applying the given action (SSIM_ERR_PENDING)
        return {"wall_time": self.engine.views["wall_time"], "err": err,
                "action_dropped": (err & _abi.SSIM_ERR_PENDING) != 0,
                "decisions": c[:, _abi.OC_DECISIONS], "num_completed_jobs": c[:, _abi.OC_NUM_COMPLETED]}

    def episode_stats(self):
        """Per-env stats as trainers/rollout_worker.py:122-129 collect_stats (metrics.RowStats): avg job duration
        over the env's last 200 completed jobs across episodes (s), avg number of jobs in the system this episode,
        completed and arrived job counts; float64 [B, 4] on the env's device."""
        import torch

        return torch.from_numpy(self.stats.stats(self.engine)).to(self.device)

    def close(self):
        self.engine.close()
