"""PPO on GPU rollouts (trainers/ppo.py:45-138 on top of trainers/trainer.py:28-190).

The reference runs `num_sequences x num_rollouts` rollout processes and ONE learner: the learner scatters the
state dict, gathers every worker's RolloutBuffer, computes returns and baselines over all of them and runs the
PPO epochs (trainer.py:85-162, ppo.py:51-103). Here, with one process per GPU:
  1. the num_sequences x num_rollouts rows (row = sequence s, rollout r; s-major as trainer.py:268-270) are split
     into contiguous blocks over the ranks; each rank's block is one vector env on its GPU, collected by
     RolloutCollector (device-side reset with the row's seed, Decima forward per decision, ssim_step). Actions
     are drawn from a counter-based stream keyed by the GLOBAL row, so a row's trajectory does not depend on
     the world size;
  2. each rank orders its samples row-major (row, decision) and the blocks are gathered over RCCL to the
     learner (rank 0), which then holds exactly the batch a 1-rank run holds, in the same order;
  3. the learner computes returns (ReturnsCalculator) and baselines (Baseline over all rows of a sequence),
     advantages = returns - baselines, and runs the PPO epochs (shuffled minibatches, CLIP loss with the entropy
     bonus, target-KL early stop, TrainableScheduler.update_parameters);
  4. the learner broadcasts the updated parameters (the reference's state-dict scatter); episode statistics are
     all-gathered (rollout_worker.py:122-129).
Seeds follow trainer.py:258-270 / rollout_worker.py:118-120: row (s, r) uses seed + s + num_sequences *
iteration. A multi-rank run therefore takes the same iteration as a 1-rank run of the same global config
(tests/test_trainers.py checks the parameters bit for bit on 2 gloo ranks).
"""

from __future__ import annotations

from typing import Any

import math

import numpy as np
import torch

from ..distributed import all_gather_var, gather_var, split_rows
from ..schedulers.decima import DagBatch, DecimaScheduler, cat_batches, learner_counts, minibatch_plans, select_envs
from .returns import Baseline, ReturnsCalculator
from .rollouts import AsyncRolloutCollector, DeviceRolloutCollector, RolloutCollector

EPS = 1e-8  # ppo.py:13
_BATCH_TENSORS = ["x", "edge_index", "edge_bits", "env_levels", "ptr", "node_dag", "node_env", "dag_env", "obs_ptr",
                  "stage_mask", "exec_cap", "num_stage_acts", "num_nodes", "num_edges"]


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def gather_batches(b: DagBatch, world: int, rank: int = 0, dst: int = 0) -> DagBatch | None:
    """Every rank's DagBatch concatenated in rank order on rank `dst` (a gather of each field, then cat_batches);
    None on the other ranks, which do not train (the single learner of trainer.py:126-131)."""
    if world <= 1:
        return b
    parts = {}
    for name in _BATCH_TENSORS:
        t = getattr(b, name)
        if name == "edge_index":
            g = gather_var(t.t().contiguous(), world, rank, dst)
            parts[name] = None if g is None else [p.t() for p in g]
        elif name in ("ptr", "obs_ptr"):  # drop the leading 0 for the variable gather, restore per rank
            g = gather_var(t[1:].contiguous(), world, rank, dst)
            parts[name] = None if g is None else [torch.cat([torch.zeros(1, dtype=p.dtype, device=p.device), p])
                                                  for p in g]
        else:
            parts[name] = gather_var(t, world, rank, dst)
    scal = torch.tensor([b.max_levels, b.num_envs, b.max_nodes], dtype=torch.int64, device=b.x.device)
    scals = gather_var(scal[None, :], world, rank, dst)
    if rank != dst:
        return None
    bs = []
    for k in range(world):
        ml, ne, mn = (int(v) for v in scals[k][0].tolist())
        bs.append(DagBatch(**{n: parts[n][k] for n in _BATCH_TENSORS}, max_levels=ml, num_envs=ne, max_nodes=mn))
    return cat_batches(bs)


class PPO:
    def __init__(self, agent_cfg: dict, env_cfg: dict, train_cfg: dict, engine_factory=None, dataset=None,
                 device=None):
        d = _dist()
        self.rank = d.get_rank() if d else 0
        self.world = d.get_world_size() if d else 1
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.seed = int(train_cfg["seed"])
        torch.manual_seed(self.seed)  # identical initial policy on every rank (trainer.py:33)
        self.num_sequences = int(train_cfg["num_sequences"])  # global, as in the reference config
        self.num_rollouts = int(train_cfg["num_rollouts"])
        self.num_iterations = int(train_cfg.get("num_iterations", 1))
        self.entropy_coeff = float(train_cfg.get("entropy_coeff", 0.0))
        self.clip_range = float(train_cfg.get("clip_range", 0.2))
        self.target_kl = train_cfg.get("target_kl", 0.01)
        self.num_epochs = int(train_cfg.get("num_epochs", 10))
        self.num_batches = int(train_cfg.get("num_batches", 3))
        assert ("reward_buff_cap" in train_cfg) ^ ("beta_discount" in train_cfg), \
            "must provide exactly one of `reward_buff_cap` and `beta_discount` in config"
        env_cfg = dict(env_cfg)
        if "beta_discount" in train_cfg:
            env_cfg["beta"] = float(train_cfg["beta_discount"])
            self.return_calc = ReturnsCalculator(beta=float(train_cfg["beta_discount"]))
        else:
            self.return_calc = ReturnsCalculator(buff_cap=int(train_cfg["reward_buff_cap"]))
        self.env_cfg = env_cfg
        self.mean_time_limit = env_cfg.get("mean_time_limit")
        self.rows = self.num_sequences * self.num_rollouts
        if self.rows < self.world:
            raise ValueError(f"{self.rows} rollout rows cannot be split over {self.world} ranks")
        self.row_lo, self.row_hi = split_rows(self.rows, self.world, self.rank)
        self.baseline = Baseline(self.num_sequences, self.num_rollouts)  # learner side, over all rows
        kw = {k: v for k, v in agent_cfg.items() if k != "agent_cls"}
        self.scheduler = DecimaScheduler(env_cfg["num_executors"], opt_cls=train_cfg.get("opt_cls", "Adam"),
                                         opt_kwargs=train_cfg.get("opt_kwargs"),
                                         max_grad_norm=train_cfg.get("max_grad_norm"), **kw).to(self.device)
        B = self.row_hi - self.row_lo
        if dataset is None:
            from ..env import resolve_dataset

            dataset = resolve_dataset(env_cfg)  # the config's data sampler (TPC-H, warns if it falls back)
        sim_cfg = {k: v for k, v in env_cfg.items() if k not in ("mean_time_limit", "dataset")}
        if engine_factory is None:
            from ..engine import DeviceEngine

            def engine_factory(cfg, n, ds):
                return DeviceEngine(cfg, n, ds, device=self.device)
        self.engine = engine_factory(sim_cfg, B, dataset)
        self.rollout_duration = train_cfg.get("rollout_duration")  # trainer.py:63, async workers :277-279
        rseed = self.seed * 7919
        if self.rollout_duration:
            base = [self.seed + r // self.num_rollouts for r in range(self.row_lo, self.row_hi)]
            self.collector = AsyncRolloutCollector(self.engine, self.scheduler, self.rollout_duration, base,
                                                   self.num_sequences, mean_time_limit=self.mean_time_limit,
                                                   seed=rseed, row_offset=self.row_lo)
        else:
            self.collector = RolloutCollector(self.engine, self.scheduler, seed=rseed, row_offset=self.row_lo)
            # device engines: the whole collection in one persistent launch (same actions, csrc/decima_rollout.h);
            # train_cfg["lockstep_rollouts"] keeps the per-decision collector
            if (self.collector.on_device and self.collector.fused and hasattr(self.engine, "decima_rollout")
                    and not train_cfg.get("lockstep_rollouts", False)):
                self.collector = DeviceRolloutCollector(self.engine, self.scheduler, seed=rseed,
                                                        row_offset=self.row_lo)
        self.gen = torch.Generator(device=self.device).manual_seed(rseed)  # learner's minibatch shuffling
        self.perm_fn = None  # (tests) epoch -> permutation of the samples, instead of the generator's
        self.time_limit_rngs = None
        if self.mean_time_limit:
            # one StochasticTimeLimit per row, seeded like the reference wrapper (seed=42, reseeded by reset seed)
            self.time_limit_rngs = [np.random.RandomState(42) for _ in range(B)]
        self.reset_count = 0

    # ------------------------------------------------------------------ rollouts
    def _seeds(self) -> list[int]:
        """rollout_worker.py:118-120 with trainer.py:258-270's base seeds: sequence s = row // num_rollouts gets
        seed + s + num_sequences * reset_count, shared by its num_rollouts rows (this rank's rows only)."""
        return [self.seed + r // self.num_rollouts + self.num_sequences * self.reset_count
                for r in range(self.row_lo, self.row_hi)]

    def _time_limits(self, seeds):
        if not self.time_limit_rngs:
            return None
        lim = []
        for i, s in enumerate(seeds):
            if s:
                self.time_limit_rngs[i] = np.random.RandomState(s)
            lim.append(float(self.time_limit_rngs[i].exponential(self.mean_time_limit)))
        return np.array(lim)

    def collect(self):
        self.scheduler.eval()
        if self.rollout_duration:
            return self.collector.collect()
        seeds = self._seeds()
        buf = self.collector.collect(seeds, self._time_limits(seeds))
        self.reset_count += 1
        return buf

    # ------------------------------------------------------------------ learning
    def gather_rollouts(self, buf):
        """This rank's buffer in row-major (row, decision) order, gathered over all ranks to one batch in global
        row order: (times [R, T+1], rewards [R, T], lengths [R], obs DagBatch, actions). times / rewards / lengths
        are all-gathered (every rank keeps the differential-return window in step); the observations and actions
        go to the learner (rank 0) only, None elsewhere."""
        times, rewards, lengths, sample = buf.trajectories()
        obs, acts = buf.samples()
        if not getattr(buf, "row_major", False):
            canon = sample[sample >= 0]  # row-major: row r's decisions in order, rows ascending
            obs = select_envs(obs, canon)
            acts = {k: v[canon] for k, v in acts.items()}
        if self.world > 1:
            T = torch.tensor([rewards.shape[1]], dtype=torch.int64, device=rewards.device)
            Tm = int(max(int(t.item()) for t in all_gather_var(T, self.world)))
            pad = Tm - rewards.shape[1]
            if pad:
                times = torch.cat([times, torch.zeros((times.shape[0], pad), dtype=times.dtype,
                                                      device=times.device)], dim=1)
                rewards = torch.cat([rewards, torch.zeros((rewards.shape[0], pad), dtype=rewards.dtype,
                                                          device=rewards.device)], dim=1)
            times = torch.cat(all_gather_var(times, self.world))
            rewards = torch.cat(all_gather_var(rewards, self.world))
            lengths = torch.cat(all_gather_var(lengths, self.world))
            obs = gather_batches(obs, self.world, self.rank, 0)
            g = {k: gather_var(v, self.world, self.rank, 0) for k, v in acts.items()}
            acts = None if self.rank != 0 else {k: torch.cat(v) for k, v in g.items()}
        return times, rewards, lengths, obs, acts

    def train_on_rollouts(self, buf) -> dict[str, Any]:
        times, rewards, lengths, obs, acts = self.gather_rollouts(buf)
        info = None
        if self.rank == 0:  # the learner (trainer.py:126-131, ppo.py:51-71)
            returns = self.return_calc(times, rewards, lengths)
            base = self.baseline(times[:, :-1], returns, lengths)
            valid = torch.arange(rewards.shape[1], device=rewards.device)[None, :] < lengths[:, None]
            advg = (returns - base)[valid]  # row-major = the gathered sample order
            info = self._train(obs, acts, advg.float())
        elif isinstance(self.return_calc.buff_cap, int) and self.return_calc.buff_cap:
            self.return_calc(times, rewards, lengths)  # keep the differential-return window in step
        self._broadcast_parameters()
        return self._broadcast_info(info)

    def _broadcast_parameters(self):
        """The learner's parameters to every rank (trainer.py:110-111's state-dict scatter)."""
        d = _dist()
        if d is None or self.world == 1:
            return
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1) for p in self.scheduler.parameters()])
            d.broadcast(flat, src=0)
            o = 0
            for p in self.scheduler.parameters():
                k = p.numel()
                p.copy_(flat[o: o + k].view_as(p))
                o += k

    def _broadcast_info(self, info):
        d = _dist()
        if d is None or self.world == 1:
            return info
        t = torch.zeros(4, dtype=torch.float64, device=self.device)
        if info is not None:
            t[:] = torch.tensor([info["policy loss"], info["entropy"], info["approx kl div"], info["samples"]],
                                dtype=torch.float64)
        d.broadcast(t, src=0)
        v = t.tolist()
        return {"policy loss": v[0], "entropy": v[1], "approx kl div": v[2], "samples": int(v[3])}

    def _train(self, obs, acts, advg) -> dict[str, Any]:
        """ppo.py:51-103. Host syncs: one per epoch for the sizes of all its minibatches (the index sets of the
        compact learner path, minibatch_plans), and one per minibatch for the approx-KL early stop, whose value
        decides whether the update runs (ppo.py:88-91); the losses are summed on the device."""
        n = obs.num_envs
        bs = n // self.num_batches + 1  # ppo.py:69
        pol_losses, ent_losses, kls = [], [], []
        cont = True
        self.scheduler.train()
        counts = learner_counts(obs)
        for epoch in range(self.num_epochs):
            if not cont:
                break
            if self.perm_fn is not None:
                perm = self.perm_fn(epoch).to(advg.device)
            else:
                perm = torch.randperm(n, device=advg.device, generator=self.gen)  # DataLoader(shuffle=True)
            groups = [perm[k: k + bs] for k in range(0, n, bs)]
            plans = minibatch_plans(obs, counts, groups)
            for idx, (sizes, plan) in zip(groups, plans):
                loss, info = self._loss(select_envs(obs, idx, sizes), {a: t[idx] for a, t in acts.items()}, advg[idx],
                                        plan)
                pol_losses.append(info["policy_loss"])
                ent_losses.append(info["entropy_loss"])
                # the gradients (and the clipped total norm) are computed before the approx-KL value is read, so the
                # forward and backward launches go out in one run and the minibatch makes ONE host sync; the update
                # itself still happens only when the KL check passes (ppo.py:88-91, then scheduler.py:34-53)
                norm = self._backward(loss)
                kl, total = torch.stack([info["approx_kl_div"].float(), norm.float()]).tolist()
                kls.append(kl)
                if self.target_kl is not None and kl > 1.5 * self.target_kl:
                    self.scheduler.optim.zero_grad()
                    cont = False  # ppo.py:88-91
                    break
                self._clip(norm, total)
                self._step()
        pl = torch.stack(pol_losses).mean().item()
        el = torch.stack(ent_losses).mean().item()
        return {"policy loss": abs(pl), "entropy": abs(el), "approx kl div": abs(float(np.mean(kls))), "samples": n}

    def _loss(self, obs, acts, advg, plan=None):
        """CLIP loss (ppo.py:105-138). The statistics stay device tensors (no host sync here)."""
        ev = self.scheduler.evaluate_actions(obs, acts["stage_idx"], acts["job_idx"], acts["exec_idx"], plan=plan)
        a = (advg - advg.mean()) / (advg.std() + EPS)  # ppo.py:118-119
        log_ratio = ev["lgprobs"] - acts["lgprob"]
        ratio = log_ratio.exp()
        pl = -torch.min(a * ratio, a * torch.clamp(ratio, 1 - self.clip_range, 1 + self.clip_range)).mean()
        el = -ev["entropies"].mean()
        loss = pl + self.entropy_coeff * el
        with torch.no_grad():
            kl = ((ratio - 1) - log_ratio).mean()
        return loss, {"policy_loss": pl.detach(), "entropy_loss": el.detach(), "approx_kl_div": kl}

    def _update(self, loss):
        """TrainableScheduler.update_parameters (scheduler.py:34-53)."""
        norm = self._backward(loss)
        self._clip(norm, float(norm))
        self._step()

    def _backward(self, loss) -> torch.Tensor:
        """scheduler.py:34-53 up to the clip: backward, then the gradients' total norm (device tensor, no sync), so the
        caller can read it together with the approx-KL value in one host sync. The gradients are not modified here."""
        s = self.scheduler
        loss.backward()
        params = [p for p in s.parameters() if p.grad is not None]
        if not s.max_grad_norm or not params:
            return loss.new_zeros(())
        return torch.nn.utils.get_total_norm([p.grad for p in params])

    def _clip(self, norm: torch.Tensor, total: float) -> None:
        """scheduler.py:44-48: with max_grad_norm set, clip_grad_norm_(error_if_nonfinite=True) — a non-finite total norm
        raises BEFORE any gradient is scaled; without it the reference steps unclipped, whatever the gradients hold."""
        s = self.scheduler
        if not s.max_grad_norm:
            return
        if not math.isfinite(total):
            raise RuntimeError(f"The total norm of order 2.0 for gradients from `parameters` is non-finite, so it "
                               f"cannot be clipped ({total})")
        params = [p for p in s.parameters() if p.grad is not None]
        torch.nn.utils.clip_grads_with_norm_(params, s.max_grad_norm, norm)

    def _step(self):
        s = self.scheduler
        s.optim.step()
        s.optim.zero_grad()

    # ------------------------------------------------------------------ statistics
    def episode_stats(self) -> torch.Tensor:
        """rollout_worker.py:122-129 per row: [avg job duration (s), avg #jobs, completed, arrived], gathered
        from every rank (RCCL all_gather) in global row order: [rows, 4]. avg job duration is the mean over
        the last 200 completed jobs of the row's env across its episodes (spark_sched_sim.py:83,243-245,697;
        the collector keeps the window, RolloutCollector.duration_window)."""
        mine = self.collector.row_stats()
        if self.world == 1:
            return mine
        return torch.cat(all_gather_var(mine, self.world))

    def train(self, num_iterations: int | None = None, log=print) -> list[dict]:
        hist = []
        for i in range(num_iterations or self.num_iterations):
            buf = self.collect()
            stats = self.episode_stats()
            learn = self.train_on_rollouts(buf)
            # Trainer.train (trainer.py:135-137): the return calculator's moving average if it has one
            avg_jobs = self.return_calc.avg_num_jobs or float(stats[:, 1].mean())
            rec = {"iteration": i, "avg_num_jobs": avg_jobs, "avg_job_duration": float(stats[:, 0].mean()),
                   "completed_jobs": float(stats[:, 2].mean()), **learn}
            hist.append(rec)
            if self.rank == 0 and log is not None:
                log(f"Iteration {i + 1} complete. Avg. # jobs: {avg_jobs:.3f}")
        return hist


# config/decima_tpch.yaml restated (trainer 1-62, agent 64-78, env 80-87); `device` and logging keys dropped
DECIMA_TPCH = {
    "trainer": {"trainer_cls": "PPO", "num_iterations": 500, "num_sequences": 4, "num_rollouts": 4, "seed": 42,
                "num_epochs": 3, "num_batches": 10, "clip_range": 0.2, "target_kl": 0.01, "entropy_coeff": 0.04,
                "beta_discount": 5.0e-3, "opt_cls": "Adam", "opt_kwargs": {"lr": 3.0e-4}, "max_grad_norm": 0.5},
    "agent": {"agent_cls": "DecimaScheduler", "embed_dim": 16,
              "gnn_mlp_kwargs": {"hid_dims": [32, 16], "act_cls": "LeakyReLU",
                                 "act_kwargs": {"inplace": True, "negative_slope": 0.2}},
              "policy_mlp_kwargs": {"hid_dims": [64, 64], "act_cls": "Tanh"}},
    "env": {"num_executors": 50, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
            "warmup_delay": 1000.0, "dataset": "tpch", "mean_time_limit": 2.0e7},
}


def make_trainer(cfg: dict, **kw) -> PPO:
    """trainers/__init__.py make_trainer for the PPO trainer_cls of config/decima_tpch.yaml."""
    tc = cfg["trainer"]
    assert tc.get("trainer_cls", "PPO") == "PPO", "only PPO is provided"
    return PPO(cfg["agent"], cfg["env"], tc, **kw)
