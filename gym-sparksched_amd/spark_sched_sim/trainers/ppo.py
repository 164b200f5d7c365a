"""PPO on GPU rollouts (trainers/ppo.py:45-138 on top of trainers/trainer.py:28-190).

One process per GPU. Each rank owns `num_sequences` job sequences x `num_rollouts` rollouts (all rollouts of a
sequence on one GPU, so the Baseline interpolation stays local) as rows of one vector env, and a
replica of the policy. Per iteration:
  1. collect: RolloutCollector runs every row to the end of its episode (device-side reset with the
     sequence's seed, Decima forward per decision, ssim_step);
  2. returns (ReturnsCalculator) and baselines (Baseline) on device; advantages = returns - baselines;
  3. PPO epochs over shuffled minibatches (num_batches per epoch): evaluate_actions with grads, CLIP loss with
     the entropy bonus; gradients all-reduced (averaged) across ranks in one flat bucket over RCCL, then
     clip_grad_norm + optimizer step on every replica (identical updates keep replicas equal); the
     minibatch advantage normalisation and the approx-KL early stop use all-reduced statistics so every
     rank takes the same decisions;
  4. episode statistics (avg job duration, avg #jobs, completed / arrived jobs) all-gathered to every rank.
Seeds follow trainer.py:258-262 / rollout_worker.py:118-120: row (sequence s, rollout r) of rank k uses
seed + global_sequence + num_sequences_total * iteration.
"""

from __future__ import annotations

import math
from typing import Any

import numpy as np
import torch

from .. import _abi
from ..schedulers.decima import DecimaScheduler, select_envs
from .returns import Baseline, ReturnsCalculator
from .rollouts import AsyncRolloutCollector, RolloutCollector

EPS = 1e-8  # ppo.py:13


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def _allreduce_(t: torch.Tensor, op="sum") -> torch.Tensor:
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t, op=d.ReduceOp.MAX if op == "max" else d.ReduceOp.SUM)
    return t


class PPO:
    def __init__(self, agent_cfg: dict, env_cfg: dict, train_cfg: dict, engine_factory=None, dataset=None,
                 device=None):
        d = _dist()
        self.rank = d.get_rank() if d else 0
        self.world = d.get_world_size() if d else 1
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.seed = int(train_cfg["seed"])
        torch.manual_seed(self.seed)  # identical initial replicas on every rank (trainer.py:33)
        self.num_sequences = int(train_cfg["num_sequences"])  # per rank
        self.num_rollouts = int(train_cfg["num_rollouts"])
        self.num_iterations = int(train_cfg.get("num_iterations", 1))
        self.entropy_coeff = float(train_cfg.get("entropy_coeff", 0.0))
        self.clip_range = float(train_cfg.get("clip_range", 0.2))
        self.target_kl = train_cfg.get("target_kl", 0.01)
        self.num_epochs = int(train_cfg.get("num_epochs", 10))
        self.num_batches = int(train_cfg.get("num_batches", 3))
        assert ("reward_buff_cap" in train_cfg) ^ ("beta_discount" in train_cfg), \
            "must provide exactly one of `reward_buff_cap` and `beta_discount` in config"
        env_cfg = {k: v for k, v in env_cfg.items() if k != "dataset"}
        if "beta_discount" in train_cfg:
            env_cfg["beta"] = float(train_cfg["beta_discount"])
            self.return_calc = ReturnsCalculator(beta=float(train_cfg["beta_discount"]))
        else:
            self.return_calc = ReturnsCalculator(buff_cap=int(train_cfg["reward_buff_cap"]))
        self.env_cfg = env_cfg
        self.mean_time_limit = env_cfg.get("mean_time_limit")
        self.baseline = Baseline(self.num_sequences, self.num_rollouts)
        kw = {k: v for k, v in agent_cfg.items() if k != "agent_cls"}
        self.scheduler = DecimaScheduler(env_cfg["num_executors"], opt_cls=train_cfg.get("opt_cls", "Adam"),
                                         opt_kwargs=train_cfg.get("opt_kwargs"),
                                         max_grad_norm=train_cfg.get("max_grad_norm"), **kw).to(self.device)
        B = self.num_sequences * self.num_rollouts
        if dataset is None:
            from ..data_samplers.synthetic_tpch import generate

            dataset = generate(0)
        if engine_factory is None:
            from ..engine import DeviceEngine

            def engine_factory(cfg, n, ds):
                return DeviceEngine(cfg, n, ds, device=self.device)
        self.engine = engine_factory({k: v for k, v in env_cfg.items() if k != "mean_time_limit"}, B, dataset)
        self.rollout_duration = train_cfg.get("rollout_duration")  # trainer.py:63, async workers :277-279
        if self.rollout_duration:
            S_tot = self.num_sequences * self.world
            base = [self.seed + self.rank * self.num_sequences + s for s in range(self.num_sequences)
                    for _ in range(self.num_rollouts)]
            self.collector = AsyncRolloutCollector(self.engine, self.scheduler, self.rollout_duration, base, S_tot,
                                                   mean_time_limit=self.mean_time_limit,
                                                   seed=self.seed * 7919 + self.rank)
        else:
            self.collector = RolloutCollector(self.engine, self.scheduler, seed=self.seed * 7919 + self.rank)
        self.gen = torch.Generator(device=self.device).manual_seed(self.seed * 7919 + self.rank)
        self.time_limit_rngs = None
        if self.mean_time_limit:
            # one StochasticTimeLimit per row, seeded like the reference wrapper (seed=42, reseeded by reset seed)
            self.time_limit_rngs = [np.random.RandomState(42) for _ in range(B)]
        self.reset_count = 0

    # ------------------------------------------------------------------ rollouts
    def _seeds(self) -> list[int]:
        """rollout_worker.py:118-120 with trainer.py:258-262's base seeds: sequence s gets
        seed + s_global + S_total * reset_count, shared by its num_rollouts rows."""
        S_tot = self.num_sequences * self.world
        out = []
        for s in range(self.num_sequences):
            sg = self.rank * self.num_sequences + s
            out += [self.seed + sg + S_tot * self.reset_count] * self.num_rollouts
        return out

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
            return self.collector.collect(generator=self.gen)
        seeds = self._seeds()
        buf = self.collector.collect(seeds, self._time_limits(seeds), generator=self.gen)
        self.reset_count += 1
        return buf

    # ------------------------------------------------------------------ learning
    def train_on_rollouts(self, buf) -> dict[str, Any]:
        times, rewards, lengths, sample = buf.trajectories()
        returns = self.return_calc(times, rewards, lengths)
        base = self.baseline(times[:, :-1], returns, lengths)
        valid = sample >= 0
        n = len(buf)
        advg = torch.zeros(n, dtype=torch.float64, device=returns.device)
        advg[sample[valid]] = (returns - base)[valid]
        obs, acts = buf.samples()
        return self._train(obs, acts, advg.float())

    def _train(self, obs, acts, advg) -> dict[str, Any]:
        n = obs.num_envs
        bs = n // self.num_batches + 1  # ppo.py:69
        pol_losses, ent_losses, kls = [], [], []
        cont = True
        self.scheduler.train()
        for _ in range(self.num_epochs):
            if not cont:
                break
            perm = torch.randperm(n, device=advg.device, generator=self.gen)
            for k in range(0, n, bs):
                idx = perm[k: k + bs]
                loss, info = self._loss(select_envs(obs, idx), {a: t[idx] for a, t in acts.items()}, advg[idx])
                pol_losses.append(info["policy_loss"])
                ent_losses.append(info["entropy_loss"])
                kls.append(info["approx_kl_div"])
                if self.target_kl is not None and info["approx_kl_div"] > 1.5 * self.target_kl:
                    cont = False  # every rank sees the same all-reduced KL
                    break
                self._update(loss)
        return {"policy loss": abs(float(np.mean(pol_losses))), "entropy": abs(float(np.mean(ent_losses))),
                "approx kl div": abs(float(np.mean(kls))), "samples": n}

    def _loss(self, obs, acts, advg):
        ev = self.scheduler.evaluate_actions(obs, acts["stage_idx"], acts["job_idx"], acts["exec_idx"])
        # minibatch advantage normalisation (ppo.py:118-119) over all ranks' minibatches
        st = torch.stack([advg.sum().double(), (advg.double() ** 2).sum(), torch.tensor(float(advg.numel()),
                          dtype=torch.float64, device=advg.device)])
        _allreduce_(st)
        m = st[0] / st[2]
        var = (st[1] - st[2] * m * m) / torch.clamp(st[2] - 1, min=1)
        a = (advg - m.float()) / (var.clamp(min=0).sqrt().float() + EPS)
        log_ratio = ev["lgprobs"] - acts["lgprob"]
        ratio = log_ratio.exp()
        pl = -torch.min(a * ratio, a * torch.clamp(ratio, 1 - self.clip_range, 1 + self.clip_range)).mean()
        el = -ev["entropies"].mean()
        loss = pl + self.entropy_coeff * el
        with torch.no_grad():
            red = torch.stack([pl.detach().double(), el.detach().double(), ((ratio - 1) - log_ratio).mean().double()])
            _allreduce_(red)
            red /= self.world
        return loss, {"policy_loss": float(red[0]), "entropy_loss": float(red[1]), "approx_kl_div": float(red[2])}

    def _update(self, loss):
        """TrainableScheduler.update_parameters (scheduler.py:34-53) with a data-parallel gradient average."""
        s = self.scheduler
        loss.backward()
        params = [p for p in s.parameters() if p.grad is not None]
        if self.world > 1 and params:
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            _allreduce_(flat)
            flat /= self.world
            o = 0
            for p in params:
                k = p.grad.numel()
                p.grad.copy_(flat[o: o + k].view_as(p.grad))
                o += k
        if s.max_grad_norm:
            torch.nn.utils.clip_grad_norm_(s.parameters(), s.max_grad_norm, error_if_nonfinite=True)
        s.optim.step()
        s.optim.zero_grad()

    # ------------------------------------------------------------------ statistics
    def episode_stats(self) -> torch.Tensor:
        """rollout_worker.py:122-129 per row: [avg job duration (s), avg #jobs, completed, arrived], gathered
        from every rank (RCCL all_gather): [world * rows, 4]."""
        eng = self.engine
        if hasattr(eng, "job_times") and isinstance(eng.views["counts"], torch.Tensor):
            ta, tc, st = eng.job_times()
            wall = eng.views["wall_time"].double()
        else:
            a, c, s_ = eng.job_times_np()
            ta, tc, st = (torch.from_numpy(x).to(self.device) for x in (a, c, s_))
            wall = torch.from_numpy(np.asarray(eng.host_views()["wall_time"])).to(self.device).double()
        arrived = st > 0
        end = torch.where(st == 2, tc, wall[:, None].expand_as(tc))
        dur = torch.where(arrived, torch.minimum(end, wall[:, None]) - ta, torch.zeros_like(ta))
        n_done = (st == 2).sum(1)
        # SparkSchedSimEnv.avg_job_duration (spark_sched_sim.py:243-245): mean completed-job duration, seconds
        avg_jd = torch.where(st == 2, tc - ta, torch.zeros_like(ta)).sum(1) / n_done.clamp(min=1) * 1e-3
        avg_jobs = dur.sum(1) / wall.clamp(min=1e-12)
        mine = torch.stack([avg_jd, avg_jobs, n_done.double(), arrived.sum(1).double()], dim=1)
        d = _dist()
        if d is None or self.world == 1:
            return mine
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        d.all_gather(parts, mine.contiguous())
        return torch.cat(parts)

    def train(self, num_iterations: int | None = None, log=print) -> list[dict]:
        hist = []
        for i in range(num_iterations or self.num_iterations):
            buf = self.collect()
            stats = self.episode_stats()
            learn = self.train_on_rollouts(buf)
            avg_jobs = float(stats[:, 1].mean())
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
