#!/usr/bin/env python
"""Diagnostic: where the PPO rollout loop's time goes (BASELINE configs[4]: 16 envs of decima_tpch.yaml,
fused Decima policy). Times the collector's phases per decision step and prints a torch.profiler table."""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))


def main():
    import torch

    from spark_sched_sim.trainers import DECIMA_TPCH, PPO

    cfg = {k: dict(v) for k, v in DECIMA_TPCH.items()}
    cfg["env"]["mean_time_limit"] = 2e6
    ppo = PPO(cfg["agent"], cfg["env"], cfg["trainer"], device="cuda:0")
    col = ppo.collector
    steps = int(os.environ.get("PROF_STEPS", "60"))
    orig = col._decide_and_step
    tm = {"decide_and_step": 0.0}

    def timed(alive, generator=None, **kw):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = orig(alive, generator, **kw)
        torch.cuda.synchronize()
        tm["decide_and_step"] += time.perf_counter() - t0
        return out

    col._decide_and_step = timed
    t0 = time.perf_counter()
    buf = col.collect(ppo._seeds(), ppo._time_limits(ppo._seeds()), generator=ppo.gen, max_steps=steps)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"{steps} steps, {len(buf)} samples: {total / steps * 1e3:.2f} ms/step, decide+step "
          f"{tm['decide_and_step'] / steps * 1e3:.2f} ms/step", flush=True)
    col._decide_and_step = orig
    # phase split of one decide-and-step (same calls as RolloutCollector._decide_and_step)
    from spark_sched_sim.schedulers.decima import build_batch, select_envs

    eng = col.engine
    eng.reset_sampled(2, seeds=ppo._seeds(), time_limits=ppo._time_limits(ppo._seeds()))
    alive = torch.ones(eng.num_envs, dtype=torch.bool, device="cuda:0")
    ph = {k: 0.0 for k in ("features", "build_batch", "node_cap", "fused_policy", "select_envs", "step")}

    def tick():
        torch.cuda.synchronize()
        return time.perf_counter()

    for it in range(steps):
        t0 = tick()
        f = eng.decima_features(*col.scales)
        t1 = tick()
        b_all = build_batch(eng.views, f, env_mask=alive)
        t2 = tick()
        cap = int(b_all.num_nodes.max().item())
        t3 = tick()
        fo = col.policy.schedule_fused(eng, f, seed=1, counter=it, env_mask=alive, node_cap=cap)
        t4 = tick()
        envs = torch.nonzero(alive).squeeze(1)
        select_envs(b_all, envs)
        t5 = tick()
        eng.step(fo["stage_idx"], fo["num_exec"])
        t6 = tick()
        for k, a, b in zip(ph, (t0, t1, t2, t3, t4, t5), (t1, t2, t3, t4, t5, t6)):
            ph[k] += b - a
    print("phase ms/step:", {k: round(v / steps * 1e3, 3) for k, v in ph.items()}, flush=True)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        col.collect(ppo._seeds(), ppo._time_limits(ppo._seeds()), generator=ppo.gen, max_steps=20)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=15), flush=True)
    # one whole PPO iteration: rollouts vs the update (trainer.py:85-162 split)
    t0 = tick()
    buf = ppo.collect()
    t1 = tick()
    ppo.train_on_rollouts(buf)
    t2 = tick()
    print(f"iteration: collect {t1 - t0:.2f} s ({len(buf)} samples), train_on_rollouts {t2 - t1:.2f} s", flush=True)
    # learn split: trajectories/returns/baseline, samples() (cat of the per-step batches), the PPO epochs
    buf = ppo.collect()
    t0 = tick()
    times, rewards, lengths, sample = buf.trajectories()
    returns = ppo.return_calc(times, rewards, lengths)
    ppo.baseline(times[:, :-1], returns, lengths)
    t1 = tick()
    obs, acts = buf.samples()
    t2 = tick()
    advg = torch.zeros(len(buf), dtype=torch.float32, device=obs.x.device)
    ppo._train(obs, acts, advg)
    t3 = tick()
    print(f"learn split: returns+baseline {t1 - t0:.3f} s, samples() {t2 - t1:.3f} s, epochs {t3 - t2:.3f} s",
          flush=True)


if __name__ == "__main__":
    main()
