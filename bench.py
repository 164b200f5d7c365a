#!/usr/bin/env python
"""Scheduling decisions/sec on BASELINE.json configs[1]: 1024 TPC-H-format envs per GPU, 50 jobs /
10 executors, uniform-random valid actions from the device RNG (the reference's examples.py ENV_CFG).

A "step" = one env.step for every env of the batch: device random policy reads the obs, then the step
kernel applies the action, runs the discrete-event loop and writes the next observation to HBM.
Modes: `rollout` (default: K steps = K x envs decisions of policy+step fused into one launch, the decisions
claimed from a shared budget so that envs with cheap decisions take more and the launch has no tail;
`--lockstep` gives every env exactly K; `--compare-lockstep` times one lockstep launch off the clock beside
the budget launch) and
`step` (two launches per step, the C-ABI call pattern of an external policy).

Output: one JSON line on rank 0. Multi-GPU: one process per GPU (torchrun), envs sharded per rank with
no data-path collective (weak scaling); decisions are summed and time is max-reduced over ranks.
"""

from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "gym-sparksched_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

ENV_CFG = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}  # examples.py:15-23
# BASELINE.json configs: "tpch" = configs[1] (the metric's config, default), "decima" = configs[2] (Decima GNN
# policy on the GPU vector env, env section of config/decima_tpch.yaml:80-87), "large" = configs[3]'s per-GPU
# shard (4096 of the 32k envs, 200 jobs / 100 executors, Poisson arrivals, mean_time_limit 2e7 ms).
WORKLOADS = {
    "tpch": dict(cfg=ENV_CFG, envs=1024, mean_time_limit=None,
                 desc="{B} envs/GPU x TPC-H 50 jobs / 10 executors, random valid actions (BASELINE configs[1])"),
    "decima": dict(cfg={"num_executors": 50, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5,
                        "moving_delay": 2000.0, "warmup_delay": 1000.0}, envs=4096, mean_time_limit=2.0e7,
                   desc="{B} envs/GPU x TPC-H 200-job cap / 50 executors, Decima GNN policy (random init) in "
                        "PyTorch-ROCm on device obs (BASELINE configs[2])"),
    "ppo": dict(cfg=None, envs=16, mean_time_limit=2.0e7,
                desc="full PPO iteration of config/decima_tpch.yaml per GPU ({B} rollouts = 4 job sequences x 4, "
                     "Decima GNN, GPU rollouts, data-parallel replicas over RCCL) (BASELINE configs[4])"),
    "large": dict(cfg={"num_executors": 100, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5,
                       "moving_delay": 2000.0, "warmup_delay": 1000.0}, envs=4096, mean_time_limit=2.0e7,
                  desc="{B} envs/GPU x TPC-H 200-job cap / 100 executors, Poisson arrivals, time limits, random "
                       "valid actions (BASELINE configs[3] per-GPU shard)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def _cpu_worker(args):
    """One reference-style rollout worker (trainers/rollout_worker.py:53-95): one env per process,
    torch.set_num_threads(1)-equivalent single thread, RandomScheduler(seed), episodes back to back."""
    seed, seconds = args
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
    from oracle.policies import RandomPolicy
    from oracle.restatement import SparkSchedOracle
    from spark_sched_sim.data_samplers.synthetic_tpch import generate

    ds = generate(0)
    env = SparkSchedOracle(ENV_CFG, ds)
    pol = RandomPolicy(42 + seed)
    env.reset(seed=seed)  # warm-up episode start (not counted)
    decisions, t0, ep = 0, time.perf_counter(), 0
    obs, _ = env.reset(seed=seed)
    while time.perf_counter() - t0 < seconds:
        a, _ = pol.schedule(obs)
        obs, _, done, _, _ = env.step(a)
        decisions += 1
        if done:
            ep += 1
            obs, _ = env.reset(seed=seed + 1000 * ep)
    return decisions, time.perf_counter() - t0


def cpu_baseline(seconds: float, procs: int) -> dict:
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(7 + i, seconds) for i in range(procs)])
    dec = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": dec / wall, "unit": "decisions/s", "cores": procs, "kind": "port",
            "sample": f"{procs} spawn processes x {seconds:.0f}s of config-2 episodes (J=50, N=10), one env per "
                      "process, RandomScheduler(seed) — the CPU oracle restatement (real CPython set/dict/heapq, "
                      "numpy Generator), mirroring trainers/rollout_worker.py"}


def pmc_traffic(kernel: str, mode: str, envs: int, steps_per_launch: int, decisions_per_launch: float):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/r*/pmc_summary*.json,
    made by scripts/pmc_profile.sh + scripts/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
    separate passes), scaled from bytes/decision to this launch. None if no matching summary."""
    import glob

    best = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_summary*.json"))):
        try:
            k = json.load(open(path))["kernels"][kernel]
        except (KeyError, ValueError, OSError):
            continue
        cfg = k.get("config") or {}
        spl = cfg.get("steps_per_launch", k.get("steps") if mode == "rollout" else 1)
        if (cfg.get("mode") == mode and cfg.get("envs_per_gpu") == envs and spl == steps_per_launch
                and "hbm_bytes_per_decision" in k):
            best = (path, k["hbm_bytes_per_decision"])
    if best is None:
        return None, None
    return best[1] * decisions_per_launch, os.path.relpath(best[0], REPO)


def run_ppo(args):
    """BASELINE configs[4]: whole PPO iterations (GPU rollouts to episode end with the Decima GNN, returns,
    baselines, PPO epochs) of config/decima_tpch.yaml; one replica per GPU, gradients averaged over RCCL.
    `--steps` = timed iterations, `--warmup` = untimed ones; value = rollout decisions / iteration time."""
    import torch
    import torch.distributed as dist

    from spark_sched_sim.distributed import rank_world, reduce_timing
    from spark_sched_sim.trainers import DECIMA_TPCH, PPO

    rank, world, local = rank_world()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device(f"cuda:{local}")
    cfg = {k: dict(v) for k, v in DECIMA_TPCH.items()}
    if args.ppo_time_limit:
        cfg["env"]["mean_time_limit"] = args.ppo_time_limit
    ppo = PPO(cfg["agent"], cfg["env"], cfg["trainer"], device=dev)
    for _ in range(args.warmup):
        ppo.train(1, log=None)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    dec = 0
    phases = {"collect_s": 0.0, "learn_s": 0.0}
    for _ in range(args.steps):
        ta = time.perf_counter()
        buf = ppo.collect()
        torch.cuda.synchronize(dev)
        tb = time.perf_counter()
        ppo.episode_stats()
        learn = ppo.train_on_rollouts(buf)
        torch.cuda.synchronize(dev)
        phases["collect_s"] += tb - ta
        phases["learn_s"] += time.perf_counter() - tb
        dec += len(buf)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = reduce_timing(torch.tensor([elapsed, float(dec)], dtype=torch.float64, device=dev), world)
    elapsed, dec = stats.tolist()
    if rank == 0:
        B = ppo.num_sequences * ppo.num_rollouts
        print(json.dumps({
            "metric": "scheduling decisions/sec (env steps/s)", "value": dec / elapsed, "unit": "decisions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 (GNN) + f64/i32 (sim)",
            "data": "synthetic TPC-H-format dataset (seeded generator), Decima GNN random init",
            "config": {"workload": WORKLOADS["ppo"]["desc"].format(B=B), "envs_per_gpu": B,
                       "mean_time_limit": cfg["env"]["mean_time_limit"], "mode": "ppo",
                       "parallelism": f"data-parallel x{world}"},
            "decisions": int(dec), "seconds_per_iteration": elapsed / args.steps,
            "phase_seconds_rank0": phases, "last_learning_stats": learn,
            "roofline": None, "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="tpch")
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the workload's)")
    ap.add_argument("--mode", choices=["rollout", "step"], default="rollout")
    ap.add_argument("--chunk", type=int, default=0,
                    help="rollout mode: steps per fused launch (0 = --steps). Warmup runs in launches of the same "
                         "length (>= --warmup steps in total), so every k_rollout launch is alike and the rocprof "
                         "per-launch average is the timed launches' duration")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = min(16, os.cpu_count())")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--torch-policy", action="store_true",
                    help="decima workload: run the PyTorch DecimaScheduler instead of the fused kernel")
    ap.add_argument("--ppo-time-limit", type=float, default=0.0,
                    help="ppo workload: override mean_time_limit (ms) of config/decima_tpch.yaml (0 = keep 2e7)")
    ap.add_argument("--lockstep", action="store_true",
                    help="rollout mode: every env takes exactly `chunk` decisions per launch (ssim_rollout_ex) "
                         "instead of sharing a budget of envs x chunk decisions (ssim_rollout_budget)")
    ap.add_argument("--compare-lockstep", action="store_true",
                    help="rollout mode: after the timed region, time one lockstep launch of the same length "
                         "(off by default so a rocprof of the default run sees only warm-up + timed launches)")
    ap.add_argument("--no-autoreset", action="store_true",
                    help="rollout mode: leave finished envs idle instead of resetting them on the device")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import gather_env_stats, rank_world, reduce_timing, shard_seeds
    from spark_sched_sim.engine import DeviceEngine

    rank, world, local = rank_world()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device(f"cuda:{local}")

    if args.workload == "ppo":
        return run_ppo(args)
    wl = WORKLOADS[args.workload]
    cfg = wl["cfg"]
    B, K, W = args.envs or wl["envs"], args.steps, args.warmup
    if args.workload == "decima":
        args.mode = "decima"
    eng = DeviceEngine(cfg, B, generate(0), device=dev)
    seeds = shard_seeds(rank, B, args.seed)
    limits = None
    if wl["mean_time_limit"]:  # StochasticTimeLimit (wrappers/stochastic_time_limit.py:5-31), per env
        from spark_sched_sim.wrappers import StochasticTimeLimitSampler

        smp = StochasticTimeLimitSampler(wl["mean_time_limit"], B, seed=42)
        limits = torch.tensor([smp.sample(i, int(seeds[i])) for i in range(B)], dtype=torch.float64, device=dev)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=None if limits is None else limits.cpu().numpy())
    kind = _abi.SSIM_POLICY_RANDOM
    stream = torch.cuda.current_stream(dev)

    chunk = args.chunk if args.chunk > 0 else K
    flags = 0 if args.no_autoreset else _abi.SSIM_ROLLOUT_AUTORESET
    if args.mode == "decima":
        from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

        torch.manual_seed(args.seed)
        pol = DecimaScheduler(cfg["num_executors"]).to(dev)  # decima_tpch.yaml:66-78 dims, random init
        gen = torch.Generator(device=dev).manual_seed(args.seed)
        cnt = eng.views["counts"]
        packed = pol.packed_params(dev)  # fixed weights during rollouts: packed once, like RolloutCollector

    def chunks(n):
        return [chunk] * (n // chunk) + ([n % chunk] if n % chunk else [])

    def run(n, events=None):
        if args.mode == "rollout":
            for k, c in enumerate(chunks(n)):
                if events is not None:
                    events[2 * k].record(stream)
                if args.lockstep:
                    eng.rollout(kind, 1234, c, flags=flags, time_limits=limits)
                else:  # the same B x c decisions, claimed by whichever env is ready (no tail)
                    eng.rollout_budget(kind, 1234, 8 * c, B * c, flags=flags, time_limits=limits)
                if events is not None:
                    events[2 * k + 1].record(stream)
        elif args.mode == "decima":
            for k in range(n):
                if args.torch_policy:  # the batched PyTorch module (~150 launches per decision)
                    act = pol.schedule(build_batch(eng.views, eng.decima_features()), generator=gen)
                else:  # one fused HIP launch (ssim_decima_policy)
                    run.counter += 1
                    act = pol.schedule_fused(eng, eng.decima_features(), seed=args.seed, counter=run.counter,
                                             params=packed)
                if events is not None:
                    events[2 * k].record(stream)
                eng.step(act["stage_idx"], act["num_exec"])
                if events is not None:
                    events[2 * k + 1].record(stream)
                done = ((cnt[:, _abi.OC_TERMINATED] != 0) | (cnt[:, _abi.OC_TRUNCATED] != 0)).to(torch.uint8)
                eng.reset_sampled(done, time_limits=limits)  # finished episodes: reset(seed=None) on device
        else:
            for k in range(n):
                si, ne = eng.policy(kind, 1234, run.counter)
                run.counter += 1
                if events is not None:
                    events[2 * k].record(stream)
                eng.step(si, ne)
                if events is not None:
                    events[2 * k + 1].record(stream)
    run.counter = 0

    if args.mode == "rollout":
        W = -(-W // chunk) * chunk if W > 0 else 0  # whole launches of `chunk` steps
    run(W)
    torch.cuda.synchronize(dev)
    counts0 = eng.views["counts"].cpu().numpy().copy()
    acc0 = eng.views["acc"].cpu().numpy().copy()
    launches = len(chunks(K)) if args.mode == "rollout" else K
    n_ev = 2 * launches
    events = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(K, events)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    counts1 = eng.views["counts"].cpu().numpy()
    acc1 = eng.views["acc"].cpu().numpy()
    lockstep = None
    if args.mode == "rollout" and not args.lockstep and args.compare_lockstep:
        # off the clock: one lockstep launch of the same length (every env exactly `chunk` decisions) for
        # comparison -- its time is set by the env whose `chunk` decisions cost the most
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        a0 = eng.views["acc"].cpu().numpy().copy()
        ev[0].record(stream)
        eng.rollout(kind, 1234, chunk, flags=flags, time_limits=limits)
        ev[1].record(stream)
        torch.cuda.synchronize(dev)
        ld = float((eng.views["acc"].cpu().numpy() - a0).sum(axis=0)[_abi.ACC_DECISIONS])
        lockstep = {"decisions": int(ld), "kernel_ms": ev[0].elapsed_time(ev[1]),
                    "decisions_per_s": ld / (ev[0].elapsed_time(ev[1]) / 1e3)}
    errs = int(np.count_nonzero(counts1[:, _abi.OC_ERR] & _abi.SSIM_ERR_STICKY))
    d_acc = (acc1 - acc0).sum(axis=0).astype(np.float64)  # S_act, E_act, J_act, events, decisions, episodes
    decisions = int(d_acc[_abi.ACC_DECISIONS])  # over all episodes (auto-reset restarts the per-episode count)
    terminated = int(counts1[:, _abi.OC_TERMINATED].sum())
    episodes_done = int(d_acc[_abi.ACC_EPISODES])
    # B_dec = 36 S_act + 20 E_act + 16 J_act + 96 K + 40 bytes per decision
    alg_bytes = 36 * d_acc[0] + 20 * d_acc[1] + 16 * d_acc[2] + 96 * d_acc[3] + 40 * decisions
    kern_ms = sum(events[2 * k].elapsed_time(events[2 * k + 1]) for k in range(launches))
    elapsed = t1 - t0
    stats = torch.tensor([elapsed, float(decisions), alg_bytes, kern_ms, float(errs), float(terminated)],
                         dtype=torch.float64, device=dev)
    stats = reduce_timing(stats, world)
    # episode statistics gather (the only data collective; RCCL all_gather, off the timed path)
    mine = torch.tensor(counts1[:, [_abi.OC_NUM_COMPLETED, _abi.OC_NUM_ARRIVED, _abi.OC_DECISIONS]],
                        dtype=torch.int32, device=dev)
    gathered = gather_env_stats(mine, world)
    elapsed, decisions, alg_bytes, kern_ms_sum, errs, terminated = stats.tolist()
    kern_ms = kern_ms_sum / world
    value = decisions / elapsed
    achieved = (alg_bytes / world / launches) / (kern_ms / launches / 1e3) / 1e9  # GB/s per GPU, dominant kernel
    kernel = "k_rollout" if args.mode == "rollout" else "k_step"
    traffic, traffic_src = pmc_traffic(kernel, args.mode, B, chunk if args.mode == "rollout" else 1,
                                       decisions / world / launches)
    if rank == 0:
        line = {
            "metric": "scheduling decisions/sec (env steps/s)",
            "value": value,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+i32",
            "data": "synthetic TPC-H-format dataset (seeded generator), " + (
                "Decima GNN policy, random-init weights" if args.mode == "decima" else
                "random valid actions (device RNG)"),
            "config": {"workload": wl["desc"].format(B=B), "envs_per_gpu": B,
                       "jobs": cfg["job_arrival_cap"], "executors": cfg["num_executors"],
                       "mean_time_limit": wl["mean_time_limit"], "mode": args.mode,
                       "policy": ("torch" if args.torch_policy else "fused HIP kernel") if args.mode == "decima"
                       else "device random",
                       "steps_per_launch": chunk if args.mode == "rollout" else 1,
                       "work_sharing": ("lockstep" if args.lockstep else "shared budget of envs x steps "
                                        "decisions per launch") if args.mode == "rollout" else None,
                       "autoreset": bool(args.mode != "step" and (flags or args.mode == "decima")),
                       "parallelism": f"env-sharded x{world}"},
            "decisions": int(decisions),
            "terminated_envs": int(terminated),
            "episodes_finished": episodes_done,
            "frozen_envs": int(errs),
            "jobs_completed": int(gathered[:, 0].sum().item()),
            "jobs_arrived": int(gathered[:, 1].sum().item()),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel,
                         "kernel_ms_per_launch": kern_ms / launches,
                         "alg_bytes_per_launch": alg_bytes / world / launches},
            "cpu_baseline": None,
        }
        if lockstep is not None:
            line["lockstep_1gpu"] = lockstep
        if not args.no_cpu_baseline and world == 1 and args.workload == "tpch":
            procs = args.cpu_procs or min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, procs)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
