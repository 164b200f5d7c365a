#!/usr/bin/env python
"""Scheduling decisions/sec on BASELINE.json configs[1]: 1024 TPC-H-format envs per GPU, 50 jobs /
10 executors, uniform-random valid actions from the device RNG (the reference's examples.py ENV_CFG).

A "step" = one env.step for every env of the batch: the device random policy reads the env's observation,
then the step applies the action, runs the discrete-event loop and writes the next observation to HBM.

Timeline of one run (all launches on one stream, inputs resident in HBM before anything is timed):
  1. reset every env on the device (ssim_reset_sampled, seeds = global env ids);
  2. pre-roll (untimed, not warm-up): env i takes a seeded, uniformly random number of decisions in
     [0, `preroll`) with auto-reset (ssim_rollout_steps), so the batch is spread over every phase of its
     episodes — early, late and restarting — instead of all envs sitting at the same decision index;
  3. warm-up: exactly `--warmup` steps (one launch of warmup x envs decisions);
  4. timed: exactly `--steps` steps (launches of `--chunk` steps, default one), bracketed by barrier +
     synchronize; HIP events on the launch stream time the kernels for the roofline.
Modes: `rollout` (default: K steps = K x envs decisions of policy+step fused into one launch, claimed from a
shared budget so envs with cheap decisions take more; once the budget is claimed, steps still simulating stop at
their next event boundary and complete in the next launch (SSIM_ROLLOUT_PREEMPT), so a launch ends within ~one
event instead of ~the longest step; decisions are counted when they complete; `--lockstep` gives every env
exactly K) and `step` (two launches per step, the C-ABI call pattern of an external policy).

Multi-GPU: `--gpus N` with no torchrun environment spawns N worker processes itself (one per GPU, before any
HIP call); under torchrun the environment is used as is. Envs are sharded in contiguous blocks per rank with no
data-path collective (weak scaling); decisions are summed and time is max-reduced over ranks.

Output: one JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "gym-sparksched_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

ENV_CFG = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}  # examples.py:15-23
DECIMA_ENV = {"num_executors": 50, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
              "warmup_delay": 1000.0}  # config/decima_tpch.yaml:80-87
LARGE_ENV = {"num_executors": 100, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
             "warmup_delay": 1000.0}
# BASELINE.json configs: "tpch" = configs[1] (the metric's config, default), "decima" = configs[2] (Decima GNN
# policy on the GPU vector env, env section of config/decima_tpch.yaml:80-87), "large" = configs[3]'s per-GPU
# shard (4096 of the 32k envs, 200 jobs / 100 executors, Poisson arrivals, mean_time_limit 2e7 ms).
# `preroll`: upper bound of the per-env pre-roll (about one episode of the workload's policy).
WORKLOADS = {
    "tpch": dict(cfg=ENV_CFG, envs=1024, mean_time_limit=None, preroll=1000, policy="random",
                 desc="{B} envs/GPU x TPC-H 50 jobs / 10 executors, random valid actions (BASELINE configs[1])"),
    "decima": dict(cfg=DECIMA_ENV, envs=4096, mean_time_limit=2.0e7, preroll=1500, policy="decima",
                   desc="{B} envs/GPU x TPC-H 200-job cap / 50 executors, Decima GNN policy (random init) on "
                        "device obs (BASELINE configs[2])"),
    "ppo": dict(cfg=DECIMA_ENV, envs=16, mean_time_limit=2.0e7, preroll=0, policy="decima",
                desc="full PPO iteration of config/decima_tpch.yaml ({B} rollouts = 4 job sequences x 4, Decima "
                     "GNN, GPU rollouts, trajectories gathered to one learner over RCCL) (BASELINE configs[4])"),
    "large": dict(cfg=LARGE_ENV, envs=4096, mean_time_limit=2.0e7, preroll=3000, policy="random",
                  desc="{B} envs/GPU x TPC-H 200-job cap / 100 executors, Poisson arrivals, time limits, random "
                       "valid actions (BASELINE configs[3] per-GPU shard)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# CPU-only reference config (BASELINE configs[0]): examples.py --sched fair, one env in one process
CPU_ONLY = {"examples": dict(cfg=ENV_CFG, mean_time_limit=None, policy="fair",
                             desc="examples.py --sched fair: one env, 50 jobs / 10 executors (BASELINE configs[0])")}


def _workload(name: str) -> dict:
    return WORKLOADS[name] if name in WORKLOADS else CPU_ONLY[name]


# ------------------------------------------------------------------------------------------------ launcher
def launch_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` without a torchrun environment: one worker process per GPU (trainer.py:264-296 fans out
    rollout processes the same way), started BEFORE this process touches HIP. Returns the worst exit code."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:  # one rank failed: the collectives of the others would hang
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


# ------------------------------------------------------------------------------------------------ CPU baseline
def usable_cpus() -> int:
    """CPUs this process may run on: the affinity mask, capped by a cgroup-v2 CPU quota (the GPU box gives a
    job a share of the host's cores; os.cpu_count() reports the whole host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(args):
    """One reference-style rollout worker (trainers/rollout_worker.py:53-95): one env per process, single
    thread, episodes back to back with the workload's policy; warm-up = the first episode (at most
    `warm_s` seconds), then decisions are counted for `seconds` of wall time."""
    workload, seed, seconds, warm_s, ds_seed = args
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
    import numpy as np

    from oracle.policies import FairPolicy, RandomPolicy
    from oracle.restatement import InvariantError, SparkSchedOracle
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.wrappers import StochasticTimeLimit

    try:
        import torch

        torch.set_num_threads(1)  # rollout_worker.py:93
    except ImportError:
        torch = None
    wl = _workload(workload)
    cfg = wl["cfg"]
    env = SparkSchedOracle(cfg, generate(ds_seed))
    if wl["mean_time_limit"]:
        env = StochasticTimeLimit(env, wl["mean_time_limit"])
    if wl["policy"] == "decima":
        from oracle import decima as D
        from oracle import decima_gnn as G
        from spark_sched_sim.schedulers.decima import DecimaScheduler

        torch.manual_seed(seed)
        sd = {k: v.detach().float() for k, v in DecimaScheduler(cfg["num_executors"]).state_dict().items()}
        rng = np.random.default_rng(seed)
        N = cfg["num_executors"]

        def act(obs):  # DecimaScheduler.schedule (scheduler.py:71-99) on the wrapped observation
            ro = D.decima_observation(obs, N)
            if not ro["stage_mask"].any():
                return {"stage_idx": -1, "num_exec": max(1, obs["num_committable_execs"])}
            with torch.no_grad():
                enc = G.encode(sd, ro)
                s = G.stage_scores(sd, ro, enc).numpy()
                si = int(np.argmax(s - np.log(-np.log(rng.random(s.shape)))))
                j = G.job_of_stage(ro, si)
                e = G.exec_scores(sd, ro, enc, j, N).numpy()
                ei = int(np.argmax(e - np.log(-np.log(rng.random(e.shape)))))
            return {"stage_idx": si, "num_exec": 1 + ei}  # DecimaActWrapper.action (env_wrapper.py:33-34)
    else:
        pol = FairPolicy(cfg["num_executors"]) if wl["policy"] == "fair" else RandomPolicy(42 + seed)

        def act(obs):
            return pol.schedule(obs)[0]
    def step(obs):
        # The reference asserts "[step]" (spark_sched_sim.py:214-217) when a round's simulation drains the event
        # queue without a decision to make before every job completes; the oracle raises InvariantError there. A
        # worker process would die on it, so the harness ends that episode instead and counts it (aborted).
        try:
            o, _, term, trunc, _ = env.step(act(obs))
            return o, term or trunc, False
        except InvariantError:
            return None, True, True

    ep, aborted = 0, 0
    obs, _ = env.reset(seed=seed)
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < warm_s:  # warm-up: one episode (bounded)
        obs, done, _ = step(obs)
        if done:
            break
    ep += 1
    obs, _ = env.reset(seed=seed + 1000 * ep)
    decisions, episodes, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        obs, done, bad = step(obs)
        decisions += not bad  # a step the [step] assertion aborted never completed: not a decision
        aborted += bad
        if done:
            ep += 1
            episodes += 1
            obs, _ = env.reset(seed=seed + 1000 * ep)
    return decisions, time.perf_counter() - t0, episodes, aborted


def cpu_baseline(workload: str, seconds: float, procs: int, warm_s: float = 5.0, ds_seed: int = 0) -> dict:
    """The reference's CPU rollout path, timed on this host's cores: the oracle restatement (same CPython
    dict/set/heapq and numpy Generator machinery as spark_sched_sim) in `procs` spawn processes, one env each,
    harness shaped like trainers/rollout_worker.py:53-95."""
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(workload, 7 + i, seconds, warm_s, ds_seed) for i in range(procs)])
    dec = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    host = os.cpu_count() or procs
    value = dec / wall
    wl = _workload(workload)
    return {"value": value, "unit": "decisions/s", "cores": procs, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": host, "usable_cpus": usable_cpus(),
            "per_core": value / procs, "projected_host": value / procs * host,
            "episodes_finished": int(sum(r[2] for r in res)), "episodes_aborted": int(sum(r[3] for r in res)),
            "seconds": wall,
            "sample": f"{procs} spawn processes (one per usable CPU of this job) x {seconds:.0f} s after a "
                      f"1-episode warm-up, {workload} workload (J={wl['cfg']['job_arrival_cap']}, "
                      f"N={wl['cfg']['num_executors']}, {wl['policy']} policy), one env per process: the CPU "
                      "oracle restatement (real CPython set/dict/heapq, numpy Generator) in the "
                      "trainers/rollout_worker.py harness shape; projected_host = per_core x host_cpus "
                      "(an upper bound for the whole host)"}


def add_ratios(cb: dict, gpu_value: float) -> dict:
    """The north-star ratio read straight off the line: this run's GPU rate over the CPU path measured on the cores
    used (`ratio_measured`) and over that path projected to every CPU of the host (`ratio_projected_host`). Both are
    for the GPUs this line measured; a node-level (8-GPU) ratio needs the driver's own 8-GPU line."""
    cb["ratio_measured"] = gpu_value / cb["value"] if cb.get("value") else None
    cb["ratio_projected_host"] = gpu_value / cb["projected_host"] if cb.get("projected_host") else None
    return cb


# ------------------------------------------------------------------------------------------------ PMC lookup
def pmc_traffic(kernel: str, mode: str, envs: int, steps_per_launch: int, decisions_per_launch: float,
                dataset_seed: int = 0, build_id: str | None = None):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/r*/pmc_summary*.json,
    made by scripts/pmc_profile.sh + scripts/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
    separate passes) of the SAME BUILD (the library's ssim_build_id, recorded in the summary from the bench line
    of its passes) and config, scaled from bytes/decision to this launch; plus the summary's issue counters per
    decision when present. (None, None, None) if no summary of this build matches the config: a summary of another
    build is never quoted for this one."""
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
                and cfg.get("dataset_seed", 0) == dataset_seed and "hbm_bytes_per_decision" in k
                and k.get("build_id") == build_id):
            best = (path, k)
    if best is None:
        return None, None, None
    return best[1]["hbm_bytes_per_decision"] * decisions_per_launch, os.path.relpath(best[0], REPO), best[1]


# ------------------------------------------------------------------------------------------------ PPO
def run_ppo(args, rank, world, local, dev):
    """BASELINE configs[4]: whole PPO iterations (GPU rollouts with the Decima GNN, returns, baselines, PPO
    epochs) of config/decima_tpch.yaml; num_sequences x num_rollouts rows split over the ranks, trajectories
    gathered to one learner (rank 0) over RCCL, parameters broadcast back (trainer.py:85-162).
    `--steps` = timed iterations, `--warmup` = untimed ones; value = rollout decisions / iteration time."""
    import torch
    import torch.distributed as dist

    from spark_sched_sim.distributed import reduce_timing
    from spark_sched_sim.trainers import DECIMA_TPCH, PPO

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
    learn = None
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
    from spark_sched_sim.distributed import gather_env_stats

    per_rank = gather_env_stats(torch.tensor([[float(rank), elapsed, float(dec)]], dtype=torch.float64, device=dev),
                                world).cpu().tolist()
    ranks_seen = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    stats = reduce_timing(torch.tensor([elapsed, float(dec)], dtype=torch.float64, device=dev), world)
    elapsed, dec = stats.tolist()
    line = None
    if rank == 0:
        B = ppo.num_sequences * ppo.num_rollouts
        line = {
            "metric": "scheduling decisions/sec (env steps/s)", "value": dec / elapsed, "unit": "decisions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32 (GNN) + f64/i32 (sim)",
            "data": "synthetic TPC-H-format dataset (seeded generator), Decima GNN random init",
            "config": {"workload": WORKLOADS["ppo"]["desc"].format(B=B), "rows_global": B,
                       "mean_time_limit": cfg["env"]["mean_time_limit"], "mode": "ppo",
                       "parallelism": f"rows split over {world} ranks, one learner"},
            "decisions": int(dec), "seconds_per_iteration": elapsed / args.steps, "ranks_seen": ranks_seen,
            "per_rank": [{"rank": int(r), "elapsed_s": e, "decisions": int(d)} for r, e, d in per_rank],
            "phase_seconds_rank0": phases, "last_learning_stats": learn,
            "roofline": None, "cpu_baseline": None}
        if not args.no_cpu_baseline and world == 1:
            # the reference iteration's rollout phase: num_sequences x num_rollouts = 16 rollout processes
            # (trainer.py:264-296) running the Decima GNN on the CPU; an upper bound on its decisions/s (the
            # learner's time is excluded)
            line["cpu_baseline"] = cpu_baseline("decima", args.cpu_seconds, B)
            line["cpu_baseline"]["sample"] += "; rollout phase of the PPO iteration only (learner excluded)"
            add_ratios(line["cpu_baseline"], line["value"])
    return line


# ------------------------------------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="tpch")
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the workload's)")
    ap.add_argument("--mode", choices=["rollout", "step"], default="rollout")
    ap.add_argument("--chunk", type=int, default=0, help="rollout mode: timed steps per fused launch (0 = --steps)")
    ap.add_argument("--preroll", type=int, default=-1,
                    help="pre-roll bound (env i takes U[0, preroll) decisions before warm-up; -1 = the workload's, "
                         "0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=60.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = every usable CPU of this job")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dataset-seed", type=int, default=0,
                    help="synthetic TPC-H-format dataset generator seed (0: stage cap 900, the bench kernel with every "
                         "shape constant; 1: stage cap 850, the kernel that reads the cap at run time, as real "
                         "traces would)")
    ap.add_argument("--torch-policy", action="store_true",
                    help="decima workload: run the PyTorch DecimaScheduler instead of the fused kernel")
    ap.add_argument("--decima-lockstep", action="store_true",
                    help="decima workload: per decision one fused policy launch + one ssim_step launch for every env "
                         "(the round-2 path) instead of the persistent Decima rollout (ssim_decima_rollout)")
    ap.add_argument("--ppo-time-limit", type=float, default=0.0,
                    help="ppo workload: override mean_time_limit (ms) of config/decima_tpch.yaml (0 = keep 2e7)")
    ap.add_argument("--lockstep", action="store_true",
                    help="rollout mode: every env takes exactly `chunk` decisions per launch (ssim_rollout_ex) "
                         "instead of sharing a budget of envs x chunk decisions (ssim_rollout_budget)")
    ap.add_argument("--no-preempt", action="store_true",
                    help="rollout mode: budget launches finish every started step (no SSIM_ROLLOUT_PREEMPT)")
    ap.add_argument("--no-autoreset", action="store_true",
                    help="rollout mode: leave finished envs idle instead of resetting them on the device")
    ap.add_argument("--force-hbm", action="store_true",
                    help="diagnostic: keep the hot blocks in HBM (SSIM_CFG_FORCE_HBM) whatever their size: the "
                         "HBM-resident kernels (4 waves per SIMD) instead of the LDS-resident one")
    ap.add_argument("--engine", choices=["hip", "host"], default="hip",
                    help="host = the TEST-ONLY CPU build of the engine (tests/hostsim) over gloo, to exercise the "
                         "launcher and the rank plumbing in the CPU test suite; never a measurement")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import numpy as np
    import torch
    import torch.distributed as dist

    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import gather_env_stats, rank_world, reduce_timing, shard_seeds

    host = args.engine == "host"
    build_id = None
    if not host:
        from spark_sched_sim import native

        build_id = native.build_id()
    rank, world, local = rank_world()
    if world > 1:
        if host:
            dist.init_process_group("gloo", init_method="env://")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cpu") if host else torch.device(f"cuda:{local}")

    def sync():
        if not host:
            torch.cuda.synchronize(dev)

    if args.workload == "ppo":
        line = run_ppo(args, rank, world, local, dev)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    wl = WORKLOADS[args.workload]
    cfg = wl["cfg"]
    B, K, W = args.envs or wl["envs"], args.steps, args.warmup
    mode = "decima" if args.workload == "decima" else args.mode
    if host:
        sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))
        from driver import HostEngine  # TEST-ONLY host build (see --engine)

        eng = HostEngine(cfg, B, generate(args.dataset_seed))
        args.lockstep = True  # the host build has no shared-budget launch
    else:
        from spark_sched_sim.engine import DeviceEngine

        eng = DeviceEngine(cfg, B, generate(args.dataset_seed), device=dev,
                           config_flags=_abi.SSIM_CFG_FORCE_HBM if args.force_hbm else 0)
    seeds = shard_seeds(rank, B, args.seed)
    limits = None
    if wl["mean_time_limit"]:  # StochasticTimeLimit (wrappers/stochastic_time_limit.py:5-31), per env
        from spark_sched_sim.wrappers import StochasticTimeLimitSampler

        smp = StochasticTimeLimitSampler(wl["mean_time_limit"], B, seed=42)
        limits = np.array([smp.sample(i, int(seeds[i])) for i in range(B)], dtype=np.float64)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=limits)
    if limits is not None and not host:
        limits = torch.tensor(limits, dtype=torch.float64, device=dev)
    kind = _abi.SSIM_POLICY_RANDOM
    stream = None if host else torch.cuda.current_stream(dev)
    flags = 0 if args.no_autoreset else _abi.SSIM_ROLLOUT_AUTORESET

    # 2. pre-roll: spread the batch over the phases of its episodes (seeded per rank)
    preroll = wl["preroll"] if args.preroll < 0 else args.preroll
    pre_steps = np.zeros(B, dtype=np.int32)
    if preroll > 0 and mode != "step":
        pre_steps = np.random.default_rng([args.seed, rank, 7]).integers(0, preroll, B).astype(np.int32)
        eng.rollout_steps(kind, 4321, pre_steps, int(pre_steps.max()) + 1,
                          flags=_abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_WARMUP, time_limits=limits)
    elif preroll > 0:  # step mode: the same spread through the fused launch, then per-step launches
        pre_steps = np.random.default_rng([args.seed, rank, 7]).integers(0, preroll, B).astype(np.int32)
        eng.rollout_steps(kind, 4321, pre_steps, int(pre_steps.max()) + 1, flags=_abi.SSIM_ROLLOUT_WARMUP,
                          time_limits=limits)

    if mode == "decima":
        from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

        torch.manual_seed(args.seed)
        pol = DecimaScheduler(cfg["num_executors"]).to(dev)  # decima_tpch.yaml:66-78 dims, random init
        gen = torch.Generator(device=dev).manual_seed(args.seed)
        cnt = eng.views["counts"]
        packed = pol.packed_params(dev)  # fixed weights during rollouts: packed once, like RolloutCollector
        overflow_total = torch.zeros((), dtype=torch.int64, device=dev)

    def rollout_launch(c, timed):
        f = flags | (0 if timed or host else _abi.SSIM_ROLLOUT_WARMUP)  # warm-up launches: k_rollout_warmup symbol
        if args.lockstep:
            eng.rollout(kind, 1234, c, flags=f, time_limits=limits)
        else:  # the same B x c decisions, claimed by whichever env is ready; preemptible at event boundaries
            pre = 0 if args.no_preempt else _abi.SSIM_ROLLOUT_PREEMPT
            eng.rollout_budget(kind, 1234, 8 * c, B * c, flags=f | pre, time_limits=limits)

    # configs[2] default: the persistent Decima rollout (features + fused policy + step per env in one launch), a
    # shared budget of B x c decisions per launch, preemptible, auto-reset (the tpch rollout's work sharing)
    persistent = mode == "decima" and not (args.decima_lockstep or args.torch_policy or host)

    def decima_launch(c, timed):
        f = _abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_PREEMPT | (0 if timed else _abi.SSIM_ROLLOUT_WARMUP)
        eng.decima_rollout(packed, args.seed, 1, 8 * c, B * c, flags=f, time_limits=limits)

    def launch_sizes(n, chunk=None):
        chunk = chunk or n
        return [chunk] * (n // chunk) + ([n % chunk] if n % chunk else [])

    def run(n, events=None, chunk=None):
        """n steps; `events` (pre-created HIP event pairs, one per kernel launch) bracket each launch on the launch
        stream."""
        if n <= 0:
            return
        if mode == "rollout" or persistent:
            for i, c in enumerate(launch_sizes(n, chunk)):
                if events is not None:
                    events[i][0].record(stream)
                (decima_launch if persistent else rollout_launch)(c, events is not None)
                if events is not None:
                    events[i][1].record(stream)
            return
        for k in range(n):
            if mode == "decima":
                if args.torch_policy:  # the batched PyTorch module (~150 launches per decision)
                    act = pol.schedule(build_batch(eng.views, eng.decima_features()), generator=gen)
                else:  # one fused HIP launch (ssim_decima_policy)
                    run.counter += 1
                    act = pol.schedule_fused(eng, eng.decima_features(), seed=args.seed, counter=run.counter,
                                             params=packed)
                    overflow_total.add_(act["overflow"].sum().to(torch.int64))
                si, ne = act["stage_idx"], act["num_exec"]
            else:
                si, ne = eng.policy(kind, 1234, run.counter)
                run.counter += 1
            if events is not None:
                events[k][0].record(stream)
            eng.step(si, ne)
            if events is not None:
                events[k][1].record(stream)
            if mode == "decima":
                done = ((cnt[:, _abi.OC_TERMINATED] != 0) | (cnt[:, _abi.OC_TRUNCATED] != 0)).to(torch.uint8)
                eng.reset_sampled(done, time_limits=limits)  # finished episodes: reset(seed=None) on device
    run.counter = 0

    # 3. warm-up: exactly W steps
    run(W)
    sync()
    acc0 = np.array(eng.to_numpy(eng.views["acc"]), dtype=np.int64).copy()
    events = None
    if not host:  # created before the timed region (event creation is host work, not part of a step)
        n_launch = len(launch_sizes(K, args.chunk or K)) if (mode == "rollout" or persistent) else K
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(n_launch)]
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run(K, events, args.chunk or K)  # 4. timed: exactly K steps
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    v = eng.host_views()
    counts1 = np.array(v["counts"])
    acc1 = np.array(v["acc"], dtype=np.int64)
    errs = int(np.count_nonzero(counts1[:, _abi.OC_ERR] & _abi.SSIM_ERR_STICKY))
    d_acc = (acc1 - acc0).sum(axis=0).astype(np.float64)  # S_act, E_act, J_act, events, decisions, episodes
    decisions = float(d_acc[_abi.ACC_DECISIONS])  # over all episodes (auto-reset restarts the per-episode count)
    episodes_done = float(d_acc[_abi.ACC_EPISODES])
    # B_dec = 36 S_act + 20 E_act + 16 J_act + 96 K + 40 bytes per decision
    alg_bytes = 36 * d_acc[0] + 20 * d_acc[1] + 16 * d_acc[2] + 96 * d_acc[3] + 40 * decisions
    launches = len(events) if events is not None else 0
    kern_ms = sum(a.elapsed_time(b) for a, b in events) if events else 0.0
    elapsed = t1 - t0
    stats = torch.tensor([elapsed, decisions, alg_bytes, kern_ms, float(errs), episodes_done, float(d_acc[3])],
                         dtype=torch.float64, device=dev)
    # what each rank measured (gathered off the timed path), so a multi-GPU line shows how many ranks the process
    # group held and that the per-rank decisions add up to the total
    per_rank = gather_env_stats(torch.tensor([[float(rank), elapsed, decisions, kern_ms]], dtype=torch.float64,
                                             device=dev), world).cpu().tolist()
    ranks_seen = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    stats = reduce_timing(stats, world)
    mine = torch.tensor(counts1[:, [_abi.OC_NUM_COMPLETED, _abi.OC_NUM_ARRIVED, _abi.OC_DECISIONS]],
                        dtype=torch.int32, device=dev)
    gathered = gather_env_stats(mine, world)  # episode statistics gather (off the timed path)
    elapsed, decisions, alg_bytes, kern_ms_sum, errs, episodes_done, events_sum = stats.tolist()
    overflow = int(overflow_total.item()) if mode == "decima" and not args.torch_policy else 0
    value = decisions / elapsed
    line = None
    if rank == 0:
        kernel = "k_rollout" if mode == "rollout" else "k_decima_rollout" if persistent else "k_step"
        roofline = None
        if not host and launches:
            kern_ms = kern_ms_sum / world
            achieved = (alg_bytes / world / launches) / (kern_ms / launches / 1e3) / 1e9  # GB/s per GPU
            traffic, traffic_src, pmc = pmc_traffic(kernel, mode, B, K if (mode == "rollout" or persistent) else 1,
                                                   decisions / world / launches, args.dataset_seed, build_id)
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                        "kernel": kernel, "kernel_ms_per_launch": kern_ms / launches,
                        "alg_bytes_per_launch": alg_bytes / world / launches}
            if traffic is None:
                roofline["traffic_note"] = f"no committed PMC summary of build {build_id} for this config"
            else:
                roofline["traffic_over_algorithmic"] = traffic / (alg_bytes / world / launches)
            if pmc is not None and "issue" in pmc:
                # the bound that binds: instruction issue of one wave per SIMD
                iss = dict(pmc["issue"])
                iss["decisions_per_s_per_simd"] = decisions / elapsed / world / pmc["issue"].get("simds", 1024)
                roofline["issue"] = iss
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
                "Decima GNN policy, random-init weights" if mode == "decima" else "random valid actions (device RNG)"),
            "build_id": build_id,
            "config": {"workload": wl["desc"].format(B=B), "envs_per_gpu": B,
                       "jobs": cfg["job_arrival_cap"], "executors": cfg["num_executors"],
                       "mean_time_limit": wl["mean_time_limit"], "mode": mode,
                       "policy": ("torch" if args.torch_policy else "persistent Decima rollout (features + fused "
                                  "policy + step per env in one launch)" if persistent else "fused HIP kernel")
                       if mode == "decima" else "device random",
                       "steps_per_launch": (args.chunk or K) if (mode == "rollout" or persistent) else 1,
                       "work_sharing": ("lockstep" if args.lockstep else "shared budget of envs x steps "
                                        "decisions per launch" + ("" if args.no_preempt else
                                                                  ", preemptible at event boundaries"))
                       if (mode == "rollout" or persistent) else None,
                       "preroll": {"bound": preroll, "mean_decisions": float(pre_steps.mean())},
                       "autoreset": bool(mode != "step" and (flags or mode == "decima")),
                       "parallelism": f"env-sharded x{world}",
                       "residency": "LDS" if int(eng.layout.lds_resident) else "HBM",
                       "dataset": {"generator": "synthetic_tpch", "seed": args.dataset_seed,
                                   "stage_cap": int(eng.layout.stage_cap),
                                   "kernel": ("shape-specialised (stage cap 900)" if int(eng.layout.stage_cap) == 900
                                              and cfg["num_executors"] == 10 and cfg["job_arrival_cap"] == 50
                                              else "stage cap read at run time")}},
            "decisions": int(decisions),
            "episodes_finished": int(episodes_done),
            "events_per_decision": events_sum / max(decisions, 1.0),
            "terminated_envs": int((counts1[:, _abi.OC_TERMINATED] != 0).sum()),
            "frozen_envs": int(errs),
            "jobs_completed": int(gathered[:, 0].sum().item()),
            "jobs_arrived": int(gathered[:, 1].sum().item()),
            "ranks_seen": ranks_seen,
            "per_rank": [{"rank": int(r), "elapsed_s": e, "decisions": int(d), "kernel_ms": k}
                         for r, e, d, k in per_rank],
            "roofline": roofline,
            "cpu_baseline": None,
        }
        if mode == "decima":
            line["policy_overflow_envs"] = overflow
        if host:
            line["engine"] = "hostsim (TEST-ONLY CPU build; not a measurement)"
        if not args.no_cpu_baseline and world == 1 and not host and args.workload in ("tpch", "large", "decima"):
            procs = args.cpu_procs or usable_cpus()
            line["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds, procs, ds_seed=args.dataset_seed)
            add_ratios(line["cpu_baseline"], value)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if mode == "decima" and overflow:
        raise SystemExit(f"fused Decima policy skipped {overflow} env-steps (LDS node cap overflow)")


if __name__ == "__main__":
    main()
