"""Episode runner and CLI of the reference's `examples.py` on the MI355X engine.

`run_episode(env_cfg, scheduler, seed)` is `examples.py:84-102`: one `SparkSchedSimEnv` episode (each step is
a gfx950 kernel launch through the C ABI) driven by a host scheduler's `schedule(obs)`, returning the
average job duration in seconds (`metrics.avg_job_duration(env) * 1e-3`).

    python -m spark_sched_sim.examples --sched fair      # examples.py --sched fair (BASELINE configs[0])
"""

from __future__ import annotations

from argparse import ArgumentDefaultsHelpFormatter, ArgumentParser
from pprint import pprint

from . import metrics
from .env import SparkSchedSimEnv
from .schedulers import RandomScheduler, RoundRobinScheduler

ENV_CFG = {  # examples.py:15-23, without the pygame renderer
    "num_executors": 10,
    "job_arrival_cap": 50,
    "job_arrival_rate": 4.0e-5,
    "moving_delay": 2000.0,
    "warmup_delay": 1000.0,
    "data_sampler_cls": "TPCHDataSampler",
}


def run_episode(env_cfg: dict, scheduler, seed: int = 1234, **env_kwargs) -> float:
    env = SparkSchedSimEnv(env_cfg, **env_kwargs)
    if getattr(scheduler, "env_wrapper_cls", None):
        env = scheduler.env_wrapper_cls(env)
    obs, _ = env.reset(seed=seed, options=None)
    terminated = truncated = False
    while not (terminated or truncated):
        action, _ = scheduler.schedule(obs)
        obs, _, terminated, truncated, _ = env.step(action)
    avg = metrics.avg_job_duration(env) * 1e-3
    env.close()
    return avg


def main(argv=None) -> None:
    parser = ArgumentParser(description=__doc__, formatter_class=ArgumentDefaultsHelpFormatter)
    parser.add_argument("--sched", choices=["fair", "fifo", "random"], required=True)
    parser.add_argument("--seed", type=int, default=1234)
    args = parser.parse_args(argv)
    n = ENV_CFG["num_executors"]
    scheduler = {"fair": lambda: RoundRobinScheduler(n, dynamic_partition=True),
                 "fifo": lambda: RoundRobinScheduler(n, dynamic_partition=False),
                 "random": lambda: RandomScheduler(42)}[args.sched]()
    print(f"Example: {scheduler.name} Scheduler")
    print("Env settings:")
    pprint(ENV_CFG)
    print("Running episode...")
    avg = run_episode(ENV_CFG, scheduler, seed=args.seed)
    print(f"Done! Average job duration: {avg:.1f}s", flush=True)


if __name__ == "__main__":
    main()
