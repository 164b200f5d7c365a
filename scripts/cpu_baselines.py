#!/usr/bin/env python
"""CPU baselines of every BASELINE.json config, timed on this host's cores: the reference's CPU
rollout path restated by the oracle (oracle/restatement.py with the same CPython set/dict/heapq and numpy
Generator machinery), in the trainers/rollout_worker.py harness shape (spawn processes, one env each, one
thread), 1-episode warm-up, then decisions counted over `--seconds` of wall time.

  configs[0] examples.py --sched fair   1 process (the reference example is single-process)
  configs[1] 1024 envs J=50 N=10 random  P = usable CPUs
  configs[2] Decima J=200 N=50           P = usable CPUs (Decima GNN on the CPU, per-observation, as the
                                          reference's rollout workers run it)
  configs[3] J=200 N=100 random, limits  P = usable CPUs
  configs[4] PPO decima_tpch.yaml        16 processes (4 sequences x 4 rollouts, trainer.py:264-296): the
                                          rollout phase only, an upper bound on the reference iteration's
                                          decisions/s (its learner time is not included)
Writes gpurun_out/cpu_baselines.json.
"""

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--only", default="", help="comma-separated subset of configs0..configs4")
    args = ap.parse_args()
    P = bench.usable_cpus()
    plan = {"configs0": ("examples", 1), "configs1": ("tpch", P), "configs2": ("decima", P),
            "configs3": ("large", P), "configs4": ("decima", 16)}
    only = [x for x in args.only.split(",") if x]
    out = {"host_cpus": os.cpu_count(), "usable_cpus": P, "cpu_model": bench.cpu_model(), "results": {}}
    for name, (wl, procs) in plan.items():
        if only and name not in only:
            continue
        r = bench.cpu_baseline(wl, args.seconds, procs)
        r["workload"] = wl
        out["results"][name] = r
        print(name, wl, procs, f"{r['value']:.1f} decisions/s", f"({r['per_core']:.1f}/core)", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "cpu_baselines.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
