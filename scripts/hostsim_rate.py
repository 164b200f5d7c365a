#!/usr/bin/env python
"""Secondary CPU baseline (SURVEY.md §8d "also report the single-thread C++ engine"): decisions/s of the engine's
own source (csrc/engine.h, policy.h) compiled for the host with g++ -O2 (the TEST-ONLY tests/hostsim build, one lane
per wave), single-threaded, on bench.py's configs[1] workload: 50 TPC-H jobs / 10 executors, random valid actions,
episodes restarted in place (auto-reset). Not the product and not bench.py's `cpu_baseline` (which times the
reference-structured Python restatement, `kind: port`): it says what one CPU core does with the same algorithm and
data layout as one GPU wave. Prints one JSON line."""

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))


def main():
    import numpy as np

    from driver import HostEngine
    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import shard_seeds

    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    cfg = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}  # bench.py ENV_CFG (examples.py:15-23)
    B, K = 64, 50
    eng = HostEngine(cfg, B, generate(0))
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=shard_seeds(0, B, 0))
    kind = _abi.SSIM_POLICY_RANDOM
    eng.rollout(kind, 4321, K, flags=_abi.SSIM_ROLLOUT_AUTORESET)  # warm-up
    d0 = int(np.asarray(eng.host_views()["acc"])[:, _abi.ACC_DECISIONS].sum())
    t0 = time.perf_counter()
    launches = 0
    while time.perf_counter() - t0 < seconds:
        eng.rollout(kind, 1234 + launches, K, flags=_abi.SSIM_ROLLOUT_AUTORESET)
        launches += 1
    dt = time.perf_counter() - t0
    v = eng.host_views()
    acc = np.asarray(v["acc"])
    dec = int(acc[:, _abi.ACC_DECISIONS].sum()) - d0
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    print(json.dumps({"what": "single-thread host build of csrc/engine.h (tests/hostsim, g++ -O2), configs[1] workload",
                      "value": dec / dt, "unit": "decisions/s", "cores": 1, "decisions": dec, "seconds": dt,
                      "envs": B, "episodes": int(acc[:, _abi.ACC_EPISODES].sum()), "cpu_model": cpu}))


if __name__ == "__main__":
    main()
