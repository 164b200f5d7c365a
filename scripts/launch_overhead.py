#!/usr/bin/env python
"""Diagnostic: fixed cost of a budget rollout launch on the bench configuration (configs[1], 1024 envs pre-rolled
over their episodes). For K steps per launch: host-timed elapsed (sync, launch, sync, as bench.py times a step
window), the kernel's HIP-event time, and decisions; a least-squares fit time = fixed + K x per_step for both."""

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))


def main():
    import numpy as np
    import torch

    import bench
    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine

    B = 1024
    eng = DeviceEngine(bench.ENV_CFG, B, generate(0), device="cuda:0")
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=np.arange(B, dtype=np.uint64))
    pre = np.random.default_rng([0, 0, 7]).integers(0, 1000, B).astype(np.int32)
    eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, 1001,
                      flags=_abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_WARMUP)
    stream = torch.cuda.current_stream()
    flags = _abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_PREEMPT
    acc = eng.views["acc"]
    rows = []
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for K in [int(k) for k in os.environ.get("LO_STEPS", "1 2 5 10 20 40 80").split()]:
        for rep in range(int(os.environ.get("LO_REPS", "6"))):
            torch.cuda.synchronize()
            d0 = acc[:, _abi.ACC_DECISIONS].sum().item()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev[0].record(stream)
            eng.rollout_budget(_abi.SSIM_POLICY_RANDOM, 1234, 8 * K, B * K, flags=flags)
            ev[1].record(stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            d1 = acc[:, _abi.ACC_DECISIONS].sum().item()
            if rep == 0:
                continue  # first launch of a length: warm-up
            rows.append({"K": K, "elapsed_ms": (t1 - t0) * 1e3, "kernel_ms": ev[0].elapsed_time(ev[1]),
                         "decisions": d1 - d0})
        r = [x for x in rows if x["K"] == K]
        print(f"K={K:4d} elapsed {np.median([x['elapsed_ms'] for x in r]):.4f} ms  kernel "
              f"{np.median([x['kernel_ms'] for x in r]):.4f} ms  decisions {np.median([x['decisions'] for x in r]):.0f}",
              flush=True)
    Ks = np.array([x["K"] for x in rows], dtype=np.float64)
    fit = {}
    for key in ("elapsed_ms", "kernel_ms"):
        y = np.array([x[key] for x in rows])
        A = np.stack([np.ones_like(Ks), Ks], axis=1)
        (a, b), *_ = np.linalg.lstsq(A, y, rcond=None)
        fit[key] = {"fixed_ms": float(a), "per_step_ms": float(b)}
        print(f"{key}: fixed {a * 1e3:.1f} us + {b * 1e3:.2f} us/step", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "launch_overhead.json"), "w") as f:
        json.dump({"rows": rows, "fit": fit}, f, indent=1)
    eng.close()


if __name__ == "__main__":
    main()
