#!/usr/bin/env python
"""Diagnostic: wall-time split of one Decima decision step (featurise, flat batch, encoder, stage scores +
sampling, exec scores, env step) at several env counts (BASELINE configs[2] env section)."""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))


def main():
    import torch

    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine
    from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

    cfg = {"num_executors": 50, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}
    ds = generate(0)
    for B in [int(x) for x in os.environ.get("PROF_ENVS", "16,4096").split(",")]:
        eng = DeviceEngine(cfg, B, ds)
        eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=list(range(B)), time_limits=[2e7] * B)
        pol = DecimaScheduler(50).cuda()
        g = torch.Generator(device="cuda").manual_seed(0)
        tm = {k: 0.0 for k in ("features", "batch", "schedule", "step")}
        n = 30
        for it in range(n + 5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f = eng.decima_features()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            b = build_batch(eng.views, f)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            act = pol.schedule(b, generator=g)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            eng.step(act["stage_idx"], act["num_exec"])
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            if it >= 5:
                for k, v in zip(tm, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                    tm[k] += v
        print(B, "envs:", {k: f"{v / n * 1e3:.2f} ms" for k, v in tm.items()}, "nodes", b.x.shape[0],
              "levels", b.max_levels, flush=True)
        tf = 0.0
        for it in range(n + 5):  # fused kernel path (ssim_decima_policy)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fo = pol.schedule_fused(eng, eng.decima_features(), seed=1, counter=it)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            eng.step(fo["stage_idx"], fo["num_exec"])
            if it >= 5:
                tf += t1 - t0
        print(B, "envs: fused features+schedule", f"{tf / n * 1e3:.2f} ms", flush=True)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                torch.profiler.ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                act = pol.schedule(build_batch(eng.views, eng.decima_features()), generator=g)
                eng.step(act["stage_idx"], act["num_exec"])
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
