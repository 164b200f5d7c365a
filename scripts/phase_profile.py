#!/usr/bin/env python
"""Diagnostic: per-phase shader-clock breakdown of the fused rollout kernel (separate -DSSIM_PROFILE build,
never the measured product). Prints cycles per decision per phase, averaged over waves, plus an
env-count sweep of the product kernel (occupancy / latency-hiding check)."""

import ctypes as ct
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))

PHASES = ["policy", "action", "round_check", "fulfill", "pop", "handle", "post_scan", "observe",
          "(sample)", "(pool ops)", "(scans)", "(hot load/save)", "(big-table staging)", "(idle_order)",
          "(duration draw)", "(job arrival)", "(executor arrival)", "(task done)", "(stage completion)",
          "#small-table ops", "#big-table ops", "#task launches", "#idle_order"] + [
          f"#decisions {1 << (b + 10)}-{1 << (b + 11)} cycles" for b in range(16)]
TOP = 8  # the first TOP phases are disjoint; the rest are inclusive sub-timers
NSTAMPS = 6  # engine.h kTEntry, kTLoaded, kTLoopEnd, kTSaved, kTCtor, kTCopy1


def build_prof():
    out = os.path.join(REPO, "gym-sparksched_amd", "build", "libsparksched_prof.so")
    if os.path.exists(out) and "--build" not in sys.argv:
        return out  # prebuilt in-tree (build on the CPU container: `python scripts/phase_profile.py --build`)
    import __graft_entry__

    return __graft_entry__.build_lib(force=True, out=out, defines=["-DSSIM_PROFILE"])


def main():
    import numpy as np
    import torch

    from spark_sched_sim import _abi, native
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine

    cfg = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}
    ds = generate(0)
    K = int(os.environ.get("PROF_STEPS", "300"))
    res = {}
    # 1) product kernel: env-count sweep
    for B in (256, 1024, 2048, 4096, 8192):
        eng = DeviceEngine(cfg, B, ds)
        eng.reset(seeds=list(range(B)))
        eng.rollout(_abi.SSIM_POLICY_RANDOM, 1, 20)
        torch.cuda.synchronize()
        d0 = eng.views["counts"][:, _abi.OC_DECISIONS].sum().item()
        t = time.perf_counter()
        eng.rollout(_abi.SSIM_POLICY_RANDOM, 1, K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        d1 = eng.views["counts"][:, _abi.OC_DECISIONS].sum().item()
        res[f"sweep_B{B}"] = {"decisions_per_s": (d1 - d0) / dt, "ms": dt * 1e3}
        print(B, "envs:", f"{(d1 - d0) / dt:.3e} decisions/s", f"{dt * 1e3:.1f} ms", flush=True)
        eng.close()
    # 2) diagnostic build: phase breakdown at B=1024
    lib = ct.CDLL(build_prof())
    lib.ssim_rollout_profiled.argtypes = [ct.c_void_p, ct.c_int32, ct.c_uint64, ct.c_int32, ct.c_void_p, ct.c_void_p]
    native._lib = None
    native.LIB_PATH = os.path.join(REPO, "gym-sparksched_amd", "build", "libsparksched_prof.so")
    B = 1024
    eng = DeviceEngine(cfg, B, ds)
    # the bench's batch: device reset, then a seeded pre-roll over the episodes' phases (bench.py step 2)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=list(range(B)))
    pre = np.random.default_rng([0, 0, 7]).integers(0, 1000, B).astype(np.int32)
    eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, 1001, flags=_abi.SSIM_ROLLOUT_AUTORESET)
    torch.cuda.synchronize()
    acc = eng.views["acc"]
    d0 = acc[:, _abi.ACC_DECISIONS].sum().item()
    e0 = acc[:, 3].sum().item()
    # per env: the phase sums, then NSTAMPS s_memrealtime stamps (engine.h kTEntry..kTCopy1)
    prof = torch.zeros((B, len(PHASES) + NSTAMPS), dtype=torch.int64, device=eng.device)
    lib.ssim_rollout_profiled(eng.handle, _abi.SSIM_POLICY_RANDOM, 1, K, prof.data_ptr(), eng._stream())
    torch.cuda.synchronize()
    d1 = acc[:, _abi.ACC_DECISIONS].sum().item()
    e1 = acc[:, 3].sum().item()
    p = prof[:, :len(PHASES)].cpu().numpy().astype(np.float64)  # s_memtime ticks = shader cycles
    dec = d1 - d0
    tot = p.sum(axis=0)
    print(f"decisions {dec}, events {e1 - e0} ({(e1 - e0) / dec:.2f}/decision)")
    top = tot[:TOP].sum()
    for name, v in zip(PHASES, tot):
        if name.startswith("#decisions"):
            print(f"  {name:32s} {v / dec * 100:8.3f}% of decisions")
        else:
            print(f"  {name:16s} {v / dec:10.1f} cycles/decision  {100 * v / top:5.1f}%")
    res["phases_ticks_per_decision"] = {n: float(v / dec) for n, v in zip(PHASES, tot)}
    res["events_per_decision"] = (e1 - e0) / dec
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "phase_profile.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if "--build" in sys.argv:
        print(build_prof())
    else:
        main()
