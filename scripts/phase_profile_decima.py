#!/usr/bin/env python
"""Diagnostic: per-phase shader-clock breakdown of the persistent Decima rollout (configs[2], bench.py --workload
decima's sequence) from the separate -DSSIM_PROFILE build (never the measured product): the engine phases plus the
Decima action driver's features / fused policy / sample copy (engine.h kPhDecFeat..)."""

import ctypes as ct
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
sys.path.insert(0, os.path.join(REPO, "scripts"))


def main():
    import numpy as np
    import torch

    import phase_profile as PP
    from spark_sched_sim import _abi, native
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import shard_seeds
    from spark_sched_sim.schedulers.decima import DecimaScheduler
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    native._lib = None
    native.LIB_PATH = PP.build_prof()
    from spark_sched_sim.engine import DeviceEngine

    lib = native.lib()
    lib.ssim_decima_profile_next.argtypes = [ct.c_void_p, ct.c_void_p]
    cfg = {"num_executors": 50, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}  # bench.py DECIMA_ENV
    B = int(os.environ.get("PROF_ENVS", "4096"))
    K = int(os.environ.get("PROF_STEPS", "40"))
    dev = torch.device("cuda:0")
    eng = DeviceEngine(cfg, B, generate(0), device=dev)
    seeds = shard_seeds(0, B, 0)
    smp = StochasticTimeLimitSampler(2.0e7, B, seed=42)
    lim = np.array([smp.sample(i, int(seeds[i])) for i in range(B)], dtype=np.float64)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=lim)
    limits = torch.tensor(lim, dtype=torch.float64, device=dev)
    pre = np.random.default_rng([0, 0, 7]).integers(0, 1500, B).astype(np.int32)
    AR, PRE, WU = _abi.SSIM_ROLLOUT_AUTORESET, _abi.SSIM_ROLLOUT_PREEMPT, _abi.SSIM_ROLLOUT_WARMUP
    eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, int(pre.max()) + 1, flags=AR | WU, time_limits=limits)
    torch.manual_seed(0)
    packed = DecimaScheduler(50).to(dev).packed_params(dev)
    eng.decima_rollout(packed, 0, 1, 8 * 5, B * 5, flags=AR | PRE | WU, time_limits=limits)
    torch.cuda.synchronize()
    acc = eng.views["acc"]
    d0, e0 = acc[:, _abi.ACC_DECISIONS].sum().item(), acc[:, 3].sum().item()
    prof = torch.zeros((B, PP.NUM_SLOTS), dtype=torch.int64, device=dev)
    native.check(lib.ssim_decima_profile_next(eng.handle, prof.data_ptr()), "ssim_decima_profile_next")
    eng.decima_rollout(packed, 0, 1, 8 * K, B * K, flags=AR | PRE, time_limits=limits)
    torch.cuda.synchronize()
    dec = acc[:, _abi.ACC_DECISIONS].sum().item() - d0
    ev = acc[:, 3].sum().item() - e0
    p = prof.cpu().numpy().astype(np.float64)
    tot = p.sum(axis=0)
    names = PP.PHASES + ["(stamp)"] * PP.NSTAMPS + PP.DEC_PHASES + PP.DEC_PARTS
    top = tot[:PP.TOP].sum()
    it = tot[PP.PHASES.index("(loop iterations)")]
    print(f"== decima persistent rollout, B={B}, K={K}: decisions {dec}, events {ev} ({ev / dec:.2f}/decision)")
    print(f"  {'whole loop iterations':24s} {it / dec:10.1f} cycles/decision")
    res = {}
    for i, name in enumerate(names):
        if name == "(stamp)" or name.startswith("#decisions"):
            continue
        v = tot[i] / dec
        res[name] = v
        if name.startswith("#"):
            print(f"  {name:24s} {v:10.3f} per decision")
        else:
            print(f"  {name:24s} {v:10.1f} cycles/decision  {100 * tot[i] / it:5.1f}% of loop")
    st = p[:, len(PP.PHASES):len(PP.PHASES) + PP.NSTAMPS]
    ent, loaded, loop_end, saved = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    t0 = ent.min()
    wall = {"entry_spread_us": float((ent.max() - t0) / 100.0), "loop_us_mean": float(((loop_end - loaded) / 100.0).mean()),
            "last_wave_end_us": float((saved.max() - t0) / 100.0), "first_wave_end_us": float((saved.min() - t0) / 100.0)}
    print("  wave timeline (us):", json.dumps({k: round(v, 2) for k, v in wall.items()}))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "phase_profile_decima.json"), "w") as f:
        json.dump({"decisions": dec, "cycles_per_decision": res, "wave_timeline_us": wall}, f, indent=1)


if __name__ == "__main__":
    main()
