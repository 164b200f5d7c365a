#!/usr/bin/env python
"""Diagnostic (profile build, never the measured product): where a budget rollout launch's time goes — wave start
skew, hot-block load, the decision loop, the tail (waves finishing after the median wave), the hot-block save —
from per-wave s_memrealtime stamps (100 MHz chip clock), for K-step launches with and without preemption, on
the bench's configuration (1024 envs, pre-rolled over their episodes)."""

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
    from spark_sched_sim.engine import DeviceEngine

    lib = ct.CDLL(PP.build_prof())
    lib.ssim_rollout_budget_profiled.argtypes = [ct.c_void_p, ct.c_int32, ct.c_uint64, ct.c_int32, ct.c_int64,
                                                 ct.c_int32, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    native._lib = None
    native.LIB_PATH = os.path.join(REPO, "gym-sparksched_amd", "build", "libsparksched_prof.so")
    cfg = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}
    B = 1024
    nph = len(PP.PHASES) + PP.NSTAMPS
    res = {}
    for K in (20, 300):
        for preempt in (False, True):
            eng = DeviceEngine(cfg, B, generate(0))
            eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=list(range(B)))
            pre = np.random.default_rng(7).integers(0, 1000, B).astype(np.int32)
            eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, 1001, flags=_abi.SSIM_ROLLOUT_AUTORESET)
            flags = _abi.SSIM_ROLLOUT_AUTORESET | (_abi.SSIM_ROLLOUT_PREEMPT if preempt else 0)
            prof = torch.zeros((B, nph), dtype=torch.int64, device=eng.device)
            out = []
            for rep in range(4):  # rep 0 = warm-up launch (5 steps)
                k = 5 if rep == 0 else K
                prof.zero_()
                a0 = eng.views["acc"][:, _abi.ACC_DECISIONS].sum().item()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                lib.ssim_rollout_budget_profiled(eng.handle, _abi.SSIM_POLICY_RANDOM, 1234, 8 * k, B * k, flags,
                                                 prof.data_ptr(), None, eng._stream())
                ev[1].record()
                torch.cuda.synchronize()
                a1 = eng.views["acc"][:, _abi.ACC_DECISIONS].sum().item()
                if rep == 0:
                    continue
                p = prof.cpu().numpy()
                st = p[:, -PP.NSTAMPS:].astype(np.float64) * 10.0  # ns (100 MHz)
                entry, loaded, loopend, saved, ctor, copy1 = st.T
                t0 = entry.min()
                le = np.sort(loopend - t0)
                out.append({"event_ms": ev[0].elapsed_time(ev[1]), "decisions": a1 - a0,
                            "entry_skew_us": (entry.max() - t0) / 1e3,
                            "load_us_p50": float(np.median(loaded - entry)) / 1e3,
                            "ctor_us_p50": float(np.median(ctor - entry)) / 1e3,
                            "copy_fixed_us_p50": float(np.median(copy1 - ctor)) / 1e3,
                            "copy_live_us_p50": float(np.median(loaded - copy1)) / 1e3,
                            "loop_end_us_p10_p50_p90_max": [float(le[int(q * (B - 1))]) / 1e3 for q in (0.1, .5, .9, 1.0)],
                            "save_us_max": float((saved - loopend).max()) / 1e3,
                            "span_us": (saved.max() - t0) / 1e3})
            res[f"K{K}_{'preempt' if preempt else 'finish'}"] = out
            print(K, "preempt" if preempt else "finish", json.dumps(out[-1]), flush=True)
            eng.close()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "launch_profile.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
