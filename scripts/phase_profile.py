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
          "(loop iterations)",
          "#small-table ops", "#big-table ops", "#task launches", "#idle_order"] + [
          f"#decisions {1 << (b + 10)}-{1 << (b + 11)} cycles" for b in range(16)]
TOP = 8  # the first TOP phases are disjoint; the rest are inclusive sub-timers
NSTAMPS = 6  # engine.h kTEntry, kTLoaded, kTLoopEnd, kTSaved, kTCtor, kTCopy1
DEC_PHASES = ["(decima features)", "(decima policy)", "(decima sample copy)"]  # engine.h kPhDecFeat.. (inside policy)
DEC_PARTS = ["[policy setup]", "[policy prep MLPs]", "[policy message passing]", "[policy DAG/global summaries]",
             "[policy stage scores]", "#nodes", "#edges", "#levels", "#schedulable", "[policy exec scores]"]
RESET_SLOTS = ["(auto-resets)", "#auto-resets"]  # engine.h kPhReset, kCtReset
NUM_SLOTS = 40 + NSTAMPS + len(DEC_PHASES) + len(DEC_PARTS) + len(RESET_SLOTS)  # engine.h kNumPhases


def build_prof():
    out = os.path.join(REPO, "gym-sparksched_amd", "build", "libsparksched_prof.so")
    if os.environ.get("SSIM_PROF_LIB"):  # another prebuilt diagnostic variant (e.g. -DSSIM_PROFILE_FINE)
        return os.environ["SSIM_PROF_LIB"]
    if os.path.exists(out) and "--build" not in sys.argv:
        return out  # prebuilt in-tree (build on the CPU container: `python scripts/phase_profile.py --build`)
    import __graft_entry__

    return __graft_entry__.build_lib(out=out, defines=["-DSSIM_PROFILE"])


def main():
    """The bench's own sequence (bench.py main, workload tpch): device reset, the seeded pre-roll with auto-reset,
    W warm-up budget launches of K steps, then ONE profiled budget launch of K steps with PREEMPT | AUTORESET, for
    K = 20 (the driver's --steps 20) and K = 300 (bench.py's default)."""
    import numpy as np
    import torch

    from spark_sched_sim import _abi, native
    from spark_sched_sim.data_samplers.synthetic_tpch import generate

    import bench
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    # PROF_WORKLOAD: one of bench.py's heuristic-policy workloads (tpch = configs[1], large = the configs[3] shard)
    wl = bench.WORKLOADS[os.environ.get("PROF_WORKLOAD", "tpch")]
    cfg = dict(wl["cfg"])
    ds = generate(int(os.environ.get("PROF_DATASET", "0")))
    B = int(os.environ.get("PROF_ENVS", wl["envs"]))
    limits = None
    if wl["mean_time_limit"]:
        smp = StochasticTimeLimitSampler(wl["mean_time_limit"], B, seed=42)
        limits = np.array([smp.sample(i, i) for i in range(B)], dtype=np.float64)
    native._lib = None
    native.LIB_PATH = build_prof()
    from spark_sched_sim.engine import DeviceEngine

    lib = native.lib()
    lib.ssim_rollout_budget_profiled.argtypes = [ct.c_void_p, ct.c_int32, ct.c_uint64, ct.c_int32, ct.c_int64,
                                                 ct.c_int32, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    res = {}
    flags = _abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_PREEMPT
    for K in [int(k) for k in os.environ.get("PROF_STEPS", "20,300").split(",")]:
        eng = DeviceEngine(cfg, B, ds)
        eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=list(range(B)), time_limits=limits)
        pre = np.random.default_rng([0, 0, 7]).integers(0, wl["preroll"], B).astype(np.int32)
        eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, int(pre.max()) + 1,
                          flags=_abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_WARMUP, time_limits=limits)
        for _ in range(int(os.environ.get("PROF_WARMUP", "5"))):
            eng.rollout_budget(_abi.SSIM_POLICY_RANDOM, 1234, 8 * K, B * K, flags=flags | _abi.SSIM_ROLLOUT_WARMUP,
                               time_limits=limits)
        torch.cuda.synchronize()
        acc = eng.views["acc"]
        d0 = acc[:, _abi.ACC_DECISIONS].sum().item()
        e0 = acc[:, 3].sum().item()
        prof = torch.zeros((B, NUM_SLOTS), dtype=torch.int64, device=eng.device)
        tl = None if limits is None else torch.as_tensor(limits, device=eng.device)
        rc = lib.ssim_rollout_budget_profiled(eng.handle, _abi.SSIM_POLICY_RANDOM, 1234, 8 * K, B * K, flags,
                                              prof.data_ptr(), None if tl is None else tl.data_ptr(), eng._stream())
        native.check(rc, "ssim_rollout_budget_profiled")
        torch.cuda.synchronize()
        d1 = acc[:, _abi.ACC_DECISIONS].sum().item()
        e1 = acc[:, 3].sum().item()
        p = prof[:, :len(PHASES)].cpu().numpy().astype(np.float64)  # s_memtime ticks = shader cycles
        st = prof[:, len(PHASES):len(PHASES) + NSTAMPS].cpu().numpy().astype(np.float64)  # 100 MHz stamps
        eng.close()
        dec = d1 - d0
        tot = p.sum(axis=0)
        top = tot[:TOP].sum()
        it = tot[PHASES.index("(loop iterations)")]
        print(f"== K={K}: decisions {dec}, events {e1 - e0} ({(e1 - e0) / dec:.2f}/decision)")
        print(f"  {'sum of top-level phases':24s} {top / dec:10.1f} cycles/decision")
        print(f"  {'whole loop iterations':24s} {it / dec:10.1f} cycles/decision (top-level phases cover "
              f"{100 * top / it:.1f}%)")
        for name, v in zip(PHASES, tot):
            if name.startswith("#decisions"):
                print(f"  {name:32s} {v / dec * 100:8.3f}% of decisions")
            elif name.startswith("#"):
                print(f"  {name:24s} {v / dec:10.3f} per decision")
            else:
                print(f"  {name:24s} {v / dec:10.1f} cycles/decision  {100 * v / top:5.1f}% of top-level")
        rs = prof[:, NUM_SLOTS - 2:].cpu().numpy().astype(np.float64).sum(axis=0)
        print(f"  {'(auto-resets)':24s} {rs[0] / dec:10.1f} cycles/decision; {int(rs[1])} resets, "
              f"{rs[0] / max(rs[1], 1):.0f} cycles each")
        # per-wave wall clock of the launch from the realtime stamps (10 ns ticks)
        ent, loaded, loop_end, saved = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
        t0 = ent.min()
        ends = (saved - t0) / 100.0
        wall = {"wave_end_us_p50": float(np.percentile(ends, 50)), "wave_end_us_p90": float(np.percentile(ends, 90)),
                "wave_end_us_p99": float(np.percentile(ends, 99)),
                "entry_spread_us": float((ent.max() - t0) / 100.0),
                "load_hot_us_mean": float(((loaded - ent) / 100.0).mean()),
                "loop_us_mean": float(((loop_end - loaded) / 100.0).mean()),
                "save_hot_us_mean": float(((saved - loop_end) / 100.0).mean()),
                "last_wave_end_us": float((saved.max() - t0) / 100.0),
                "first_wave_end_us": float((saved.min() - t0) / 100.0)}
        print("  wave timeline (us):", json.dumps({k: round(v, 2) for k, v in wall.items()}))
        res[f"K{K}"] = {"decisions": dec, "events_per_decision": (e1 - e0) / dec,
                        "cycles_per_decision": {n: float(v / dec) for n, v in zip(PHASES, tot)},
                        "top_level_sum": float(top / dec), "loop_iterations": float(it / dec),
                        "wave_timeline_us": wall}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "phase_profile.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if "--build" in sys.argv:
        print(build_prof())
    else:
        main()
