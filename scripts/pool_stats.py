#!/usr/bin/env python
"""Diagnostic (host build, no GPU): what the engine's CPython-set operations and live stage windows look like on
bench.py's workloads. Runs the TEST-ONLY host build of csrc/engine.h (tests/hostsim, built here as a variant with
-DSSIM_POOL_STATS) with the device random policy and auto-reset, one decision per call, and prints per workload:
  * set operations per decision by kind (add / remove / idle order) and table size, with the mean keys held;
  * the live stage window (live_hi - scan_live_lo, what an LDS copy of the per-stage sections must cover), the
    active stages and active jobs, as percentiles over (env, decision) samples.
Usage: python scripts/pool_stats.py [workload ...] [--envs B] [--decisions K]"""

import argparse
import ctypes as ct
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tests", "hostsim", "_hostsim_poolstats.so")
os.environ["HOSTSIM_SO"] = SO
os.environ["HOSTSIM_FLAGS"] = "-DSSIM_POOL_STATS"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))


def main():
    import numpy as np

    import bench
    import driver
    from driver import HostEngine
    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import shard_seeds
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["tpch", "large", "decima"])
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--decisions", type=int, default=1500)
    args = ap.parse_args()
    L = driver.lib()
    L.hs_live_stats.argtypes = [ct.c_void_p, ct.c_void_p]
    L.hs_pool_stats.argtypes = [ct.c_void_p]
    out = {}
    for name in args.workloads:
        wl = bench.WORKLOADS[name]
        B = args.envs
        eng = HostEngine(dict(wl["cfg"]), B, generate(0))
        limits = None
        if wl["mean_time_limit"]:
            smp = StochasticTimeLimitSampler(wl["mean_time_limit"], B, seed=42)
            limits = np.array([smp.sample(e) for e in range(B)])
        eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=shard_seeds(0, B, 0), time_limits=limits)
        st = np.zeros((B, 4), dtype=np.int32)
        ps = np.zeros(96, dtype=np.int64)
        L.hs_pool_stats(ps.ctypes.data)  # (reset-time operations excluded)
        samples = []
        d0 = int(np.asarray(eng.host_views()["acc"])[:, _abi.ACC_DECISIONS].sum())
        for k in range(args.decisions):
            eng.rollout(_abi.SSIM_POLICY_RANDOM, 1234 + k, 1, flags=_abi.SSIM_ROLLOUT_AUTORESET, time_limits=limits)
            L.hs_live_stats(eng.handle, st.ctypes.data)
            samples.append(st.copy())
        dec = int(np.asarray(eng.host_views()["acc"])[:, _abi.ACC_DECISIONS].sum()) - d0
        L.hs_pool_stats(ps.ctypes.data)
        ops, keys = ps[:48].reshape(3, 16), ps[48:].reshape(3, 16)
        s = np.concatenate(samples).astype(np.float64)
        pct = lambda c: {p: float(np.percentile(s[:, c], p)) for p in (50, 90, 99, 100)}
        res = {"decisions": dec, "set_ops_per_decision": {}, "live_window": pct(0), "active_stages": pct(1),
               "active_jobs": pct(2)}
        for op, nm in enumerate(("add", "remove", "idle_order")):
            for b in range(16):
                if ops[op, b]:
                    res["set_ops_per_decision"][f"{nm}@{1 << b}"] = {
                        "per_decision": round(ops[op, b] / dec, 3), "mean_keys": round(keys[op, b] / ops[op, b], 2)}
        out[name] = res
        print(name, json.dumps(res, indent=1), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
