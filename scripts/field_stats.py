#!/usr/bin/env python
"""Diagnostic (host build, no GPU): wave-uniform reads of hot-block fields and records per decision, by section, on
bench.py's workloads (the dependent LDS round trips of the LDS-resident device kernel: each is ds_read -> wait ->
readfirstlane there). Runs the TEST-ONLY host build of csrc/engine.h (tests/hostsim) built as a variant with
-DSSIM_FIELD_STATS, random policy with auto-reset, one decision per env per call.
Usage: python scripts/field_stats.py [workload ...] [--envs B] [--decisions K]"""

import argparse
import ctypes as ct
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HOSTSIM_SO"] = os.path.join(REPO, "tests", "hostsim", "_hostsim_fieldstats.so")
os.environ["HOSTSIM_FLAGS"] = "-DSSIM_FIELD_STATS"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gym-sparksched_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))

SECTIONS = {0: "stage field", 1: "job field", 2: "job times", 3: "executor field", 4: "executor event field",
            5: "pool cfrom", 6: "stage recent duration", 10: "pool record", 11: "stage record", 12: "executor record",
            13: "commitment scan"}


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
    ap.add_argument("--decisions", type=int, default=500)
    args = ap.parse_args()
    L = driver.lib()
    L.hs_field_stats.argtypes = [ct.c_void_p]
    fs = np.zeros(16, dtype=np.int64)
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
        L.hs_field_stats(fs.ctypes.data)  # (reset-time reads excluded)
        d0 = int(np.asarray(eng.host_views()["acc"])[:, _abi.ACC_DECISIONS].sum())
        for k in range(args.decisions):
            eng.rollout(_abi.SSIM_POLICY_RANDOM, 1234 + k, 1, flags=_abi.SSIM_ROLLOUT_AUTORESET, time_limits=limits)
        dec = int(np.asarray(eng.host_views()["acc"])[:, _abi.ACC_DECISIONS].sum()) - d0
        L.hs_field_stats(fs.ctypes.data)
        res = {"decisions": dec, "reads_per_decision": {SECTIONS[i]: round(float(fs[i]) / dec, 2)
                                                        for i in SECTIONS if fs[i]}}
        res["total_per_decision"] = round(float(fs.sum()) / dec, 1)
        out[name] = res
        print(name, json.dumps(res, indent=1), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
