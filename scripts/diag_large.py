#!/usr/bin/env python
"""Diagnostic: the configs[3] shard's fused rollout at several batch sizes / trace settings, each launch synchronised
and timed (a hang shows up as the launch that never reports). Usage: python scripts/diag_large.py [B,K,trace ...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-sparksched_amd")]


def main():
    import numpy as np
    import torch

    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine

    cfg = {"num_executors": 100, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}
    ds = generate(0)
    specs = sys.argv[1:] or ["64,40,0", "512,40,0", "4096,40,0", "4096,40,8000"]
    for spec in specs:
        B, K, tc = (int(x) for x in spec.split(","))
        eng = DeviceEngine(cfg, B, ds, device="cuda:0", trace_cap=tc)
        eng.reset(seeds=[5000 + i for i in range(B)])
        torch.cuda.synchronize()
        for k in range(K):
            t0 = time.perf_counter()
            eng.rollout(_abi.SSIM_POLICY_RANDOM, 99, 1)
            torch.cuda.synchronize()
            e = eng.views["counts"][:, _abi.OC_ERR].cpu().numpy()
            bad = e.nonzero()[0]
            if len(bad):  # EnvHeader::err_line (layout.h: 2 doubles, 6 u64/u32 pairs, 22 int32 before it)
                st = eng.state.cpu().numpy()
                eb = int(eng.layout.env_bytes)
                off = 136
                lines = [int(st[4096 + i * eb + off: 4096 + i * eb + off + 4].view(np.int32)[0]) for i in bad[:6]]
                print("  err lines", lines, flush=True)
            print(f"B={B} trace={tc} step {k}: {1e3 * (time.perf_counter() - t0):.2f} ms, envs with err {len(bad)}"
                  + (f" e.g. env {bad[:6].tolist()} err {[hex(int(x)) for x in e[bad[:6]]]}" if len(bad) else ""),
                  flush=True)
        eng.close()


if __name__ == "__main__":
    main()
