#!/usr/bin/env python
"""Diagnostic: the configs[3] shard's fused rollout one decision at a time, saving the state blocks of a few envs
after every step (npz), so two kernel builds (e.g. SSIM_GENERIC=1 vs the specialised kernels) can be diffed offline
to find the first step and byte where they part. Usage: python scripts/diag_diff.py OUT.npz B K env,env,..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-sparksched_amd")]


def main():
    import numpy as np
    import torch

    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine

    out, B, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    envs = [int(x) for x in sys.argv[4].split(",")]
    cfg = {"num_executors": 100, "job_arrival_cap": 200, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
           "warmup_delay": 1000.0}
    eng = DeviceEngine(cfg, B, generate(0), device="cuda:0")
    eng.reset(seeds=[5000 + i for i in range(B)])
    eb = int(eng.layout.env_bytes)
    blocks = []
    for k in range(K + 1):
        if k:
            eng.rollout(_abi.SSIM_POLICY_RANDOM, 99, 1)
        torch.cuda.synchronize()
        st = eng.state
        blocks.append(np.stack([st[4096 + i * eb: 4096 + (i + 1) * eb].cpu().numpy() for i in envs]))
        print(f"step {k} saved", flush=True)
    np.savez_compressed(out, blocks=np.stack(blocks), envs=np.array(envs), env_bytes=eb)
    eng.close()


if __name__ == "__main__":
    main()
