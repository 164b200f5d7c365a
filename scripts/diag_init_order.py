#!/usr/bin/env python
"""Diagnostic: which initialisation orders of torch's HIP runtime and libsparksched's let ssim_create succeed.
Each variant runs in its own process (python scripts/diag_init_order.py <variant>); no argument runs them all."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(variant):
    sys.path[:0] = [REPO, os.path.join(REPO, "gym-sparksched_amd")]
    import torch

    if variant in ("torch_first", "torch_first_ctx"):
        torch.zeros(1, device="cuda:0")
    from spark_sched_sim import native

    if variant == "lib_first":
        native.build_id()
        native.lib()
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.engine import DeviceEngine

    cfg = dict(num_executors=10, job_arrival_cap=8, job_arrival_rate=4e-5, moving_delay=2000.0, warmup_delay=1000.0)
    eng = DeviceEngine(cfg, 2, generate(0), device="cuda:0")
    print(variant, "OK", int(eng.layout.chip_cus))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for v in ("plain", "lib_first", "torch_first"):
            r = subprocess.run([sys.executable, __file__, v], capture_output=True, text=True, timeout=300)
            print(v, "rc", r.returncode, (r.stdout + r.stderr).strip().splitlines()[-1:])
