"""Batched Decima GNN policy (spark_sched_sim/schedulers/decima.py) vs the per-observation CPU fp32
restatement (oracle/decima_gnn.py), on the test-only host build of the engine (CPU suite) and on the
device engine (`-m gpu`, the policy on the GPU)."""

import pytest

import cases


@pytest.fixture(scope="module")
def make_host():
    from hostsim.driver import HostEngine

    def _make(cfg, B, ds, trace_cap):
        return HostEngine(cfg, B, ds, trace_cap=trace_cap)

    return _make


@pytest.mark.parametrize("cfg_over,B,seed0,every", cases.POLICY_CONFIGS)
def test_decima_policy_host(make_host, dataset, env_cfg, cfg_over, B, seed0, every):
    cases.case_decima_policy(make_host, dataset, env_cfg, cfg_over, min(B, 2), seed0, every * 2, max_steps=250)


def test_decima_schedule_host(make_host, dataset, env_cfg):
    cases.case_decima_schedule_runs(make_host, dataset, env_cfg, B=6, steps=20)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_over,B,seed0,every", cases.POLICY_CONFIGS)
def test_decima_policy_gpu(gpu_device, dataset, env_cfg, cfg_over, B, seed0, every):
    from spark_sched_sim.engine import DeviceEngine

    def make(cfg, B, ds, trace_cap):
        return DeviceEngine(cfg, B, ds, device=gpu_device, trace_cap=trace_cap)

    cases.case_decima_policy(make, dataset, env_cfg, cfg_over, B, seed0, every, device=gpu_device)


@pytest.mark.gpu
def test_decima_schedule_gpu(gpu_device, dataset, env_cfg):
    from spark_sched_sim.engine import DeviceEngine

    def make(cfg, B, ds, trace_cap):
        return DeviceEngine(cfg, B, ds, device=gpu_device, trace_cap=trace_cap)

    cases.case_decima_schedule_runs(make, dataset, env_cfg, B=64, steps=50, device=gpu_device)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_over,B,seed0,every", cases.POLICY_CONFIGS)
def test_decima_fused_kernel_gpu(gpu_device, dataset, env_cfg, cfg_over, B, seed0, every):
    from spark_sched_sim.engine import DeviceEngine

    def make(cfg, B, ds, trace_cap):
        return DeviceEngine(cfg, B, ds, device=gpu_device, trace_cap=trace_cap)

    cases.case_decima_fused(make, dataset, env_cfg, cfg_over, 32, seed0, device=gpu_device)
