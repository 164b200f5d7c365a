"""CPU parity of the engine logic via the TEST-ONLY host build (tests/hostsim): same cases as the device
suite (cases.py), sized for the CPU suite. The product path is the gfx950 library; see test_gpu_parity.py."""

import pytest

import cases
from spark_sched_sim import _abi


@pytest.fixture(scope="module", params=[False, True], ids=["hbm", "lds"])
def make(request):
    """`lds`: the device's LDS residency emulated (hostsim.cpp hs_set_resident): every step / rollout runs on a
    working copy of the hot block made by the engine's own live-range load_hot / save_hot, pre-filled with poison,
    so a record read outside the copied range or a write the save drops breaks parity here on the CPU."""
    from hostsim.driver import HostEngine

    def _make(cfg, B, ds, trace_cap):
        return HostEngine(cfg, B, ds, trace_cap=trace_cap, resident=request.param)

    return _make


def test_lockstep_fair(make, dataset, env_cfg):
    cases.case_lockstep_fair(make, dataset, env_cfg, B=3)


def test_device_fair_policy(make, dataset, env_cfg):
    cases.case_device_fair_policy(make, dataset, env_cfg, B=2)


@pytest.mark.parametrize("cfg_over,B,seed0,pol", cases.LOCKSTEP_CONFIGS)
def test_lockstep_configs(make, dataset, env_cfg, cfg_over, B, seed0, pol):
    cases.case_lockstep_config(make, dataset, env_cfg, cfg_over, min(B, 2), seed0, pol)


@pytest.mark.parametrize("kind", [_abi.SSIM_POLICY_RANDOM, _abi.SSIM_POLICY_FAIR])
def test_rollout_replay(make, dataset, env_cfg, kind):
    cases.case_rollout_replay(make, dataset, env_cfg, kind, B=8, K=300, stride=2)


def test_invalid_actions(make, dataset, env_cfg):
    cases.case_invalid_actions(make, dataset, env_cfg)


def test_reset_continuation(make, dataset, env_cfg):
    cases.case_reset_continuation(make, dataset, env_cfg)


@pytest.mark.parametrize("cfg_over,B,seed0,pol,every", cases.DECIMA_CONFIGS)
def test_decima_features(make, dataset, env_cfg, cfg_over, B, seed0, pol, every):
    cases.case_decima_features(make, dataset, env_cfg, cfg_over, min(B, 2), seed0, pol, every * 3)


@pytest.mark.parametrize("cfg_over,B,seed0,mean_limit", cases.SAMPLED_RESET_CONFIGS)
def test_sampled_reset(make, dataset, env_cfg, cfg_over, B, seed0, mean_limit):
    cases.case_sampled_reset(make, dataset, env_cfg, cfg_over, min(B, 4), seed0, mean_limit)


@pytest.mark.parametrize("mean_limit", [None, 2.0e5])
def test_autoreset_replay(make, dataset, env_cfg, mean_limit):
    cases.case_autoreset_replay(make, dataset, env_cfg, B=6, K=600, mean_limit=mean_limit)


def test_async_rollouts(make, dataset, env_cfg):
    cases.case_async_rollouts(make, dataset, env_cfg)
