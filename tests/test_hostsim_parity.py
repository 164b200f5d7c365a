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


WINDOW_CASES = [  # (config overrides, envs, steps, mean time limit, ring variant)
    (dict(num_executors=100, job_arrival_cap=200), 3, 400, 2.0e5, 0),   # configs[3] shape, the device's rings
    (dict(num_executors=50, job_arrival_cap=200), 3, 400, 2.0e5, 0),    # configs[2] env, the device's rings
    (dict(num_executors=50, job_arrival_cap=200), 3, 300, 2.0e5, 1),    # tiny rings: overflow mid-step -> HBM path
    (dict(), 4, 1500, None, 1),                                         # J = 50: windows outgrow tiny rings often
]


@pytest.mark.parametrize("cfg_over,B,K,mean_limit,variant", WINDOW_CASES)
def test_windowed_rollout_matches_plain(dataset, env_cfg, cfg_over, B, K, mean_limit, variant):
    """The device's fused rollout on the WINDOWED engine (rollout.h rollout_loop; engine.h kWS / kWJ: rings of stages
    and jobs in a poisoned LDS emulation, auto-resets through the home layout, the HBM-resident engine for envs whose
    window outgrows the rings) leaves every env exactly as the plain rollout does: the action log, every
    observation field, the accumulators, wall times and job times. Variant 1's tiny rings (32 stages / 4 jobs) make
    windows overflow at load, at arrivals mid-step and at reloads after resets, so the fallback paths run too."""
    import numpy as np

    from hostsim.driver import HostEngine
    from spark_sched_sim.distributed import shard_seeds

    cfg = dict(env_cfg, **cfg_over)
    limits = cases.bench_time_limits(mean_limit, shard_seeds(0, B, 0)) if mean_limit else None
    engs = [HostEngine(cfg, B, dataset) for _ in range(2)]
    logs = []
    for e in engs:
        e.reset_sampled(_abi.SSIM_RESET_SEED, seeds=shard_seeds(0, B, 0), time_limits=limits)
        logs.append(e.alloc_action_log(K))
    flags = _abi.SSIM_ROLLOUT_AUTORESET
    engs[0].rollout(_abi.SSIM_POLICY_RANDOM, 77, K, logs[0], flags=flags, time_limits=limits)
    fell = engs[1].rollout_windowed(_abi.SSIM_POLICY_RANDOM, 77, K, variant=variant, action_log=logs[1], flags=flags,
                                    time_limits=limits)
    assert np.array_equal(logs[0], logs[1])
    a, b = engs[0].host_views(), engs[1].host_views()
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    ta0, tc0, st0 = engs[0].job_times_np()
    ta1, tc1, st1 = engs[1].job_times_np()
    assert np.array_equal(ta0, ta1) and np.array_equal(tc0, tc1) and np.array_equal(st0, st1)
    assert int(np.count_nonzero(a["counts"][:, _abi.OC_ERR])) == 0
    assert int(a["acc"][:, _abi.ACC_EPISODES].sum()) > 0  # auto-resets ran inside the call
    if variant == 1:
        assert fell.any()  # the fallback path ran
    else:
        assert not fell.any()
