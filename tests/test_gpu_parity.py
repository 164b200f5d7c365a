"""Device parity (`-m gpu`): the gfx950 kernels through the C ABI vs the CPU oracle (cases.py)."""

import pytest

import cases
from spark_sched_sim import _abi

pytestmark = pytest.mark.gpu


@pytest.fixture
def make(gpu_device):
    from spark_sched_sim.engine import DeviceEngine

    def _make(cfg, B, ds, trace_cap):
        return DeviceEngine(cfg, B, ds, device=gpu_device, trace_cap=trace_cap)

    return _make


def test_native_library_is_the_hip_build(gpu_device):
    from spark_sched_sim import native

    L = native.lib()
    assert native.LIB_PATH.endswith("libsparksched.so") and hasattr(L, "ssim_step")


def test_lockstep_fair(make, dataset, env_cfg):
    cases.case_lockstep_fair(make, dataset, env_cfg)


def test_device_fair_policy(make, dataset, env_cfg):
    cases.case_device_fair_policy(make, dataset, env_cfg)


@pytest.mark.parametrize("cfg_over,B,seed0,pol", cases.LOCKSTEP_CONFIGS)
def test_lockstep_configs(make, dataset, env_cfg, cfg_over, B, seed0, pol):
    cases.case_lockstep_config(make, dataset, env_cfg, cfg_over, B, seed0, pol)


@pytest.mark.parametrize("kind", [_abi.SSIM_POLICY_RANDOM, _abi.SSIM_POLICY_FAIR])
def test_rollout_replay(make, dataset, env_cfg, kind):
    cases.case_rollout_replay(make, dataset, env_cfg, kind)


@pytest.mark.parametrize("kind", [_abi.SSIM_POLICY_RANDOM, _abi.SSIM_POLICY_FAIR])
def test_rollout_budget_replay(make, dataset, env_cfg, kind):
    cases.case_rollout_replay(make, dataset, env_cfg, kind, B=64, K=400, stride=4, budget=150)


def test_rollout_replay_full_episodes(make, dataset, env_cfg):
    cases.case_rollout_replay(make, dataset, env_cfg, _abi.SSIM_POLICY_RANDOM, B=256, K=2500, stride=32)


def test_invalid_actions(make, dataset, env_cfg):
    cases.case_invalid_actions(make, dataset, env_cfg)


def test_reset_continuation(make, dataset, env_cfg):
    cases.case_reset_continuation(make, dataset, env_cfg)


@pytest.mark.parametrize("cfg_over,B,seed0,pol,every", cases.DECIMA_CONFIGS)
def test_decima_features(make, dataset, env_cfg, cfg_over, B, seed0, pol, every):
    cases.case_decima_features(make, dataset, env_cfg, cfg_over, B, seed0, pol, every)


@pytest.mark.parametrize("cfg_over,B,seed0,mean_limit", cases.SAMPLED_RESET_CONFIGS)
def test_sampled_reset(make, dataset, env_cfg, cfg_over, B, seed0, mean_limit):
    cases.case_sampled_reset(make, dataset, env_cfg, cfg_over, B, seed0, mean_limit)


@pytest.mark.parametrize("mean_limit", [None, 2.0e5])
def test_autoreset_replay(make, dataset, env_cfg, mean_limit):
    cases.case_autoreset_replay(make, dataset, env_cfg, B=48, K=1500, mean_limit=mean_limit, stride=3)


def test_async_rollouts(make, dataset, env_cfg):
    cases.case_async_rollouts(make, dataset, env_cfg, device="cuda:0", B=16)


def test_render_history_device(gpu_device, dataset, env_cfg):
    from spark_sched_sim.env import SparkSchedSimEnv
    from test_env_facade import check_render_history

    from oracle.restatement import SparkSchedOracle

    env = SparkSchedSimEnv(env_cfg, dataset, device=gpu_device, history_cap=1 << 16)
    check_render_history(env, SparkSchedOracle(env_cfg, dataset))


def test_full_size_bench_shape_budget_replay(make, dataset, env_cfg):
    """BASELINE configs[1] at full size (1024 envs, 50 jobs / 10 executors, the bench's kernel instantiation
    and shared-budget launch of 300 decisions per env): every env error-free, the budget spent exactly, and
    every 64th env replayed on the oracle bit-exactly (trace, job times, final observation)."""
    cases.case_rollout_replay(make, dataset, env_cfg, _abi.SSIM_POLICY_RANDOM, B=1024, K=2400, stride=64,
                              budget=300)


def test_full_size_large_shard_replay(make, dataset, env_cfg):
    """BASELINE configs[3] per-GPU shard at full size (4096 envs, 200 jobs / 100 executors, the HBM-resident
    kernel compiled for 4 waves/SIMD): 40 fused decisions per env, every 512th env replayed on the oracle."""
    cfg = dict(env_cfg, num_executors=100, job_arrival_cap=200)
    cases.case_rollout_replay(make, dataset, cfg, _abi.SSIM_POLICY_RANDOM, B=4096, K=40, stride=512)
