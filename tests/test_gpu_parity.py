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


@pytest.mark.parametrize("autoreset", [True, False])
def test_rollout_preempt_replay(make, dataset, env_cfg, autoreset):
    cases.case_rollout_preempt(make, dataset, env_cfg, autoreset=autoreset)


def test_rollout_replay_full_episodes(make, dataset, env_cfg):
    cases.case_rollout_replay(make, dataset, env_cfg, _abi.SSIM_POLICY_RANDOM, B=256, K=2500, stride=4)


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


@pytest.mark.parametrize("mean_limit", [None, 2.0e5])
def test_autoreset_budget_replay(make, dataset, env_cfg, mean_limit):
    cases.case_autoreset_replay(make, dataset, env_cfg, B=48, K=1500, mean_limit=mean_limit, stride=3, budget=600)


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
    every 8th env replayed on the oracle bit-exactly (trace, job times, final observation)."""
    cases.case_rollout_replay(make, dataset, env_cfg, _abi.SSIM_POLICY_RANDOM, B=1024, K=2400, stride=8,
                              budget=300)


def test_full_size_large_shard_replay(make, dataset, env_cfg):
    """BASELINE configs[3] per-GPU shard at full size (4096 envs, 200 jobs / 100 executors, the HBM-resident
    kernel compiled for 4 waves/SIMD): 40 fused decisions per env, every 16th env replayed on the oracle."""
    cfg = dict(env_cfg, num_executors=100, job_arrival_cap=200)
    cases.case_rollout_replay(make, dataset, cfg, _abi.SSIM_POLICY_RANDOM, B=4096, K=40, stride=16)


@pytest.mark.parametrize("name", __import__("test_golden").NAMES)
def test_golden_fixtures_device(gpu_device, dataset, name):
    """The committed golden fixtures (tests/golden/*.json) replayed through the device engine step by step:
    obs digests, wall times, rewards, the full event trace and job times."""
    from spark_sched_sim.engine import DeviceEngine
    from test_golden import load, replay_on_engine

    fx = load(name)
    eng = DeviceEngine(fx["cfg"], 1, dataset, device=gpu_device, trace_cap=fx["trace_len"] + 16)
    replay_on_engine(eng, fx)


def test_env_facade_device(gpu_device, dataset, env_cfg):
    """The single-env facade on the device (test_env_facade.py runs the same checks on the host build):
    a fair episode and a second one, observation space membership and the 200-job duration window."""
    from oracle import restatement as R
    from oracle.policies import FairPolicy
    from spark_sched_sim.env import SparkSchedSimEnv
    from test_env_facade import run_facade_vs_oracle

    env = SparkSchedSimEnv(env_cfg, dataset, device=gpu_device)
    ref = R.SparkSchedOracle(env_cfg, dataset)
    for seed in (1234, 99, 5, 6, 7):
        assert run_facade_vs_oracle(env, ref, FairPolicy(10), seed=seed) > 100
        assert env.avg_job_duration == pytest.approx(ref.avg_job_duration, rel=1e-12)
    obs, _ = env.reset(seed=3)
    assert env.observation_space.contains(obs)


@pytest.mark.parametrize("B", [1024])
def test_vec_env_device_reset(gpu_device, dataset, env_cfg, B):
    """SparkSchedSimVecEnv.reset through ONE ssim_reset_sampled launch (B >= 1024) gives exactly the host-sampled
    reset (numpy Generator), for reset(seed) with StochasticTimeLimit limits and for reset(seed=None)."""
    import numpy as np

    from spark_sched_sim.vec_env import SparkSchedSimVecEnv

    cfg = dict(env_cfg, job_arrival_cap=None)
    kw = dict(device=gpu_device, job_cap=400, mean_time_limit=5.0e5)  # > 400 jobs needs a 20-mean limit
    dev = SparkSchedSimVecEnv(cfg, B, dataset, device_reset=True, **kw)
    host = SparkSchedSimVecEnv(cfg, B, dataset, device_reset=False, **kw)
    assert SparkSchedSimVecEnv(env_cfg, B, dataset, device=gpu_device).device_reset  # the default at this size
    dev.reset(seed=100)
    host.reset(seed=100)
    assert np.array_equal(dev.engine.snapshot_obs(), host.engine.snapshot_obs())
    for _ in range(20):
        si, ne = host.policy(_abi.SSIM_POLICY_FAIR)
        host.step(si, ne)
        dev.step(si, ne)
    dev.reset()
    host.reset()
    assert np.array_equal(dev.engine.snapshot_obs(), host.engine.snapshot_obs())
    c = dev.engine.host_views()["counts"]
    assert int(np.count_nonzero(c[:, _abi.OC_ERR])) == 0 and (c[:, _abi.OC_EPISODE] == 2).all()


def test_full_size_decima_config2(gpu_device, dataset):
    """BASELINE configs[2] at full size: 4096 envs, decima_tpch.yaml env section (N=50, J cap 200, StochasticTimeLimit
    mean 2e7 ms), the fused Decima policy (LDS plan forced above 64 KB, the opt-in path) + ssim_step for K
    decisions: no env errors, no policy overflow, and every 512th env's logged actions replayed on the oracle
    reproduce its final observation, wall time and decision count bit-exactly."""
    import numpy as np
    import torch

    import parity
    from oracle.restatement import SparkSchedOracle
    from spark_sched_sim.engine import DeviceEngine, obs_dict
    from spark_sched_sim.schedulers.decima import DecimaScheduler
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    cfg = dict(num_executors=50, job_arrival_cap=200, job_arrival_rate=4.0e-5, moving_delay=2000.0,
               warmup_delay=1000.0)
    B, K = 4096, 48
    dev = torch.device(gpu_device)
    eng = DeviceEngine(cfg, B, dataset, device=gpu_device)
    seeds = [6000 + i for i in range(B)]
    smp = StochasticTimeLimitSampler(2.0e7, B, seed=42)
    limits = np.array([smp.sample(i, seeds[i]) for i in range(B)])
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=limits)
    torch.manual_seed(0)
    pol = DecimaScheduler(50).to(dev)
    packed = pol.packed_params(dev)
    log = torch.zeros((K, B, 2), dtype=torch.int32, device=dev)
    big_plan = 0
    for k in range(K):
        feats = eng.decima_features()
        nodes = int(eng.views["counts"][:, _abi.OC_NUM_NODES].max().item())
        cap = max(nodes, 400)  # 400 nodes x ~199 B + the per-DAG rows > 64 KB
        fo = pol.schedule_fused(eng, feats, seed=11, counter=k, node_cap=cap, params=packed)
        assert int(fo["overflow"].item()) == 0, f"step {k}"
        big_plan += 1
        log[k, :, 0] = fo["stage_idx"]
        log[k, :, 1] = fo["num_exec"]
        eng.step(fo["stage_idx"], fo["num_exec"])
    assert big_plan == K
    v = eng.host_views()
    c = v["counts"]
    assert int(np.count_nonzero(c[:, _abi.OC_ERR])) == 0
    assert int(c[:, _abi.OC_NUM_NODES].max()) > 20
    lg = log.cpu().numpy()
    for i in range(0, B, 512):
        o = SparkSchedOracle(cfg, dataset)
        ob, _ = o.reset(seed=seeds[i], options={"time_limit": float(limits[i])})
        n = int(c[i, _abi.OC_DECISIONS])
        for k in range(n):
            ob, _, term, _, _ = o.step({"stage_idx": int(lg[k, i, 0]), "num_exec": int(lg[k, i, 1])})
        assert n == K or term, f"env{i}: {n} decisions"
        assert float(v["wall_time"][i]) == float(o.wall_time)
        parity.compare_obs(ob, obs_dict(v, i), f"env{i} final")


def test_rollout_replay_other_stage_cap(make, env_cfg):
    """A TPC-H-format dataset whose largest query has 17 stages (stage cap 850, not the default set's 900) runs the
    (executors, jobs)-specialised kernels with the stage cap read at run time; replayed on the oracle."""
    from spark_sched_sim.data_samplers.synthetic_tpch import generate

    ds = generate(1)
    assert max(a.shape[0] for a, _ in ds.values()) == 17
    cases.case_rollout_replay(make, ds, env_cfg, _abi.SSIM_POLICY_RANDOM, B=64, K=400, stride=8)
