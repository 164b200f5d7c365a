"""The exact timed paths of bench.py, replayed on the CPU oracle at the sizes and depths they are timed (`-m gpu`).

Each test runs bench.py's own launch sequence for one workload (device reset with the shard seeds and
StochasticTimeLimit draws, the seeded pre-roll, the warm-up and timed launches with the bench's flags) with action
logging on, then replays sampled envs on the oracle across their episode boundaries (cases.case_bench_rollout_sequence).
"""

import numpy as np
import pytest

import cases
from spark_sched_sim import _abi

pytestmark = pytest.mark.gpu

TPCH = {"num_executors": 10, "job_arrival_cap": 50, "job_arrival_rate": 4.0e-5, "moving_delay": 2000.0,
        "warmup_delay": 1000.0}  # bench.py ENV_CFG (examples.py:15-23)
DECIMA = dict(TPCH, num_executors=50, job_arrival_cap=200)  # bench.py DECIMA_ENV (config/decima_tpch.yaml:80-87)
LARGE = dict(TPCH, num_executors=100, job_arrival_cap=200)  # bench.py LARGE_ENV (configs[3] shard)


@pytest.fixture
def make(gpu_device):
    from spark_sched_sim.engine import DeviceEngine

    def _make(cfg, B, ds, trace_cap, config_flags=0):
        return DeviceEngine(cfg, B, ds, device=gpu_device, trace_cap=trace_cap, config_flags=config_flags)

    return _make


@pytest.mark.parametrize("K,warmup,stride", [(20, 5, 1), (300, 50, 4)])
def test_bench_tpch_timed_launch_replay(make, dataset, K, warmup, stride):
    """configs[1] as the driver times it (`bench.py --steps 20 --warmup 5`) and as bench.py's default (300 / 50):
    1024 envs on the LDS-resident bench kernel, pre-roll in [0, 1000) with auto-reset, the PREEMPT | AUTORESET
    budget launches, a closing launch. The driver's sequence replays EVERY env on the oracle (obs, wall time, job
    times, episodes, decisions; fanned out over the box's CPUs), the 300-step one every 4th."""
    r = cases.case_bench_rollout_sequence(make, dataset, TPCH, B=1024, preroll=1000, warmup=warmup, K=K, stride=stride,
                                          expect_resident=True)
    assert r["envs_replayed"] >= 1024 // stride
    assert r["pending_at_timed_end"] > 0  # the timed launch did preempt steps (completed by the closing launch)
    assert r["crossed_replayed"] >= 1  # replayed envs crossed episode boundaries (auto-resets inside the sequence)


def test_bench_tpch_large_batch_hbm_replay(make, dataset):
    """configs[1]'s env at 4096 envs per GPU (`bench.py --envs 4096`): a batch past 1.5x what the LDS-resident kernel
    holds at once runs on the HBM-resident (10 executors, 50 jobs)-specialised kernels (layout.h lds_concurrent_envs,
    k_hbm_n10.hip). bench.py's 300-step sequence; every 4th env replayed on the oracle."""
    r = cases.case_bench_rollout_sequence(make, dataset, TPCH, B=4096, preroll=1000, warmup=50, K=300, stride=4,
                                          expect_resident=False)
    assert r["envs_replayed"] >= 4096 // 4
    assert r["crossed_replayed"] >= 1


def test_bench_tpch_timed_launch_replay_traced(make, dataset):
    """The same sequence with event tracing on (trace records are written by a uniform branch the bench skips): the
    replayed envs' current-episode event traces (event order, executors, stage / job completions) bit for bit."""
    r = cases.case_bench_rollout_sequence(make, dataset, TPCH, B=1024, preroll=1000, warmup=5, K=20, stride=16,
                                          trace_cap=12000, expect_resident=True)
    assert r["pending_at_timed_end"] > 0


def test_bench_large_shard_deep_replay(make, dataset):
    """configs[3] shard as bench.py --workload large runs it: 4096 envs, J=200 / N=100, StochasticTimeLimit mean 2e7,
    the HBM-resident 4-wave kernel, pre-roll in [0, 3000) (hundreds of active stages), then the warm-up and timed
    budget launches; every 8th env replayed (512 envs, fanned out over the box's CPUs)."""
    r = cases.case_bench_rollout_sequence(make, dataset, LARGE, B=4096, preroll=3000, warmup=5, K=20, stride=8,
                                          mean_limit=2.0e7, expect_resident=False)
    assert r["envs_replayed"] >= 4096 // 8
    assert r["decisions_replayed"] > 256 * 1500


def test_bench_decima_env_deep_replay_hbm_rollout(make, dataset):
    """The configs[2] env shape on the HBM-resident rollout kernel 1500+ decisions deep (4096 envs, J=200 / N=50,
    time limits): the pre-roll of bench.py --workload decima, then budget launches; every 8th env replayed."""
    r = cases.case_bench_rollout_sequence(make, dataset, DECIMA, B=4096, preroll=3000, warmup=5, K=20, stride=8,
                                          mean_limit=2.0e7, expect_resident=False)
    assert r["envs_replayed"] >= 4096 // 8


def test_bench_decima_persistent_rollout_replay(make, dataset):
    """configs[2] as bench.py --workload decima now times it: 4096 envs (J=200 / N=50, time limits), the pre-roll,
    then the warm-up and timed persistent Decima rollouts (ssim_decima_rollout: features, fused GNN policy and step
    per env in one launch, a shared budget, PREEMPT | AUTORESET) and a closing launch; every 8th env's actions
    replayed on the oracle across its episode boundaries."""
    r = cases.case_bench_rollout_sequence(make, dataset, DECIMA, B=4096, preroll=1500, warmup=5, K=20, stride=8,
                                          mean_limit=2.0e7, expect_resident=False, policy="decima")
    assert r["envs_replayed"] >= 4096 // 8
    assert r["decisions_replayed"] > 512 * 700


def test_decima_persistent_rollout_small_batch_replay(make, dataset):
    """The LDS-resident instantiation of the persistent Decima rollout (batches of <= 256 J=200 envs, e.g. PPO's 16)
    through the same budget sequence; every 4th env replayed on the oracle."""
    cases.case_bench_rollout_sequence(make, dataset, DECIMA, B=16, preroll=300, warmup=5, K=40, stride=4,
                                      mean_limit=2.0e6, expect_resident=True, policy="decima")


@pytest.mark.parametrize("cfg,B,seed0", [(dict(DECIMA, beta=5e-3), 2, 11), (LARGE, 1, 21)])
def test_forced_hbm_full_episode_lockstep(make, dataset, cfg, B, seed0):
    """J=200 full-episode lockstep cases that batches of <= 256 envs would run LDS-resident, forced onto the
    HBM-resident kernels (SSIM_CFG_FORCE_HBM): every observation, the event trace and the job times vs the oracle."""
    import parity
    from oracle.policies import RandomPolicy
    from oracle.restatement import SparkSchedOracle

    eng = make(cfg, B, dataset, 100000, config_flags=_abi.SSIM_CFG_FORCE_HBM)
    assert int(eng.layout.lds_resident) == 0
    oracles = [SparkSchedOracle(cfg, dataset) for _ in range(B)]
    steps = parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)],
                                policy_factory=lambda i: RandomPolicy(42 + i), check_every=5)
    assert min(steps) > 500
    parity.compare_traces(eng, oracles)
    ta, tc, _ = eng.job_times_np()
    parity.compare_job_times(ta, tc, oracles)


def test_forced_hbm_bench_sequence(make, dataset):
    """bench.py's tpch sequence (small batch) on the HBM-resident kernels: the same replay checks."""

    def make_hbm(cfg, B, ds, trace_cap):
        return make(cfg, B, ds, trace_cap, config_flags=_abi.SSIM_CFG_FORCE_HBM)

    cases.case_bench_rollout_sequence(make_hbm, dataset, TPCH, B=128, preroll=1000, warmup=5, K=20, stride=8,
                                      trace_cap=12000, expect_resident=False)


def test_bench_decima_timed_steps_replay(gpu_device, dataset):
    """configs[2] as bench.py --workload decima times it: 4096 envs (J=200, N=50, StochasticTimeLimit mean 2e7),
    pre-roll in [0, 1500) with auto-reset, then per decision the fused Decima policy launch, the HBM-resident k_step
    launch and the device reset of finished episodes (ssim_reset_sampled). Every 16th env's actions (pre-roll and
    policy steps) replayed on the oracle across its episode boundaries."""
    import torch

    from spark_sched_sim.distributed import shard_seeds
    from spark_sched_sim.engine import DeviceEngine
    from spark_sched_sim.schedulers.decima import DecimaScheduler

    SENT = -99
    B, W, K, stride = 4096, 5, 20, 16
    dev = torch.device(gpu_device)
    eng = DeviceEngine(DECIMA, B, dataset, device=gpu_device)
    assert int(eng.layout.lds_resident) == 0
    seeds = shard_seeds(0, B, 0)
    lim = cases.bench_time_limits(2.0e7, seeds)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=lim)
    limits = torch.tensor(lim, dtype=torch.float64, device=dev)
    actions = [[] for _ in range(B)]
    pre = np.random.default_rng([0, 0, 7]).integers(0, 1500, B).astype(np.int32)
    log = eng.alloc_action_log(int(pre.max()) + 1)
    log.fill_(SENT)
    eng.rollout_steps(_abi.SSIM_POLICY_RANDOM, 4321, pre, int(pre.max()) + 1, log,
                      flags=_abi.SSIM_ROLLOUT_AUTORESET | _abi.SSIM_ROLLOUT_WARMUP, time_limits=limits)
    lg = log.cpu().numpy()
    for i in range(B):
        actions[i].extend(lg[lg[:, i, 0] != SENT, i].tolist())
    torch.manual_seed(0)
    pol = DecimaScheduler(DECIMA["num_executors"]).to(dev)
    packed = pol.packed_params(dev)
    cnt = eng.views["counts"]
    steps = torch.zeros((W + K, B, 2), dtype=torch.int32, device=dev)
    for k in range(W + K):
        act = pol.schedule_fused(eng, eng.decima_features(), seed=0, counter=k + 1, params=packed)
        assert int(act["overflow"].sum().item()) == 0
        steps[k, :, 0] = act["stage_idx"]
        steps[k, :, 1] = act["num_exec"]
        eng.step(act["stage_idx"], act["num_exec"])
        assert int(torch.count_nonzero(cnt[:, _abi.OC_ERR]).item()) == 0, f"step {k}"
        done = ((cnt[:, _abi.OC_TERMINATED] != 0) | (cnt[:, _abi.OC_TRUNCATED] != 0)).to(torch.uint8)
        eng.reset_sampled(done, time_limits=limits)
    st = steps.cpu().numpy()
    for i in range(B):
        actions[i].extend(st[:, i].tolist())
    v = eng.host_views()
    ta, tc, _ = eng.job_times_np()
    sample = list(range(0, B, stride))
    res = cases.replay_many(DECIMA, dataset, [(seeds[i], lim[i], actions[i]) for i in sample])
    for i, (o, ob, ep, dec, last) in zip(sample, res):
        cases.check_replayed_env(eng, v, ta, tc, i, o, ob, ep, dec, last, "decima-bench")


@pytest.mark.parametrize("n_exec,jobs,B,seed0", [(3, 20, 3, 31), (16, 30, 2, 41), (127, 20, 1, 51)])
def test_forced_hbm_generic_kernel_lockstep(make, dataset, n_exec, jobs, B, seed0):
    """Shapes without a specialised unit on the generic HBM-resident kernels (`hbm`: run-time executor count, the
    executor records' LDS copy sized at run time, the opaque lane index): full-episode lockstep with random actions, every
    5th observation, the event trace and the job times vs the oracle. N = 16 and 127 take the paged set tables."""
    import parity
    from oracle.policies import RandomPolicy
    from oracle.restatement import SparkSchedOracle
    from spark_sched_sim import native

    cfg = dict(TPCH, num_executors=n_exec, job_arrival_cap=jobs)
    eng = make(cfg, B, dataset, 100000, config_flags=_abi.SSIM_CFG_FORCE_HBM)
    assert int(eng.layout.lds_resident) == 0
    assert native.lib().ssim_debug_kernel_name(eng.handle, 0).decode() == "hbm"
    oracles = [SparkSchedOracle(cfg, dataset) for _ in range(B)]
    steps = parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)],
                                policy_factory=lambda i: RandomPolicy(42 + i), check_every=5)
    assert min(steps) > 20
    parity.compare_traces(eng, oracles)
    ta, tc, _ = eng.job_times_np()
    parity.compare_job_times(ta, tc, oracles)
