"""The single-env drop-in facade (spark_sched_sim.env.SparkSchedSimEnv), StochasticTimeLimit and metrics vs the
CPU oracle. CPU suite: the facade is driven through its engine seam with the test-only host build; the device
variant of the same checks is in test_gpu_parity.py::test_env_facade_device."""

import numpy as np
import pytest

import parity
from oracle import restatement as R
from oracle.policies import FairPolicy, RandomPolicy
from spark_sched_sim import metrics
from spark_sched_sim.env import SparkSchedSimEnv
from spark_sched_sim.wrappers import StochasticTimeLimit


def host_factory(job_cap=None):
    from hostsim.driver import HostEngine

    return lambda cfg, ds: HostEngine(cfg, 1, ds, job_cap=job_cap)


def run_facade_vs_oracle(env, ref, policy_ref, seed, max_steps=100000, options=None):
    obs, info = env.reset(seed=seed, options=options)
    robs, rinfo = ref.reset(seed=seed, options=options)
    parity.compare_obs(robs, obs, "reset")
    assert info == rinfo or info["wall_time"] == rinfo["wall_time"]
    done = trunc = False
    steps = 0
    while not (done or trunc) and steps < max_steps:
        a, _ = policy_ref.schedule(robs)
        obs, r, done, trunc, info = env.step(a)
        robs, rr, rdone, rtrunc, rinfo = ref.step(a)
        parity.compare_obs(robs, obs, f"step {steps}")
        assert parity.close_rel(r, rr) and done == rdone and trunc == rtrunc
        assert info["wall_time"] == rinfo["wall_time"]
        steps += 1
    return steps


def test_facade_fair_episode_matches_oracle(dataset, env_cfg):
    env = SparkSchedSimEnv(env_cfg, dataset, _engine_factory=host_factory())
    ref = R.SparkSchedOracle(env_cfg, dataset)
    steps = run_facade_vs_oracle(env, ref, FairPolicy(10), seed=1234)
    assert steps > 100 and env.all_jobs_complete
    assert env.num_completed_jobs == len(ref.completed_ids) and env.num_active_jobs == 0
    assert env.job_arrival_cap == ref.job_arrival_cap
    assert np.isclose(env.avg_job_duration, ref.avg_job_duration, rtol=1e-12)
    assert np.isclose(metrics.avg_job_duration(env), R.avg_job_duration(ref), rtol=1e-12)
    assert np.isclose(metrics.avg_num_jobs(env), R.avg_num_jobs(ref), rtol=1e-12)
    # second episode: the duration buffer spans resets (deque(maxlen=200), spark_sched_sim.py:83)
    run_facade_vs_oracle(env, ref, FairPolicy(10), seed=99)
    assert np.isclose(env.avg_job_duration, ref.avg_job_duration, rtol=1e-12)


def test_facade_raises_like_reference(dataset, env_cfg):
    env = SparkSchedSimEnv(env_cfg, dataset, _engine_factory=host_factory())
    ref = R.SparkSchedOracle(env_cfg, dataset)
    obs, _ = env.reset(seed=5)
    ref.reset(seed=5)
    n = obs["dag_batch"].nodes.shape[0]
    bad = [{"stage_idx": n, "num_exec": 1}, {"stage_idx": 0, "num_exec": 0}, {"stage_idx": 0},
           {"stage_idx": 0.0, "num_exec": 1}, {"stage_idx": np.int64(-2), "num_exec": 1},
           {"stage_idx": 0, "num_exec": 11}]
    for a in bad:
        with pytest.raises(ValueError):
            env.step(a)
        with pytest.raises(ValueError):
            ref.step(a)
    ns = int(obs["dag_batch"].nodes[:, 2].sum())
    if ns < n:
        with pytest.raises(KeyError):
            env.step({"stage_idx": ns, "num_exec": 1})
        with pytest.raises(KeyError):
            ref.step({"stage_idx": ns, "num_exec": 1})
    # a valid numpy-int action after the failures behaves exactly like the oracle
    a, _ = FairPolicy(10).schedule(obs)
    a = {"stage_idx": np.int64(a["stage_idx"]), "num_exec": np.int32(a["num_exec"])}
    o1, r1, d1, _, _ = env.step(a)
    o2, r2, d2, _, _ = ref.step(a)
    parity.compare_obs(o2, o1, "after errors")


def test_reset_requires_a_limit(dataset, env_cfg):
    cfg = dict(env_cfg, job_arrival_cap=None)
    env = SparkSchedSimEnv(cfg, dataset, job_cap=400, _engine_factory=host_factory(job_cap=400))
    with pytest.raises(ValueError):
        env.reset(seed=1)
    with pytest.raises(ValueError):
        R.SparkSchedOracle(cfg, dataset).reset(seed=1)


def test_stochastic_time_limit_episode(dataset, env_cfg):
    """Time-limited episode without a job cap (decima_tpch.yaml-style), truncation semantics."""
    cfg = dict(env_cfg, job_arrival_cap=None)
    env = StochasticTimeLimit(SparkSchedSimEnv(cfg, dataset, job_cap=400,
                                               _engine_factory=host_factory(job_cap=400)), 1.5e6, seed=3)
    ref = StochasticTimeLimit(R.SparkSchedOracle(cfg, dataset), 1.5e6, seed=3)
    for seed in (17, None):
        obs, _ = env.reset(seed=seed)
        robs, _ = ref.reset(seed=seed)
        assert env.time_limit == ref.time_limit
        parity.compare_obs(robs, obs, "reset")
        pol = RandomPolicy(7)
        done = trunc = False
        k = 0
        while not (done or trunc):
            a, _ = pol.schedule(robs)
            obs, r, done, trunc, info = env.step(a)
            robs, rr, rdone, rtrunc, rinfo = ref.step(a)
            parity.compare_obs(robs, obs, f"step {k}")
            assert (done, trunc) == (rdone, rtrunc) and parity.close_rel(r, rr)
            k += 1
        assert trunc or done


def test_decima_env_wrapper_matches_reference_wrapper(dataset, env_cfg):
    """spark_sched_sim.decima.DecimaEnvWrapper (device featurisation; host build here) vs the Decima wrapper
    restatement on the oracle's observations, with Decima-format actions (num_exec offset by one)."""
    from oracle.decima import decima_observation
    from spark_sched_sim.decima import DecimaEnvWrapper

    env = DecimaEnvWrapper(SparkSchedSimEnv(env_cfg, dataset, _engine_factory=host_factory()))
    ref = R.SparkSchedOracle(env_cfg, dataset)
    N = env_cfg["num_executors"]
    obs, _ = env.reset(seed=4321)
    robs, _ = ref.reset(seed=4321)
    parity.compare_decima(decima_observation(robs, N), obs, "reset")
    pol = RandomPolicy(5)
    done, steps = False, 0
    while not done:
        a, _ = pol.schedule(robs)
        obs, r, done, _, _ = env.step({"stage_idx": a["stage_idx"], "num_exec": a["num_exec"] - 1})
        robs, rr, rdone, _, _ = ref.step(a)
        assert done == rdone and parity.close_rel(r, rr)
        parity.compare_decima(decima_observation(robs, N), obs, f"step {steps}")
        steps += 1
    assert steps > 100


def test_render_history_matches_oracle(dataset, env_cfg):
    """Render data export (spark_sched_sim.py:408-424): executor histories (executor.py:22-44) rebuilt from the
    engine's event trace equal the oracle's Executor.history lists, mid-episode and at the end; completion
    times follow the reference's completed-job set order."""
    from hostsim.driver import HostEngine

    cap = 1 << 16
    env = SparkSchedSimEnv(env_cfg, dataset, history_cap=cap,
                           _engine_factory=lambda cfg, ds: HostEngine(cfg, 1, ds, trace_cap=cap))
    check_render_history(env, R.SparkSchedOracle(env_cfg, dataset))


def check_render_history(env, ref):
    pol = RandomPolicy(seed=4)
    obs, _ = env.reset(seed=77)
    robs, _ = ref.reset(seed=77)
    done, steps, moves = False, 0, 0
    while not done:
        a, _ = pol.schedule(robs)
        obs, _, done, _, _ = env.step(a)
        robs, _, _, _, _ = ref.step(a)
        steps += 1
        if steps % 40 == 0 or done:
            got = env.executor_histories()
            want = [ex.history for ex in ref.executors]
            assert got == want, f"step {steps}"
    moves = sum(len(h) - 1 for h in got)
    assert moves > 20 and any(j == -1 for h in got for _, j in h[1:])  # attachments and releases to COMMON
    rd = env.render_data()
    assert rd["job_completion_times"] == [ref.jobs[j].t_completed for j in ref.completed_ids]
    assert rd["average_job_duration"] == int(R.avg_job_duration(ref) * 1e-3)
    assert rd["num_jobs_completed"] == len(ref.completed_ids) and rd["wall_time"] == ref.wall_time


def test_observation_space_matches_reference_structure(dataset, env_cfg):
    """spark_sched_sim.py:96-125 (+ the updates at :157 and :403-404): the env's observations are members of
    its observation_space; source_job_idx.n = jobs + 1 after reset, dag_ptr.feature_space.n = nodes + 1."""
    env = SparkSchedSimEnv(env_cfg, dataset, _engine_factory=host_factory())
    sp = env.observation_space
    assert set(sp.keys()) == {"dag_batch", "dag_ptr", "num_committable_execs", "source_job_idx", "exec_supplies"}
    assert sp["num_committable_execs"].n == 11 and sp["exec_supplies"].feature_space.n == 20
    assert sp["dag_batch"].node_space.shape == (3,)
    obs, _ = env.reset(seed=21)
    assert sp["source_job_idx"].n == env.job_arrival_cap + 1
    pol = FairPolicy(10)
    for k in range(60):
        assert sp.contains(obs), f"step {k}"
        assert sp["dag_ptr"].feature_space.n == obs["dag_batch"].nodes.shape[0] + 1
        assert env.action_space["stage_idx"].n == obs["dag_batch"].nodes.shape[0] + 1
        obs, *_ = env.step(pol.schedule(obs)[0])
    bad = dict(obs, num_committable_execs=11)
    assert not sp.contains(bad)


def test_avg_job_duration_window_spans_episodes(dataset, env_cfg):
    """The duration buffer is one deque(maxlen=200) over all episodes (spark_sched_sim.py:83,243-245,697): with
    50-job episodes the window is full after 4 episodes and then holds only the last 200 completions."""
    env = SparkSchedSimEnv(env_cfg, dataset, _engine_factory=host_factory())
    ref = R.SparkSchedOracle(env_cfg, dataset)
    for ep, seed in enumerate((3, 4, 5, 6, 7)):
        run_facade_vs_oracle(env, ref, FairPolicy(10), seed=seed)
        assert np.isclose(env.avg_job_duration, ref.avg_job_duration, rtol=1e-12), f"episode {ep}"
    assert len(ref.duration_buff) == 200
