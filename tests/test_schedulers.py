"""Host scheduler plugins (spark_sched_sim.schedulers: RoundRobinScheduler / RandomScheduler / make_scheduler)
and the examples.py episode runner, checked against the oracle's restatement of
schedulers/heuristics/*.py on the oracle's own observations, then end to end through the facade."""

import numpy as np
import pytest

from oracle import restatement as R
from oracle.policies import FairPolicy, RandomPolicy
from spark_sched_sim.examples import ENV_CFG, run_episode
from spark_sched_sim.schedulers import RandomScheduler, RoundRobinScheduler, make_scheduler


def host_factory(job_cap=None):
    from hostsim.driver import HostEngine

    return lambda cfg, ds: HostEngine(cfg, 1, ds, job_cap=job_cap)


def _copy(obs):
    return {k: v for k, v in obs.items()}


@pytest.mark.parametrize("make", [
    lambda: (RoundRobinScheduler(10, dynamic_partition=True), FairPolicy(10, True)),
    lambda: (RoundRobinScheduler(10, dynamic_partition=False), FairPolicy(10, False)),
    lambda: (RandomScheduler(11), RandomPolicy(11)),
])
def test_scheduler_actions_match_oracle(dataset, env_cfg, make):
    """Same action for every observation of an episode (the oracle policy drives the episode)."""
    sched, ref_pol = make()
    ref = R.SparkSchedOracle(env_cfg, dataset)
    obs, _ = ref.reset(seed=2024)
    done, steps = False, 0
    while not done:
        a, info = sched.schedule(_copy(obs))
        b, _ = ref_pol.schedule(_copy(obs))
        assert info == {}
        assert (int(a["stage_idx"]), int(a["num_exec"])) == (int(b["stage_idx"]), int(b["num_exec"])), steps
        obs, _, done, _, _ = ref.step(b)
        steps += 1
    assert steps > 100


def test_make_scheduler():
    s = make_scheduler({"agent_cls": "RoundRobinScheduler", "num_executors": 50, "dynamic_partition": False})
    assert isinstance(s, RoundRobinScheduler) and s.name == "FIFO" and s.num_executors == 50
    assert isinstance(make_scheduler({"agent_cls": "RandomScheduler", "seed": 3}), RandomScheduler)
    with pytest.raises(AssertionError):
        make_scheduler({"agent_cls": "NoSuchScheduler"})


def test_run_episode_fair_matches_oracle(dataset):
    """examples.py --sched fair: average job duration of the facade episode == the oracle's (host build)."""
    got = run_episode(ENV_CFG, RoundRobinScheduler(10), seed=1234, dataset=dataset,
                      _engine_factory=host_factory())
    ref = R.SparkSchedOracle(dict(ENV_CFG), dataset)
    obs, _ = ref.reset(seed=1234)
    pol, done = FairPolicy(10), False
    while not done:
        obs, _, done, _, _ = ref.step(pol.schedule(obs)[0])
    assert np.isclose(got, R.avg_job_duration(ref) * 1e-3, rtol=1e-12)


@pytest.mark.gpu
def test_run_episode_fair_device(dataset, gpu_device):
    """The same episode with every step on the gfx950 kernels."""
    got = run_episode(ENV_CFG, RoundRobinScheduler(10), seed=1234, dataset=dataset, device=gpu_device)
    ref = R.SparkSchedOracle(dict(ENV_CFG), dataset)
    obs, _ = ref.reset(seed=1234)
    pol, done = FairPolicy(10), False
    while not done:
        obs, _, done, _, _ = ref.step(pol.schedule(obs)[0])
    assert np.isclose(got, R.avg_job_duration(ref) * 1e-3, rtol=1e-12)
