"""Parity cases shared by the device tests (test_gpu_parity.py, `-m gpu`, gfx950 kernels through the C ABI)
and the CPU tests of the test-only host build (test_hostsim_parity.py). Each case takes an engine factory
`make(cfg, B, dataset, trace_cap)` returning a DeviceEngine or HostEngine.

Bit-exact: every observation (float32 node features, int64 edge links, dag_ptr, supplies, committable,
source index), wall times (float64), terminated flags, decision counts, the full event trace (event order,
executor assignments, stage/job completions) and job completion times. Rewards within 1e-9 relative.
"""

import numpy as np
import pytest

import parity
from oracle.decima import decima_observation
from oracle.policies import FairPolicy, RandomPolicy
from oracle.restatement import SparkSchedOracle
from spark_sched_sim import _abi
from spark_sched_sim.engine import decima_obs_dict, decode_trace, obs_dict

LOCKSTEP_CONFIGS = [
    (dict(beta=5e-3), 4, 7, "random"),
    (dict(num_executors=50, job_arrival_cap=200, beta=5e-3), 2, 11, "random"),
    (dict(num_executors=100, job_arrival_cap=200), 1, 21, "fair"),
    (dict(num_executors=3, job_arrival_cap=20, job_arrival_rate=1e-4, moving_delay=500.0, warmup_delay=100.0),
     8, 31, "random"),
]


def case_lockstep_fair(make, dataset, env_cfg, B=8, seed0=1234):
    eng = make(env_cfg, B, dataset, 20000)
    oracles = [SparkSchedOracle(env_cfg, dataset) for _ in range(B)]
    steps = parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)])
    assert min(steps) > 100
    parity.compare_traces(eng, oracles)
    ta, tc, _ = eng.job_times_np()
    parity.compare_job_times(ta, tc, oracles)


def case_device_fair_policy(make, dataset, env_cfg, B=6):
    """The on-device RoundRobinScheduler picks exactly the actions of round_robin.py:14-49."""
    eng = make(env_cfg, B, dataset, 0)
    oracles = [SparkSchedOracle(env_cfg, dataset) for _ in range(B)]
    pols = [FairPolicy(env_cfg["num_executors"]) for _ in range(B)]
    obs = [o.reset(seed=77 + i)[0] for i, o in enumerate(oracles)]
    eng.reset(seeds=[77 + i for i in range(B)])
    done = [False] * B
    for k in range(5000):
        if all(done):
            break
        si, ne = eng.policy(_abi.SSIM_POLICY_FAIR)
        si, ne = np.array(eng.to_numpy(si)), np.array(eng.to_numpy(ne))
        for i in range(B):
            if done[i]:
                continue
            a, _ = pols[i].schedule(obs[i])
            assert (int(a["stage_idx"]), int(a["num_exec"])) == (int(si[i]), int(ne[i])), f"env{i} step{k}"
        eng.step(si, ne)
        for i in range(B):
            if not done[i]:
                obs[i], _, done[i], _, _ = oracles[i].step({"stage_idx": int(si[i]), "num_exec": int(ne[i])})
    assert all(done)


def case_lockstep_config(make, dataset, env_cfg, cfg_over, B, seed0, pol):
    cfg = dict(env_cfg, **cfg_over)
    eng = make(cfg, B, dataset, 100000)
    oracles = [SparkSchedOracle(cfg, dataset) for _ in range(B)]
    fac = (lambda i: FairPolicy(cfg["num_executors"])) if pol == "fair" else (lambda i: RandomPolicy(42 + i))
    parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)], policy_factory=fac, check_every=7)
    parity.compare_traces(eng, oracles)
    ta, tc, _ = eng.job_times_np()
    parity.compare_job_times(ta, tc, oracles)


def case_rollout_replay(make, dataset, env_cfg, kind, B=64, K=400, stride=4, budget=0):
    """ssim_rollout (policy+step fused in one launch) logs its actions; replaying them on the oracle
    reproduces the trace, job times, decision counts and final observation bit-exactly. budget > 0: the
    work-conserving ssim_rollout_budget (B*budget decisions shared by the envs, at most K each)."""
    eng = make(env_cfg, B, dataset, 8000)
    seeds = [5000 + i for i in range(B)]
    eng.reset(seeds=seeds)
    log = eng.alloc_action_log(K)
    if budget:
        eng.rollout_budget(kind, 99, K, B * budget, log)
    else:
        eng.rollout(kind, 99, K, log)
    log = np.asarray(eng.to_numpy(log))
    v = eng.host_views()
    if budget:
        dec = v["counts"][:, _abi.OC_DECISIONS].astype(np.int64)
        live = (v["counts"][:, _abi.OC_TERMINATED] == 0) & (dec < K)
        assert dec.sum() <= B * budget and (dec.sum() == B * budget or not live.any())
        assert dec.max() > dec.min()  # the budget went unevenly (cheap envs took more)
    ta, tc, _ = eng.job_times_np()
    sample = list(range(0, B, stride))
    # many envs: the replays fanned out over the CPUs (cases.replay_many), otherwise in this process
    items = [(seeds[i], None, log[: int(v["counts"][i][_abi.OC_DECISIONS]), i].tolist()) for i in sample]
    done = replay_many(env_cfg, dataset, items, trace=True, autoreset=False) if len(sample) >= 16 else [
        replay_with_autoreset(env_cfg, dataset, s_, None, a_, trace=True, autoreset=False) for s_, _, a_ in items]
    for i, (o, ob, _, _, _) in zip(sample, done):
        c = v["counts"][i]
        assert int(c[_abi.OC_ERR]) == 0
        assert bool(c[_abi.OC_TERMINATED]) == o.terminated
        assert float(v["wall_time"][i]) == float(o.wall_time)
        parity.compare_obs(ob, obs_dict(v, i), f"env{i} final")
        got = decode_trace(np.asarray(v["trace"][i]), int(c[_abi.OC_TRACE_LEN]))
        ref = [tuple(float(x) if j == 0 else int(x) for j, x in enumerate(r)) for r in o.trace]
        assert len(ref) == int(c[_abi.OC_TRACE_LEN]) and got == ref[: len(got)]
        for jid, job in o.jobs.items():
            assert ta[i][jid] == job.t_arrival
            assert tc[i][jid] == job.t_completed or (np.isinf(tc[i][jid]) and np.isinf(job.t_completed))


def case_rollout_preempt(make, dataset, env_cfg, B=64, launches=8, per_launch=25, autoreset=True):
    """ssim_rollout_budget with SSIM_ROLLOUT_PREEMPT: once a launch's budget is claimed, steps still simulating
    stop at their next event boundary and stay pending (SSIM_ERR_PENDING); the next launch completes them first.
    Preemption must not change anything the env computes: each env's actions, logged launch by launch and
    concatenated, replayed on the oracle give its final observation, wall time, decision count and event trace
    bit for bit, after a closing launch (0 new steps) has completed the pending steps. Completed decisions
    (ob_acc) across the launches add up to the decisions applied."""
    SENT = -99
    eng = make(env_cfg, B, dataset, 8000)
    seeds = [6100 + i for i in range(B)]
    eng.reset(seeds=seeds)
    flags = _abi.SSIM_ROLLOUT_PREEMPT | (_abi.SSIM_ROLLOUT_AUTORESET if autoreset else 0)
    K = 8 * per_launch
    actions = [[] for _ in range(B)]
    pending_seen = 0
    for _ in range(launches):
        log = eng.alloc_action_log(K)
        log.fill_(SENT)
        eng.rollout_budget(_abi.SSIM_POLICY_RANDOM, 17, K, B * per_launch, log, flags=flags)
        lg = np.asarray(eng.to_numpy(log))
        for i in range(B):
            rows = lg[:, i, 0] != SENT
            actions[i] += [(int(a), int(b)) for a, b in lg[rows, i]]
        c = eng.host_views()["counts"]
        pending_seen += int(np.count_nonzero(c[:, _abi.OC_ERR] & _abi.SSIM_ERR_PENDING))
    assert pending_seen > B, pending_seen  # preemption actually happened, launch after launch
    eng.rollout(_abi.SSIM_POLICY_RANDOM, 17, 0, flags=_abi.SSIM_ROLLOUT_AUTORESET if autoreset else 0)
    v = eng.host_views()
    assert int(np.count_nonzero(v["counts"][:, _abi.OC_ERR])) == 0  # nothing pending, no errors
    applied = sum(len(a) for a in actions)
    assert int(v["acc"][:, _abi.ACC_DECISIONS].sum()) == applied
    episodes = 0
    for i in range(0, B, 4):
        o = SparkSchedOracle(env_cfg, dataset)
        o.trace = []
        ob, _ = o.reset(seed=seeds[i])
        ep = 1
        for a in actions[i]:
            ob, rew, term, _, info = o.step({"stage_idx": a[0], "num_exec": a[1]})
            if term and autoreset:
                o.trace = []
                ob, _ = o.reset(seed=None)
                ep += 1
        c = v["counts"][i]
        assert int(c[_abi.OC_EPISODE]) == ep
        assert float(v["wall_time"][i]) == float(o.wall_time), f"env{i}"
        parity.compare_obs(ob, obs_dict(v, i), f"env{i} final")
        got = decode_trace(np.asarray(v["trace"][i]), int(c[_abi.OC_TRACE_LEN]))
        ref = [tuple(float(x) if j == 0 else int(x) for j, x in enumerate(r)) for r in o.trace]
        assert got == ref[: len(got)] and len(ref) == int(c[_abi.OC_TRACE_LEN]), f"env{i} trace"
        episodes += ep


def case_invalid_actions(make, dataset, env_cfg, B=8):
    """ValueError/KeyError cases of _take_action (spark_sched_sim.py:276-295) -> per-env error bits, state
    untouched; a following valid action proceeds exactly like the oracle."""
    N = env_cfg["num_executors"]
    eng = make(env_cfg, B, dataset, 0)
    oracles = [SparkSchedOracle(env_cfg, dataset) for _ in range(B)]
    obs = [o.reset(seed=3 + i)[0] for i, o in enumerate(oracles)]
    eng.reset(seeds=[3 + i for i in range(B)])
    pols = [FairPolicy(N) for _ in range(B)]
    for _ in range(37):  # move into mid-episode states (some with 0 < committable < N)
        acts = [pols[i].schedule(obs[i])[0] for i in range(B)]
        eng.step([a["stage_idx"] for a in acts], [a["num_exec"] for a in acts])
        obs = [oracles[i].step(acts[i])[0] for i in range(B)]
    v = eng.host_views()
    bad, expect = [], []
    for i in range(B):
        c = v["counts"][i]
        nn, ns, cm = int(c[_abi.OC_NUM_NODES]), int(c[_abi.OC_NUM_SCHEDULABLE]), int(c[_abi.OC_COMMITTABLE])
        kind = i % 4
        if kind == 0:
            bad.append((nn, 1)), expect.append(_abi.SSIM_ERR_SPACE)
        elif kind == 1:
            bad.append((-1, 0)), expect.append(_abi.SSIM_ERR_SPACE)
        elif kind == 2 and ns < nn:
            bad.append((ns, 1)), expect.append(_abi.SSIM_ERR_KEY)
        elif kind == 3 and cm < N:
            bad.append((0, cm + 1)), expect.append(_abi.SSIM_ERR_TOO_MANY)
        else:
            bad.append((0, N + 1)), expect.append(_abi.SSIM_ERR_SPACE)
    before = eng.snapshot_obs()
    dec_before = [int(v["counts"][i][_abi.OC_DECISIONS]) for i in range(B)]
    eng.step([b[0] for b in bad], [b[1] for b in bad])
    v = eng.host_views()
    for i in range(B):
        assert int(v["counts"][i][_abi.OC_ERR]) == expect[i], f"env{i} {bad[i]}"
        assert int(v["counts"][i][_abi.OC_DECISIONS]) == dec_before[i]
    for i in range(B):  # the oracle raises on the same actions
        with pytest.raises((ValueError, KeyError)):
            oracles[i].step({"stage_idx": bad[i][0], "num_exec": bad[i][1]})
    after = eng.snapshot_obs()
    L = eng.layout
    lo, hi = L.ob_counts, L.ob_counts + L.num_envs * _abi.NUM_COUNTS * 4
    assert np.array_equal(before[:lo], after[:lo]) and np.array_equal(before[hi:], after[hi:])
    acts = [pols[i].schedule(obs[i])[0] for i in range(B)]
    eng.step([a["stage_idx"] for a in acts], [a["num_exec"] for a in acts])
    v = eng.host_views()
    for i in range(B):
        ob, rew, term, _, info = oracles[i].step(acts[i])
        parity.compare_obs(ob, obs_dict(v, i), f"env{i}")
        assert int(v["counts"][i][_abi.OC_ERR]) == 0


def case_reset_continuation(make, dataset, env_cfg, B=3):
    """reset(seed=None) continues each env's Generator where the device left it (gymnasium semantics)."""
    eng = make(env_cfg, B, dataset, 0)
    oracles = [SparkSchedOracle(env_cfg, dataset) for _ in range(B)]
    parity.run_lockstep(eng, oracles, seeds=[900 + i for i in range(B)], max_steps=150)
    obs = [o.reset(seed=None)[0] for o in oracles]
    eng.reset(seeds=None)
    v = eng.host_views()
    for i in range(B):
        parity.compare_obs(obs[i], obs_dict(v, i), f"env{i} reset(None)")
        assert int(v["counts"][i][_abi.OC_EPISODE]) == 2
    pols = [FairPolicy(env_cfg["num_executors"]) for _ in range(B)]
    for k in range(120):
        acts = [pols[i].schedule(obs[i])[0] for i in range(B)]
        eng.step([a["stage_idx"] for a in acts], [a["num_exec"] for a in acts])
        v = eng.host_views()
        for i in range(B):
            obs[i], r, t, _, info = oracles[i].step(acts[i])
            parity.compare_obs(obs[i], obs_dict(v, i), f"env{i} step{k}")
            assert float(v["wall_time"][i]) == float(info["wall_time"])


SAMPLED_RESET_CONFIGS = [
    (dict(), 16, 4100, None),
    (dict(num_executors=50, job_arrival_cap=200), 4, 4200, 3.0e6),
    (dict(num_executors=3, job_arrival_cap=20, job_arrival_rate=1e-4, moving_delay=500.0, warmup_delay=100.0),
     16, 4300, 8.0e5),
]


def _time_limits(mean, B, seed):
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    if mean is None:
        return None
    smp = StochasticTimeLimitSampler(mean, B, seed=seed)
    return np.array([smp.sample(i, seed + i) for i in range(B)])


def case_sampled_reset(make, dataset, env_cfg, cfg_over, B, seed0, mean_limit):
    """ssim_reset_sampled: job sequences drawn on the device (SeedSequence seeding, integers/choice, ziggurat
    exponential: tpch.py:54-73) give exactly the host-sampled reset (numpy), for reset(seed) and, after a
    stretch of stepping, for reset(seed=None) continuing each env's stream."""
    cfg = dict(env_cfg, **cfg_over)
    host, dev = make(cfg, B, dataset, 0), make(cfg, B, dataset, 0)
    seeds = [seed0 + 37 * i for i in range(B)]
    lim = _time_limits(mean_limit, B, seed0)
    opts = None if lim is None else [{"time_limit": float(x)} for x in lim]
    host.reset(seeds=seeds, options=opts)
    dev.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=lim)
    assert np.array_equal(host.snapshot_obs(), dev.snapshot_obs()), "reset(seed) obs"
    # every job's arrival time (t += exponential(1/rate), tpch.py:70: a rounded product, then the add)
    assert np.array_equal(host.job_times_np()[0], dev.job_times_np()[0]), "job arrival times"
    for k in range(60):  # same actions on both
        si, ne = host.policy(_abi.SSIM_POLICY_FAIR)
        si, ne = np.array(host.to_numpy(si)), np.array(host.to_numpy(ne))
        host.step(si, ne)
        dev.step(si, ne)
    lim2 = _time_limits(mean_limit, B, seed0 + 1)
    opts2 = None if lim2 is None else [{"time_limit": float(x)} for x in lim2]
    host.reset(seeds=None, options=opts2)
    dev.reset_sampled(_abi.SSIM_RESET_CONTINUE, time_limits=lim2)
    a, b = host.snapshot_obs(), dev.snapshot_obs()
    assert np.array_equal(a, b), "reset(seed=None) obs"
    assert np.array_equal(host.job_times_np()[0], dev.job_times_np()[0]), "job arrival times after reset(None)"
    v = dev.host_views()
    assert all(int(v["counts"][i][_abi.OC_EPISODE]) == 2 for i in range(B))
    assert all(int(v["counts"][i][_abi.OC_ERR]) == 0 for i in range(B))


def case_autoreset_replay(make, dataset, env_cfg, B=32, K=1500, mean_limit=None, stride=1, budget=0):
    """Fused rollout with SSIM_ROLLOUT_AUTORESET: finished episodes (terminated, or truncated by the time
    limit) restart in place with reset(seed=None). Replaying the logged actions on the oracle, resetting it the
    same way, reproduces every env's final observation, wall time and episode count. budget > 0: the same through
    the work-conserving ssim_rollout_budget (B*budget decisions shared, at most K per env, no preemption)."""
    SENT = -99
    cfg = dict(env_cfg, num_executors=4, job_arrival_cap=6, job_arrival_rate=1e-4)
    eng = make(cfg, B, dataset, 0)
    seeds = [7100 + i for i in range(B)]
    lim = _time_limits(mean_limit, B, 99) if mean_limit else None
    opts = None if lim is None else [{"time_limit": float(x)} for x in lim]
    eng.reset(seeds=seeds, options=opts)
    log = eng.alloc_action_log(K)
    if budget:
        log.fill_(SENT)
        eng.rollout_budget(_abi.SSIM_POLICY_RANDOM, 5, K, B * budget, log, flags=_abi.SSIM_ROLLOUT_AUTORESET,
                           time_limits=lim)
    else:
        eng.rollout(_abi.SSIM_POLICY_RANDOM, 5, K, log, flags=_abi.SSIM_ROLLOUT_AUTORESET, time_limits=lim)
    log = np.asarray(eng.to_numpy(log))
    v = eng.host_views()
    if budget:
        applied = (log[:, :, 0] != SENT).sum(axis=0)
        assert applied.sum() == B * budget and applied.max() > applied.min()
    episodes = 0
    for i in range(0, B, stride):
        limit = float("inf") if lim is None else float(lim[i])
        o = SparkSchedOracle(cfg, dataset)
        ob, _ = o.reset(seed=seeds[i], options={"time_limit": limit})
        ep = 1
        for k in range(int(applied[i]) if budget else K):
            ob, rew, term, _, info = o.step({"stage_idx": int(log[k, i, 0]), "num_exec": int(log[k, i, 1])})
            if term or info["wall_time"] >= limit:
                ob, _ = o.reset(seed=None, options={"time_limit": limit})
                ep += 1
        c = v["counts"][i]
        assert int(c[_abi.OC_ERR]) == 0, f"env{i}"
        assert int(c[_abi.OC_EPISODE]) == ep, f"env{i} episodes {int(c[_abi.OC_EPISODE])} != {ep}"
        assert float(v["wall_time"][i]) == float(o.wall_time)
        parity.compare_obs(ob, obs_dict(v, i), f"env{i} final")
        episodes += ep
    assert episodes > 3 * B // stride, episodes


DECIMA_CONFIGS = [
    (dict(), 4, 101, "random", 1),
    (dict(num_executors=50, job_arrival_cap=200, beta=5e-3), 2, 211, "random", 5),
    (dict(num_executors=3, job_arrival_cap=20, job_arrival_rate=1e-4, moving_delay=500.0, warmup_delay=100.0),
     6, 307, "fair", 1),
]


def case_decima_features(make, dataset, env_cfg, cfg_over, B, seed0, pol, every):
    """ssim_decima_features (node features, exec/stage masks, DAG-layer edge masks) equals the Decima
    wrapper restatement (oracle/decima.py: env_wrapper.py:69-143, utils.py:238-267) on the oracle's
    observation, at reset and every `every`-th decision of a full lockstep episode."""
    cfg = dict(env_cfg, **cfg_over)
    N = cfg["num_executors"]
    eng = make(cfg, B, dataset, 0)
    oracles = [SparkSchedOracle(cfg, dataset) for _ in range(B)]
    fac = (lambda i: FairPolicy(N)) if pol == "fair" else (lambda i: RandomPolicy(900 + i))
    seen = {"checks": 0, "masked": 0}

    def hook(k, obs, live):
        if k % every != 0:
            return
        dec = {key: eng.to_numpy(x) if not isinstance(x, np.ndarray) else x
               for key, x in eng.decima_features_np().items()}
        v = eng.host_views()
        for i in range(B):
            if not live[i]:
                continue
            ref = decima_observation(obs[i], N)
            got = decima_obs_dict(v, dec, i, N)
            parity.compare_decima(ref, got, f"env{i} step{k}")
            seen["checks"] += 1
            seen["masked"] += int(ref["edge_masks"].shape[0] > 0)

    parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)], policy_factory=fac, check_every=50,
                        hook=hook)
    assert seen["checks"] > 50 and seen["masked"] > 10, seen


POLICY_CONFIGS = [
    (dict(), 4, 610, 7),
    (dict(num_executors=50, job_arrival_cap=200, beta=5e-3), 2, 620, 11),
]


def case_decima_policy(make, dataset, env_cfg, cfg_over, B, seed0, every, device="cpu", max_steps=400):
    """The batched Decima GNN (spark_sched_sim/schedulers/decima.py) on the engine's device observation and
    features equals the per-observation CPU fp32 restatement (oracle/decima_gnn.py) on the oracle's
    reference-format observation: stage scores, exec scores of the first schedulable stage's job, and the
    evaluate_actions log-probabilities / entropies (collated-batch semantics), within 1e-5."""
    import torch

    from oracle import decima_gnn as G
    from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

    cfg = dict(env_cfg, **cfg_over)
    N = cfg["num_executors"]
    eng = make(cfg, B, dataset, 0)
    oracles = [SparkSchedOracle(cfg, dataset) for _ in range(B)]
    torch.manual_seed(seed0)
    pol = DecimaScheduler(N).to(device)
    for p in pol.parameters():  # non-zero biases too, so the bias paths are exercised
        p.data.add_(0.05 * torch.randn_like(p))
    sd = {k: v.detach().cpu().float() for k, v in pol.state_dict().items()}
    seen = {"checks": 0, "mp": 0}
    tol = dict(rtol=1e-5, atol=1e-5)

    def tt(x):
        return x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))

    def hook(k, obs, live):
        if k % every != 0:
            return
        feats = {key: tt(x).to(device) for key, x in eng.decima_features_np().items()}
        v = {key: tt(x).to(device) for key, x in eng.host_views().items() if key != "trace"}
        alive = torch.tensor(live, device=device)
        b = build_batch(v, feats, env_mask=alive)
        with torch.no_grad():
            h = pol.encoder(b, per_obs_no_mp=True)
            scores = pol.stage_policy_network(b, h).cpu()
        base = (torch.cumsum(b.num_stage_acts, 0) - b.num_stage_acts).cpu()
        stage_sel, job_sel, exec_sel, refs = [], [], [], []
        for i in range(B):
            if not live[i]:
                stage_sel.append(0), job_sel.append(0), exec_sel.append(0)
                continue
            ro = decima_observation(obs[i], N)
            enc = G.encode(sd, ro)
            rs = G.stage_scores(sd, ro, enc)
            ns = int(b.num_stage_acts[i])
            got = scores[int(base[i]): int(base[i]) + ns]
            assert torch.allclose(got, rs, **tol), f"env{i} step{k}: stage scores\n{got}\n{rs}"
            si = (k + i) % ns
            j = G.job_of_stage(ro, si)
            re = G.exec_scores(sd, ro, enc, j, N)
            with torch.no_grad():
                es, _, _ = pol.exec_policy_network(b, h, (b.obs_ptr[i] + j).view(1), torch.tensor([i], device=device))
            assert torch.allclose(es.cpu(), re, **tol), f"env{i} step{k}: exec scores"
            ei = (k * 7 + i) % re.numel()
            stage_sel.append(si), job_sel.append(j), exec_sel.append(ei)
            refs.append((i, ro, si, j, ei))
            seen["checks"] += 1
        if not refs:
            return
        # evaluate_actions over the live envs as one collated batch (scheduler.py:103-145)
        idx = torch.tensor([r[0] for r in refs], device=device)
        b2 = build_batch({key: x[idx] for key, x in v.items()}, {key: x[idx] for key, x in feats.items()})
        ev = pol.evaluate_actions(b2, torch.tensor([r[2] for r in refs], device=device),
                                  torch.tensor([r[3] for r in refs], device=device),
                                  torch.tensor([r[4] for r in refs], device=device))
        mp = b2.max_levels > 0
        seen["mp"] += int(mp)
        for n, (i, ro, si, j, ei) in enumerate(refs):
            enc = G.encode(sd, ro, collated_mp=mp)
            slp, sent = G.evaluate(G.stage_scores(sd, ro, enc), si)
            elp, eent = G.evaluate(G.exec_scores(sd, ro, enc, j, N), ei)
            nn_ = ro["nodes"].shape[0]
            ent = (sent + eent) / float(np.log(np.float32(N * nn_)))
            assert abs(float(ev["lgprobs"][n].detach()) - (slp + elp)) <= 1e-4 + 1e-5 * abs(slp + elp), f"env{i} lgprob"
            assert abs(float(ev["entropies"][n].detach()) - ent) <= 1e-4 + 1e-5 * abs(ent), f"env{i} entropy"

    fac = lambda i: RandomPolicy(300 + i)  # noqa: E731
    parity.run_lockstep(eng, oracles, seeds=[seed0 + i for i in range(B)], policy_factory=fac, check_every=50,
                        max_steps=max_steps, hook=hook)
    assert seen["checks"] > 20 and seen["mp"] > 0, seen


def case_decima_schedule_runs(make, dataset, env_cfg, B=16, steps=30, device="cpu"):
    """DecimaScheduler.schedule drives the engine: every sampled action is valid (no error bits) and
    log-probabilities are finite."""
    import torch

    from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

    N = env_cfg["num_executors"]
    eng = make(env_cfg, B, dataset, 0)
    eng.reset(seeds=list(range(B)))
    torch.manual_seed(0)
    pol = DecimaScheduler(N).to(device)
    g = torch.Generator(device=device).manual_seed(1)

    def tt(x):
        return x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))

    for _ in range(steps):
        feats = {key: tt(x).to(device) for key, x in eng.decima_features_np().items()}
        v = {key: tt(x).to(device) for key, x in eng.host_views().items() if key != "trace"}
        act = pol.schedule(build_batch(v, feats), generator=g)
        assert torch.isfinite(act["lgprob"]).all()
        eng.step(act["stage_idx"].cpu().numpy(), act["num_exec"].cpu().numpy())
        c = eng.host_views()["counts"]
        assert int(np.count_nonzero(np.asarray(c)[:, _abi.OC_ERR])) == 0


def case_decima_fused(make, dataset, env_cfg, cfg_over, B, seed0, iters=12, device="cuda:0"):
    """ssim_decima_policy (one fused kernel) vs the PyTorch DecimaScheduler on the same device observations:
    stage scores of every schedulable node, exec scores of the sampled DAG, and the log-probability of the
    sampled action, within fp32 rounding; the sampled actions are valid env actions."""
    import torch

    from spark_sched_sim.schedulers.decima import DecimaScheduler, build_batch

    cfg = dict(env_cfg, **cfg_over)
    N = cfg["num_executors"]
    eng = make(cfg, B, dataset, 0)
    eng.reset(seeds=[seed0 + i for i in range(B)])
    torch.manual_seed(seed0)
    pol = DecimaScheduler(N).to(device)
    for p in pol.parameters():
        p.data.add_(0.05 * torch.randn_like(p))
    checked = 0
    for it in range(iters):
        feats = eng.decima_features()
        b = build_batch(eng.views, feats)
        with torch.no_grad():
            h = pol.encoder(b, per_obs_no_mp=True)
            ref = pol.stage_policy_network.scores_all(b, h)
        fo = pol.schedule_fused(eng, feats, seed=7, counter=it, with_scores=True)
        assert int(fo["overflow"].item()) == 0
        si, ji, ei = fo["stage_idx"].cpu(), fo["job_idx"].cpu(), fo["exec_idx"].cpu()
        ss, lg = fo["stage_scores"].cpu(), fo["lgprob"].cpu()
        node_env, mask = b.node_env.cpu(), b.stage_mask.cpu()
        refc = ref.cpu()
        for e in range(B):
            rows = torch.nonzero((node_env == e) & mask).squeeze(1)
            if rows.numel() == 0:
                assert int(si[e]) == -1
                continue
            local = rows - int((node_env < e).sum())
            got = ss[e, local]
            assert torch.allclose(got, refc[rows], rtol=1e-4, atol=1e-5), f"env{e} it{it} stage scores"
            assert 0 <= int(si[e]) < rows.numel()
            dag = int(b.obs_ptr[e]) + int(ji[e])
            with torch.no_grad():
                es, valid = pol.exec_policy_network.scores_grid(b, h, torch.tensor([dag], device=device),
                                                                torch.tensor([e], device=device))
            cap = int(valid.sum())
            assert torch.allclose(fo["exec_scores"][e, :cap].cpu(), es[0, :cap].cpu(), rtol=1e-4, atol=1e-5)
            want = (torch.log_softmax(refc[rows], 0)[int(si[e])]
                    + torch.log_softmax(es[0, :cap].cpu(), 0)[int(ei[e])])
            assert abs(float(lg[e]) - float(want)) <= 1e-4 + 1e-4 * abs(float(want)), f"env{e} lgprob"
            checked += 1
        eng.step(fo["stage_idx"], fo["num_exec"])
        c = eng.host_views()["counts"]
        assert int(np.count_nonzero(np.asarray(c)[:, _abi.OC_ERR])) == 0
        eng.rollout(_abi.SSIM_POLICY_RANDOM, 3 + it, 4)
    assert checked > B * iters // 2


def case_async_rollouts(make, dataset, env_cfg, device="cpu", B=6, calls=3, duration=2.5e5, mean_limit=4e5):
    """AsyncRolloutCollector (trainers/rollout_worker.py:160-206, RolloutWorkerAsync): episodes span
    `collect` calls, each call runs every env for `duration` ms of simulated time, finished episodes are reset
    in place with seed = base + seed_step * reset_count and a fresh StochasticTimeLimit draw. The applied
    actions are replayed on the oracle through the reference's async loop (restated below); per env and call
    the decision count, the elapsed times (bit-exact), rewards (1e-9 rel), reset steps and the final
    observation must agree."""
    import torch

    from spark_sched_sim.schedulers.decima import DecimaScheduler
    from spark_sched_sim.trainers import AsyncRolloutCollector

    cfg = dict(env_cfg, num_executors=4, job_arrival_cap=6, job_arrival_rate=1e-4)
    eng = make(cfg, B, dataset, 0)
    torch.manual_seed(3)
    pol = DecimaScheduler(4).to(device)  # decima_tpch.yaml architecture: the fused kernel on the device
    base = [11 + i // 2 for i in range(B)]  # trainer.py:265-267: num_rollouts=2 rows per sequence
    col = AsyncRolloutCollector(eng, pol, duration, base, 3, mean_time_limit=mean_limit, fused=True, seed=5)
    gen = torch.Generator(device=device).manual_seed(1)
    bufs = [col.collect(generator=gen) for _ in range(calls)]
    v = eng.host_views()
    total_resets = 0
    for e in range(B):
        o = SparkSchedOracle(cfg, dataset)
        rng, reset_count = np.random.RandomState(42), 0
        limit = None

        def reset():
            nonlocal rng, reset_count, limit
            seed = base[e] + 3 * reset_count
            if seed:  # stochastic_time_limit.py:15-16
                rng = np.random.RandomState(seed)
            limit = float(rng.exponential(mean_limit))
            ob, _ = o.reset(seed=seed, options={"time_limit": limit})
            reset_count += 1
            return ob

        ob = reset()
        next_wall = 0.0
        for c, buf in enumerate(bufs):
            times, rewards, lengths, sample = buf.trajectories()
            flat_si = torch.cat(buf.stage_idx).cpu().numpy()
            flat_ne = torch.cat(buf.num_exec).cpu().numpy()
            n = int(lengths[e])
            elapsed, k, resets = 0.0, 0, []
            while elapsed < duration:
                wall = next_wall
                assert k < n, f"env{e} call{c}: device stopped after {n} decisions, oracle continues"
                i = int(sample[e, k])
                ob, rew, term, trunc, info = o.step({"stage_idx": int(flat_si[i]), "num_exec": int(flat_ne[i])})
                trunc = trunc or info["wall_time"] >= limit
                assert float(times[e, k]) == elapsed, f"env{e} call{c} step{k} elapsed"
                assert parity.close_rel(float(rewards[e, k]), rew), f"env{e} call{c} step{k} reward"
                next_wall = info["wall_time"]
                elapsed += next_wall - wall
                if term or trunc:
                    ob = reset()
                    next_wall = 0.0
                    resets.append(k)
                k += 1
            assert k == n, f"env{e} call{c}: {n} device decisions, oracle {k}"
            assert float(times[e, n]) == elapsed
            assert sorted(kk for ee, kk in buf.resets if ee == e) == resets
            total_resets += len(resets)
        parity.compare_obs(ob, obs_dict(v, e), f"env{e} final")
    assert total_resets >= B, total_resets


def _env_trace(eng, i: int, n: int):
    """Env i's trace records (the current episode), read without copying the whole obs arena to the host."""
    raw = eng.views["trace"][i]
    raw = raw.cpu().numpy() if hasattr(raw, "cpu") else np.asarray(raw)
    return decode_trace(raw, n)


def bench_time_limits(mean_limit, seeds):
    """bench.py's per-env StochasticTimeLimit draws (seed 42 sampler, one draw per env with its reset seed)."""
    from spark_sched_sim.wrappers import StochasticTimeLimitSampler

    if not mean_limit:
        return None
    smp = StochasticTimeLimitSampler(mean_limit, len(seeds), seed=42)
    return np.array([smp.sample(i, int(seeds[i])) for i in range(len(seeds))], dtype=np.float64)


def replay_with_autoreset(cfg, dataset, seed, limit, actions, trace=False, autoreset=True):
    """The oracle driven through `actions` from reset(seed), restarting like the device's auto-reset: after a step
    that terminates the episode or reaches its time limit, reset(seed=None) with the same limit (autoreset=False:
    never, the launches without SSIM_ROLLOUT_AUTORESET). Returns the oracle, its last observation, the episode count,
    the decisions of the current episode and the last step's reward (None if the last step ended an episode)."""
    limit = float("inf") if limit is None else float(limit)
    o = SparkSchedOracle(cfg, dataset)
    if trace:
        o.trace = []
    ob, _ = o.reset(seed=seed, options={"time_limit": limit})
    ep, dec, last = 1, 0, None
    for a in actions:
        ob, rew, term, _, info = o.step({"stage_idx": int(a[0]), "num_exec": int(a[1])})
        dec, last = dec + 1, rew
        if autoreset and (term or info["wall_time"] >= limit):
            if trace:
                o.trace = []
            ob, _ = o.reset(seed=None, options={"time_limit": limit})
            ep, dec, last = ep + 1, 0, None
    return o, ob, ep, dec, last


class _Replayed:
    """What check_replayed_env reads of a replayed oracle (wall time, job times, trace), picklable for the pool."""

    def __init__(self, o):
        from types import SimpleNamespace

        self.wall_time = o.wall_time
        self.jobs = {jid: SimpleNamespace(t_arrival=j.t_arrival, t_completed=j.t_completed) for jid, j in o.jobs.items()}
        self.trace = getattr(o, "trace", None)
        self.terminated = o.terminated


_POOL_DATASET = None


def _pool_init(dataset):
    global _POOL_DATASET
    _POOL_DATASET = dataset


def _replay_one(args):
    cfg, seed, limit, actions, trace, autoreset = args
    o, ob, ep, dec, last = replay_with_autoreset(cfg, _POOL_DATASET, seed, limit, actions, trace=trace,
                                                 autoreset=autoreset)
    return _Replayed(o), ob, ep, dec, last


def replay_many(cfg, dataset, items, trace=False, autoreset=True):
    """replay_with_autoreset for many envs, fanned out over the CPUs this job may use (spawn processes: the
    parent holds a GPU context). items: (seed, limit, actions) per env. Returns (oracle view, obs, episodes,
    decisions, last reward) per env, in order."""
    import multiprocessing as mp

    import bench

    jobs = [(cfg, s, lim, a, trace, autoreset) for s, lim, a in items]
    procs = min(bench.usable_cpus(), 16, len(jobs))
    if procs <= 1:
        return [_replay_one_local(dataset, j) for j in jobs]
    with mp.get_context("spawn").Pool(procs, initializer=_pool_init, initargs=(dataset,)) as pool:
        return pool.map(_replay_one, jobs, chunksize=max(1, len(jobs) // (4 * procs)))


def _replay_one_local(dataset, job):
    cfg, seed, limit, actions, trace, autoreset = job
    o, ob, ep, dec, last = replay_with_autoreset(cfg, dataset, seed, limit, actions, trace=trace, autoreset=autoreset)
    return o, ob, ep, dec, last


def check_replayed_env(eng, v, ta, tc, i, o, ob, ep, dec, last, what, trace=False):
    c = v["counts"][i]
    assert int(c[_abi.OC_ERR]) == 0, f"{what} env{i} err {int(c[_abi.OC_ERR])}"
    assert int(c[_abi.OC_EPISODE]) == ep, f"{what} env{i} episodes {int(c[_abi.OC_EPISODE])} != {ep}"
    assert int(c[_abi.OC_DECISIONS]) == dec, f"{what} env{i} decisions {int(c[_abi.OC_DECISIONS])} != {dec}"
    assert float(v["wall_time"][i]) == float(o.wall_time), f"{what} env{i} wall time"
    if last is not None:
        assert float(v["reward"][i]) == pytest.approx(float(last), rel=1e-9, abs=1e-12), f"{what} env{i} reward"
    parity.compare_obs(ob, obs_dict(v, i), f"{what} env{i} final")
    for jid, job in o.jobs.items():
        assert ta[i][jid] == job.t_arrival, f"{what} env{i} job {jid} arrival"
        assert tc[i][jid] == job.t_completed or (np.isinf(tc[i][jid]) and np.isinf(job.t_completed)), \
            f"{what} env{i} job {jid} completion"
    if trace:
        n = int(c[_abi.OC_TRACE_LEN])
        ref = [tuple(float(x) if j == 0 else int(x) for j, x in enumerate(r)) for r in o.trace]
        # the device counts every record of the episode but keeps the first trace_cap of them
        kept = min(n, int(eng.layout.trace_cap))
        got = _env_trace(eng, i, kept)
        first = next((k for k, (a, b) in enumerate(zip(got, ref)) if a != b), min(len(got), len(ref)))
        assert len(ref) == n and got == ref[:kept], (
            f"{what} env{i} trace: {n} device records vs {len(ref)} oracle, first difference at {first}: "
            f"{got[first:first + 3]} vs {ref[first:first + 3]}")


def case_bench_rollout_sequence(make, dataset, cfg, B, preroll, warmup, K, stride, mean_limit=None, trace_cap=0,
                                seed=0, rank=0, expect_resident=None, policy="random"):
    """bench.py's rollout sequence verbatim (bench.py main(), rollout mode): the device reset with the rank's shard
    seeds and StochasticTimeLimit draws; the seeded pre-roll of U[0, preroll) decisions per env (ssim_rollout_steps,
    AUTORESET | WARMUP); one warm-up launch of `warmup` steps and the timed launch of K steps, both shared-budget
    launches of B x steps decisions at most 8 x steps per env (ssim_rollout_budget, PREEMPT | AUTORESET); then a
    closing launch of 0 steps, which completes the steps the timed launch preempted. Every launch logs its
    actions; each sampled env's actions, concatenated in launch order and replayed on the oracle with the same
    auto-resets (terminated, or truncated by the time limit), give its episode count, the decisions, wall time,
    job arrival / completion times and final observation of its current episode bit for bit (and, with trace_cap,
    that episode's event trace). Reference: spark_sched_sim.py:127-343 (reset, step, the event loop).
    policy="decima": the budget launches are bench.py's configs[2] persistent Decima rollouts (ssim_decima_rollout:
    features + fused GNN policy + step per env, random-init weights as bench.py), the pre-roll stays random."""
    from spark_sched_sim.distributed import shard_seeds

    SENT = -99
    AR, PRE, WU = _abi.SSIM_ROLLOUT_AUTORESET, _abi.SSIM_ROLLOUT_PREEMPT, _abi.SSIM_ROLLOUT_WARMUP
    kind = _abi.SSIM_POLICY_RANDOM
    eng = make(cfg, B, dataset, trace_cap)
    if expect_resident is not None:
        assert int(eng.layout.lds_resident) == int(expect_resident), "kernel path (LDS / HBM residency)"
    seeds = shard_seeds(rank, B, seed)
    lim = bench_time_limits(mean_limit, seeds)
    eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=lim)
    actions = [[] for _ in range(B)]

    def collect(log):
        lg = np.asarray(eng.to_numpy(log))
        n = 0
        for i in range(B):
            rows = lg[:, i, 0] != SENT
            actions[i].extend(lg[rows, i].tolist())
            n += int(rows.sum())
        return n

    pre = np.random.default_rng([seed, rank, 7]).integers(0, preroll, B).astype(np.int32)
    log = eng.alloc_action_log(int(pre.max()) + 1)
    log.fill_(SENT)
    eng.rollout_steps(kind, 4321, pre, int(pre.max()) + 1, log, flags=AR | WU, time_limits=lim)
    assert collect(log) == int(pre.sum())
    acc0 = np.array(eng.to_numpy(eng.views["acc"]), dtype=np.int64).copy()
    started = 0
    if policy == "decima":
        import torch

        from spark_sched_sim.schedulers.decima import DecimaScheduler

        torch.manual_seed(seed)
        packed = DecimaScheduler(cfg["num_executors"]).to(eng.device).packed_params(eng.device)
        dlim = None if lim is None else torch.tensor(lim, dtype=torch.float64, device=eng.device)

        def budget_launch(c, f, log):
            eng.decima_rollout(packed, seed, 1, 8 * c, B * c, flags=f, time_limits=dlim, action_log=log)
    else:
        def budget_launch(c, f, log):
            eng.rollout_budget(kind, 1234, 8 * c, B * c, log, flags=f, time_limits=lim)
    for c, f in ((warmup, AR | PRE | WU), (K, AR | PRE)):
        log = eng.alloc_action_log(8 * c)
        log.fill_(SENT)
        budget_launch(c, f, log)
        n = collect(log)
        # the launch hands out its budget in chunks of <= 8 decisions; a wave stopped by preemption (or its step cap)
        # while holding part of a chunk leaves that part unstarted, so the steps started are within 8 per env of it
        assert B * c - 8 * B <= n <= B * c, (n, B * c)
        started += n
    pend = np.asarray(eng.to_numpy(eng.views["counts"]))[:, _abi.OC_ERR] & _abi.SSIM_ERR_PENDING
    eng.rollout(kind, 1234, 0, flags=AR, time_limits=lim)  # closing launch: completes the pending steps
    v = eng.host_views()
    ta, tc, _ = eng.job_times_np()
    applied = np.array([len(a) for a in actions])
    d_acc = (np.asarray(v["acc"], dtype=np.int64) - acc0).sum(axis=0)
    assert int(d_acc[_abi.ACC_DECISIONS]) == started  # every started decision completed, none twice
    assert int(np.count_nonzero(v["counts"][:, _abi.OC_ERR])) == 0
    episodes, crossed = 0, 0
    # every stride-th env, plus the first envs (up to 4 more) that went through an auto-reset
    multi = [int(i) for i in np.nonzero(v["counts"][:, _abi.OC_EPISODE] > 1)[0] if i % stride][:4]
    sample = sorted(set(range(0, B, stride)) | set(multi))
    replays = replay_many(cfg, dataset, [(seeds[i], None if lim is None else lim[i], actions[i]) for i in sample],
                          trace=trace_cap > 0)
    for i, (o, ob, ep, dec, last) in zip(sample, replays):
        check_replayed_env(eng, v, ta, tc, i, o, ob, ep, dec, last, "bench-sequence", trace=trace_cap > 0)
        episodes += ep
        crossed += ep > 1
    return {"pending_at_timed_end": int(np.count_nonzero(pend)), "episodes_replayed": episodes,
            "crossed_replayed": crossed, "decisions_replayed": int(applied[sample].sum()), "envs_replayed": len(sample),
            "episodes_total": int(v["counts"][:, _abi.OC_EPISODE].sum())}
