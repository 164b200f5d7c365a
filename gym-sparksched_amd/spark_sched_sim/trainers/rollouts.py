"""GPU rollout collection (trainers/rollout_worker.py:18-46, 135-157: RolloutBuffer, RolloutWorkerSync).

All envs of one GPU step together: every decision is one batched Decima forward (DecimaScheduler.schedule)
over the envs still running, one ssim_step launch, and the observation, action, log-probability, reward and
wall time of every live env are appended to a device-resident buffer. An env is done when terminated or
truncated by its StochasticTimeLimit (wrappers/stochastic_time_limit.py:26-31); from then on it is held with
an invalid action (the engine leaves its state untouched, SSIM_ERR_SPACE) until the next collection.
The reference runs one env per process (RolloutWorkerSync); here a "worker" is a row of the batch.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _abi
from ..wrappers import StochasticTimeLimitSampler
from ..schedulers.decima import live_sizes, DagBatch, build_batch, cat_batches, select_envs


class GpuRolloutBuffer:
    """Per decision step t: the live envs' observations as one DagBatch (select_envs order = `envs[t]`),
    actions, log-probs, rewards and the wall time before the step. `trajectories()` pads per-env rows."""

    def __init__(self, num_envs: int):
        self.num_envs = num_envs
        self.batches: list[DagBatch] = []
        self.envs: list[torch.Tensor] = []
        self.stage_idx: list[torch.Tensor] = []
        self.job_idx: list[torch.Tensor] = []
        self.exec_idx: list[torch.Tensor] = []
        self.lgprobs: list[torch.Tensor] = []
        self.num_exec: list[torch.Tensor] = []  # the action the env applied (DecimaActWrapper: 1 + exec_idx)
        self.rewards: list[torch.Tensor] = []
        self.wall_before: list[torch.Tensor] = []
        self.final_wall: torch.Tensor | None = None

    def add(self, batch, envs, act, reward, wall_before):
        self.batches.append(batch)
        self.envs.append(envs)
        self.stage_idx.append(act["stage_idx"][envs].long())
        self.job_idx.append(act["job_idx"][envs])
        self.exec_idx.append(act["exec_idx"][envs])
        self.lgprobs.append(act["lgprob"][envs])
        self.num_exec.append(act["num_exec"][envs])
        self.rewards.append(reward)
        self.wall_before.append(wall_before)

    def __len__(self) -> int:
        return int(sum(e.numel() for e in self.envs))

    def trajectories(self):
        """Padded per-env rows: times [B, T+1] (wall before each decision, then the final wall time),
        rewards [B, T], lengths [B], and for each (env, k) its flat sample index into `samples()`."""
        dev = self.final_wall.device
        B = self.num_envs
        env = torch.cat(self.envs)
        lengths = torch.bincount(env, minlength=B)
        T = int(lengths.max().item()) if env.numel() else 0
        # position of each sample in its env row = number of earlier samples of that env
        order = torch.arange(env.numel(), device=dev)
        pos = torch.zeros_like(env)
        # steps are appended in time order, so a stable sort by env keeps each env's decisions in order
        perm = torch.argsort(env, stable=True)
        starts = torch.cumsum(lengths, 0) - lengths
        pos[perm] = order - starts[env[perm]]
        times = torch.zeros((B, T + 1), dtype=torch.float64, device=dev)
        rewards = torch.zeros((B, T), dtype=torch.float64, device=dev)
        times[env, pos] = torch.cat(self.wall_before)
        rewards[env, pos] = torch.cat(self.rewards)
        times[torch.arange(B, device=dev), lengths] = self.final_wall
        sample = torch.full((B, T), -1, dtype=torch.long, device=dev)
        sample[env, pos] = order
        return times, rewards, lengths, sample

    def samples(self) -> tuple[DagBatch, dict[str, torch.Tensor]]:
        """All stored observations as one DagBatch (sample i = observation row i) and the flat actions."""
        acts = {"stage_idx": torch.cat(self.stage_idx), "job_idx": torch.cat(self.job_idx),
                "exec_idx": torch.cat(self.exec_idx), "lgprob": torch.cat(self.lgprobs)}
        return cat_batches(self.batches), acts


class RolloutCollector:
    """Drives a DeviceEngine (or the test-only HostEngine) with a DecimaScheduler until every env is done."""

    def __init__(self, engine, policy, num_tasks_scale: float = 200.0, work_scale: float = 1e5, fused: bool = True,
                 seed: int = 0, row_offset: int = 0):
        self.engine = engine
        self.policy = policy
        # global id of the engine's env 0: actions are sampled from a counter-based stream of (seed, decision
        # counter, global row), so a row draws the same actions whichever rank holds it
        self.row_offset = int(row_offset)
        self.scales = (num_tasks_scale, work_scale)
        from ..schedulers.decima import DECIMA_PARAMS

        # the fused kernel implements the decima_tpch.yaml architecture only
        self.fused = fused and sum(p.numel() for p in policy.parameters()) == DECIMA_PARAMS
        self.seed = seed
        # decision counter of the sampling stream: (collect call << 32) + decision index within the call. A row
        # takes its k-th decision of a call at loop step k on any rank, so the stream is rank-independent.
        self.calls = 0
        self.counter = 0
        self.on_device = isinstance(engine.views["counts"], torch.Tensor)  # DeviceEngine vs test host build
        self._params = None  # packed policy weights, valid during one collect()
        self._pre = None  # (views, feats, live ids, batch sizes) fetched by _live for the next step
        from ..metrics import RowStats

        self.stats = RowStats(engine.num_envs)  # per-row collect_stats, duration windows across episodes

    def row_stats(self) -> torch.Tensor:
        """rollout_worker.py:122-129 per row, float64 [B, 4] on the policy's device (metrics.RowStats)."""
        return torch.from_numpy(self.stats.stats(self.engine)).to(self.policy.device)

    def _views(self, features: bool = True):
        eng = self.engine
        if self.on_device:
            return eng.views, (eng.decima_features(*self.scales) if features else None)
        dev = self.policy.device  # host build: numpy views -> tensors on the policy's device
        v = {k: torch.from_numpy(x).to(dev) for k, x in eng.host_views().items() if k != "trace"}
        if not features:
            return v, None
        f = {k: torch.from_numpy(x).to(dev) for k, x in eng.decima_features_np(*self.scales).items()}
        return v, f

    def _decide_and_step(self, alive: torch.Tensor, generator=None, all_alive: bool = False,
                         envs: torch.Tensor | None = None):
        """One batched decision for the `alive` envs (the others get an invalid action and stay untouched),
        then one engine step. Returns (live env ids, their observations as a DagBatch, action dict, views).
        `all_alive` (known to the caller): the full batch already is the live envs' batch (no re-selection);
        `envs` (optional): the caller's nonzero(alive)."""
        eng = self.engine
        if self._pre is not None:  # views, features and live sizes already fetched by the loop (live())
            v, f, envs, sizes = self._pre
            self._pre = None
        else:
            v, f = self._views()
            sizes = None
        if envs is None:
            envs = torch.nonzero(alive).squeeze(1)
        if self.on_device and self.fused:  # one fused kernel launch (ssim_decima_policy)
            # the policy reads the obs arena itself: only the live envs' batch is built (for the buffer),
            # its sizes (from the loop's one sync) also give the LDS node cap
            batch = build_batch(v, f, envs=None if all_alive else envs, sizes=sizes)
            self.counter += 1
            if self._params is None:  # weights are fixed for a whole collect(): pack them once
                self._params = self.policy.packed_params(eng.device)
            # the kernel hashes (local env * C + counter); adding row_offset * C to the counter makes that the
            # hash of the global row (C = 0x9E3779B97F4A7C15, csrc/decima_policy.h decima_policy_env)
            ctr = (self.counter + self.row_offset * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
            fo = self.policy.schedule_fused(eng, f, seed=self.seed, counter=ctr, env_mask=alive,
                                            node_cap=batch.max_nodes, params=self._params)
            act = {"stage_idx": fo["stage_idx"], "num_exec": fo["num_exec"], "job_idx": fo["job_idx"].long(),
                   "exec_idx": fo["exec_idx"].long(), "lgprob": fo["lgprob"]}
        else:
            b_all = build_batch(v, f, env_mask=alive)
            self.counter += 1
            rows = self.row_offset + torch.arange(b_all.num_envs, device=b_all.x.device)
            act = self.policy.schedule(b_all, stream=(self.seed, self.counter, rows))
            batch = b_all if all_alive else select_envs(b_all, envs)
        si = torch.where(alive, act["stage_idx"], torch.full_like(act["stage_idx"], -2))
        if self.on_device:
            eng.step(si, act["num_exec"])
        else:
            eng.step(si.cpu().numpy(), act["num_exec"].cpu().numpy())
        v, _ = self._views(features=False)
        return envs, batch, act, v

    def _live(self, alive: torch.Tensor) -> torch.Tensor:
        """Live env ids for the next decision. Device fused path: the step's single host sync (live_sizes),
        with the views/features kept for _decide_and_step; otherwise a plain nonzero."""
        if self.on_device and self.fused:
            v, f = self._views()
            envs, sizes = live_sizes(v, f, alive)
            self._pre = (v, f, envs, sizes)
            return envs
        self._pre = None
        return torch.nonzero(alive).squeeze(1)

    @staticmethod
    def _done(v) -> torch.Tensor:
        c = v["counts"]
        return (c[:, _abi.OC_TERMINATED] != 0) | (c[:, _abi.OC_TRUNCATED] != 0)

    @torch.no_grad()
    def collect(self, seeds, time_limits=None, generator=None, max_steps: int = 10**9) -> GpuRolloutBuffer:
        """RolloutWorkerSync.collect_rollout (rollout_worker.py:135-157): reset every env with its seed,
        step until each env's episode ends."""
        self._params = None  # re-pack the (possibly updated) policy weights
        self.calls += 1
        self.counter = self.calls << 32
        eng = self.engine
        B = eng.num_envs
        limits = None if time_limits is None else torch.as_tensor(time_limits, dtype=torch.float64)
        self.stats.flush(range(B), eng)  # the finished episodes' completions enter the duration windows
        eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds,
                          time_limits=None if limits is None else limits.cpu().numpy())
        v, _ = self._views(features=False)
        dev = v["counts"].device
        buf = GpuRolloutBuffer(B)
        alive = torch.ones(B, dtype=torch.bool, device=dev)
        wall = torch.zeros(B, dtype=torch.float64, device=dev)
        for _ in range(max_steps):
            envs = self._live(alive)  # the loop's one size sync
            if envs.numel() == 0:
                break
            envs, batch, act, v = self._decide_and_step(alive, generator, all_alive=envs.numel() == B, envs=envs)
            reward = v["reward"][envs].double()
            buf.add(batch, envs, act, reward, wall[envs])
            wall = torch.where(alive, v["wall_time"].double(), wall)
            alive = alive & ~self._done(v)
        buf.final_wall = wall
        return buf


class DecimaSampleArena:
    """Device sample arena of the persistent Decima rollout (include/sparksched.h ssim_decima_samples): per env, one
    64-B record per decision and the decision's observation as node / edge / DAG rows. Regions grow (doubling, the
    used prefix copied) when the kernel reports one full; the env then continues where it stopped."""

    def __init__(self, num_envs: int, device, cap_samples: int = 1024, cap_nodes: int = 1 << 16,
                 cap_edges: int = 1 << 16, cap_dags: int = 1 << 14):
        self.B = num_envs
        self.device = device
        i32 = dict(dtype=torch.int32, device=device)
        self.cursor = torch.zeros((num_envs, _abi.CURSOR_WORDS), **i32)
        self.caps = [int(cap_samples), int(cap_nodes), int(cap_edges), int(cap_dags)]
        self.rec = torch.zeros((num_envs, self.caps[0], _abi.SAMPLE_BYTES // 4), **i32)
        self.nodes = torch.zeros((num_envs, self.caps[1], 6), dtype=torch.float32, device=device)
        self.edges = torch.zeros((num_envs, self.caps[2], 4), **i32)
        self.dags = torch.zeros((num_envs, self.caps[3], 2), **i32)

    def struct(self) -> _abi.SsimDecimaSamples:
        return _abi.SsimDecimaSamples(self.cursor.data_ptr(), self.rec.data_ptr(), self.nodes.data_ptr(),
                                      self.edges.data_ptr(), self.dags.data_ptr(), *self.caps)

    def clear(self) -> None:
        self.cursor.zero_()

    @staticmethod
    def _grown(t: torch.Tensor, cap: int) -> torch.Tensor:
        out = torch.zeros((t.shape[0], cap) + tuple(t.shape[2:]), dtype=t.dtype, device=t.device)
        out[:, : t.shape[1]] = t
        return out

    @staticmethod
    def required(cur: np.ndarray) -> list[int]:
        """Per region (samples, node rows, edge rows, DAG rows): what the full envs' stopped observations need, i.e.
        the rows used plus the rows the kernel recorded for the observation that did not fit (cursor[5..7])."""
        f = cur[cur[:, _abi.CUR_FULL] != 0]
        need = [f[:, _abi.CUR_SAMPLES] + 1, f[:, _abi.CUR_NODES] + f[:, _abi.CUR_NEED_NODES],
                f[:, _abi.CUR_EDGES] + f[:, _abi.CUR_NEED_EDGES], f[:, _abi.CUR_DAGS] + f[:, _abi.CUR_NEED_DAGS]]
        return [int(n.max()) if len(n) else 0 for n in need]

    def grow(self, cur: np.ndarray) -> None:
        """After a launch that left envs with the full flag: every region a stopped observation overflows is grown
        (doubling until it fits) so the next launch records it, then the flags are cleared."""
        names = ["rec", "nodes", "edges", "dags"]
        for i, req in enumerate(self.required(cur)):
            if req > self.caps[i]:
                cap = self.caps[i]
                while cap < req:
                    cap *= 2
                self.caps[i] = cap
                setattr(self, names[i], self._grown(getattr(self, names[i]), cap))
        self.cursor[:, _abi.CUR_FULL:] = 0  # the flags and the recorded needs

    def buffer(self, final_wall: torch.Tensor) -> "ArenaRolloutBuffer":
        return ArenaRolloutBuffer(self, final_wall)


class ArenaRolloutBuffer:
    """GpuRolloutBuffer's interface over a DecimaSampleArena: samples in env-major order (env 0's decisions in
    order, then env 1's, ...), built into one DagBatch with a fixed number of launches (no per-step batches)."""

    row_major = True  # samples() is already in (row, decision) order

    def __init__(self, arena: DecimaSampleArena, final_wall: torch.Tensor):
        self.arena = arena
        self.num_envs = arena.B
        self.final_wall = final_wall
        self.lengths = arena.cursor[:, _abi.CUR_SAMPLES].long()
        self._n = int(self.lengths.sum().item())
        self._rows = None

    def __len__(self) -> int:
        return self._n

    def _sample_rows(self):
        """(env, k) of every sample in env-major order and its record fields."""
        if self._rows is None:
            a = self.arena
            B = self.num_envs
            dev = a.cursor.device
            env = torch.repeat_interleave(torch.arange(B, device=dev), self.lengths, output_size=self._n)
            k = torch.arange(self._n, device=dev) - (torch.cumsum(self.lengths, 0) - self.lengths)[env]
            rec = a.rec[env, k]  # [n, 16] int32 words
            self._rows = (env, k, rec)
        return self._rows

    def trajectories(self):
        B = self.num_envs
        dev = self.final_wall.device
        env, k, rec = self._sample_rows()
        T = int(self.lengths.max().item()) if self._n else 0
        f64 = rec.view(torch.float64)  # [n, 8]
        times = torch.zeros((B, T + 1), dtype=torch.float64, device=dev)
        rewards = torch.zeros((B, T), dtype=torch.float64, device=dev)
        times[env, k] = f64[:, _abi.SAMPLE_WALL]
        rewards[env, k] = f64[:, _abi.SAMPLE_REWARD]
        times[torch.arange(B, device=dev), self.lengths] = self.final_wall.double()
        sample = torch.full((B, T), -1, dtype=torch.long, device=dev)
        sample[env, k] = torch.arange(self._n, device=dev)
        return times, rewards, self.lengths, sample

    def samples(self):
        from ..schedulers.decima import _expand, _excl, _ptr

        a = self.arena
        env, _, rec = self._sample_rows()
        dev = rec.device
        f = {name: rec[:, i].long() for i, name in enumerate(_abi.SAMPLE_I32)}
        n, ne, nj = f["num_nodes"], f["num_edges"], f["num_dags"]
        Ns = self._n
        if Ns:
            Nt, Et, Gt, L, Nmax = (int(v) for v in torch.stack(
                [n.sum(), ne.sum(), nj.sum(), (torch.clamp(f["depth"] - 1, min=0) * (n > 0)).max(),
                 n.max()]).tolist())
        else:
            Nt = Et = Gt = L = Nmax = 0
        node_s, nl = _expand(n, Nt)
        node_src = env[node_s] * a.caps[1] + f["node_off"][node_s] + nl
        rows = a.nodes.reshape(-1, 6)[node_src]
        edge_s, el = _expand(ne, Et)
        edge_src = env[edge_s] * a.caps[2] + f["edge_off"][edge_s] + el
        erows = a.edges.reshape(-1, 4)[edge_src]
        dag_s, dl = _expand(nj, Gt)
        dag_src = env[dag_s] * a.caps[3] + f["dag_off"][dag_s] + dl
        drows = a.dags.reshape(-1, 2)[dag_src].long()
        node_base = _excl(n)
        stage_mask = rows[:, 5] != 0
        node_dag, _ = _expand(drows[:, 0], Nt)
        from ..schedulers.decima import DagBatch

        batch = DagBatch(
            x=rows[:, :5].contiguous(),
            edge_index=(erows[:, :2].long() + node_base[edge_s][:, None]).t().contiguous(),
            edge_bits=erows[:, 2].contiguous(), max_levels=L,
            env_levels=torch.clamp(f["depth"] - 1, min=0) * (n > 0), ptr=_ptr(drows[:, 0]), node_dag=node_dag,
            node_env=node_s, dag_env=dag_s, obs_ptr=_ptr(nj), stage_mask=stage_mask, exec_cap=drows[:, 1],
            num_stage_acts=torch.zeros(Ns, dtype=torch.long, device=dev).index_add_(0, node_s, stage_mask.long()),
            num_nodes=n, num_edges=ne, num_envs=Ns, max_nodes=Nmax)
        acts = {"stage_idx": f["stage_idx"], "job_idx": f["job_idx"], "exec_idx": f["exec_idx"],
                "lgprob": rec[:, _abi.SAMPLE_LGPROB].view(torch.float32).contiguous()}
        return batch, acts


class DeviceRolloutCollector(RolloutCollector):
    """RolloutWorkerSync.collect_rollout (rollout_worker.py:135-157) for every row at once in ONE kernel launch
    (ssim_decima_rollout, csrc/decima_rollout.h): each env's wave runs its own decision loop (features, fused Decima
    policy, step) until its episode ends and leaves every decision in a DecimaSampleArena. Same sampling stream as
    RolloutCollector's fused path (counter = call << 32 + decision index + 1, keyed by the global row), so both draw
    the same actions from the same observations."""

    def __init__(self, engine, policy, **kw):
        super().__init__(engine, policy, **kw)
        if not (self.on_device and self.fused):
            raise ValueError("DeviceRolloutCollector needs a DeviceEngine and the decima_tpch.yaml architecture")
        self.arena = DecimaSampleArena(engine.num_envs, engine.device)
        self.launches = 0

    @torch.no_grad()
    def collect(self, seeds, time_limits=None, generator=None, max_steps: int = 10**9) -> ArenaRolloutBuffer:
        self.calls += 1
        eng = self.engine
        B = eng.num_envs
        limits = None if time_limits is None else np.asarray(time_limits, dtype=np.float64)
        self.stats.flush(range(B), eng)
        eng.reset_sampled(_abi.SSIM_RESET_SEED, seeds=seeds, time_limits=limits)
        params = self.policy.packed_params(eng.device)
        ctr = ((self.calls << 32) + 1 + self.row_offset * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        self.arena.clear()
        steps = int(min(max_steps, 2**31 - 1))
        while True:
            eng.decima_rollout(params, self.seed, ctr, steps, samples=self.arena, num_tasks_scale=self.scales[0],
                               work_scale=self.scales[1])
            self.launches += 1
            cur = self.arena.cursor.cpu().numpy()
            if not (cur[:, _abi.CUR_FULL] != 0).any():
                break
            self.arena.grow(cur)
        err = eng.views["counts"][:, _abi.OC_ERR].cpu().numpy() & _abi.SSIM_ERR_STICKY
        if err.any():  # e.g. an action the engine refused (frozen with SSIM_ERR_INVARIANT): its samples are invalid
            bad = np.flatnonzero(err)
            raise RuntimeError(f"decima rollout: envs {bad[:8].tolist()} frozen with error bits "
                               f"{[hex(int(x)) for x in err[bad[:8]]]}")
        wall = eng.views["wall_time"].double().clone()
        return self.arena.buffer(wall)


class AsyncRolloutCollector(RolloutCollector):
    """RolloutWorkerAsync (rollout_worker.py:160-206): model updates at regular intervals of simulated time,
    regardless of episode boundaries. Each env (a "worker" row) keeps its episode across `collect` calls and
    steps until `rollout_duration` ms of simulated time have elapsed in this call; an env whose episode ends
    is reset in place with seed = base_seed + seed_step * reset_count (rollout_worker.py:118-120) and a new
    StochasticTimeLimit draw. Times stored in the buffer are the elapsed time of the call (the reference's
    `elapsed_time`), so the buffer feeds the same returns/baseline code as the sync collector; `buf.resets`
    holds (env, step) pairs like RolloutBuffer.add_reset (the reference's returns ignore them too)."""

    def __init__(self, engine, policy, rollout_duration: float, base_seeds, seed_step: int,
                 mean_time_limit: float | None = None, **kw):
        super().__init__(engine, policy, **kw)
        B = engine.num_envs
        self.rollout_duration = float(rollout_duration)
        self.base_seeds = np.asarray(base_seeds, dtype=np.int64).reshape(B)
        self.seed_step = int(seed_step)
        self.reset_count = np.zeros(B, dtype=np.int64)
        self.limits = None if not mean_time_limit else StochasticTimeLimitSampler(mean_time_limit, B)
        self.next_wall = None  # wall time before each env's next decision (0 after a reset)

    def _reset(self, env_ids: np.ndarray) -> None:
        B = self.engine.num_envs
        mode = np.zeros(B, dtype=np.uint8)
        seeds = np.zeros(B, dtype=np.uint64)
        lim = np.full(B, np.inf)
        mode[env_ids] = _abi.SSIM_RESET_SEED
        self.stats.flush(env_ids, self.engine)  # the finished episodes' completions enter the duration windows
        for e in env_ids:
            seeds[e] = int(self.base_seeds[e] + self.seed_step * self.reset_count[e])
            if self.limits is not None:
                lim[e] = self.limits.sample(int(e), int(seeds[e]))
        self.reset_count[env_ids] += 1
        self.engine.reset_sampled(mode, seeds=seeds, time_limits=None if self.limits is None else lim)

    @torch.no_grad()
    def collect(self, generator=None, max_steps: int = 10**9) -> GpuRolloutBuffer:
        self._params = None  # re-pack the (possibly updated) policy weights
        self.calls += 1
        self.counter = self.calls << 32
        B = self.engine.num_envs
        if self.next_wall is None:  # first call: reset every worker (rollout_worker.py:174-176)
            self._reset(np.arange(B))
        v, _ = self._views(features=False)
        dev = v["counts"].device
        if self.next_wall is None:
            self.next_wall = torch.zeros(B, dtype=torch.float64, device=dev)
        buf = GpuRolloutBuffer(B)
        buf.resets = []
        elapsed = torch.zeros(B, dtype=torch.float64, device=dev)
        step = torch.zeros(B, dtype=torch.long, device=dev)
        alive = elapsed < self.rollout_duration
        for _ in range(max_steps):
            envs = self._live(alive)  # the loop's one size sync
            if envs.numel() == 0:
                break
            envs, batch, act, v = self._decide_and_step(alive, generator, all_alive=envs.numel() == B, envs=envs)
            reward = v["reward"][envs].double()
            buf.add(batch, envs, act, reward, elapsed[envs])
            new_wall = v["wall_time"].double()
            elapsed = torch.where(alive, elapsed + (new_wall - self.next_wall), elapsed)
            self.next_wall = torch.where(alive, new_wall, self.next_wall)
            done = alive & self._done(v)
            if bool(done.any()):
                ids = torch.nonzero(done).squeeze(1)
                buf.resets += [(int(e), int(k)) for e, k in zip(ids.tolist(), step[ids].tolist())]
                self._reset(ids.cpu().numpy())
                self.next_wall[ids] = 0.0
            step += alive.long()
            alive = alive & (elapsed < self.rollout_duration)
        buf.final_wall = elapsed
        return buf
