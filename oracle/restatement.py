"""CPU restatement of the reference Spark scheduling simulator — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module. The product (``gym-sparksched_amd/``) never imports, links or executes anything in ``oracle/``.

What it restates (reference snapshot 2025-02-22, paths under /root/reference):
  * ``spark_sched_sim/spark_sched_sim.py`` (env: reset/step/observe/event handlers/helpers)
  * ``spark_sched_sim/components/{event,executor_tracker,job,stage,executor,task}.py``
  * ``spark_sched_sim/data_samplers/tpch.py`` (job sequence, preprocessing, task durations)
  * ``spark_sched_sim/utils.py`` (subgraph), ``spark_sched_sim/metrics.py``

Parity status. The reference cannot be imported or run in this pipeline (environment denial recorded in
SURVEY.md §8c; gymnasium, networkx-era deps and the TPC-H data are absent as well), and its test suite holds
no golden vectors or known-answer tests. This restatement therefore relies on the *same
third-party machinery the reference relies on* — real CPython 3.10 ``set``/``dict``/``heapq`` and numpy's
``Generator(PCG64(SeedSequence(seed)))`` — so set iteration order, dict insertion order, heap tie-breaks and
RNG consumption are reference-faithful by construction; those boundaries are pinned by the KATs in
``tests/test_oracle_kats.py``. End-to-end parity against the reference itself is **unpinned** (no reference
run and no reference fixtures exist); the committed fixtures in ``tests/golden/`` are produced by this module.

Only behaviour on the hot path is restated; drawing (``renderer.py``, pygame) is out of scope, but the data
the renderer draws — ``Executor.history`` (executor.py:22-44, appended at spark_sched_sim.py:445,782) — is
kept, as the checker of the device's render-history export.
"""

from __future__ import annotations

import bisect
import copy
import heapq
import itertools
from collections import deque, namedtuple

import numpy as np

QUERY_SIZES = ["2g", "5g", "10g", "20g", "50g", "80g", "100g"]  # tpch.py:14
NUM_QUERIES = 22  # tpch.py:15
EXEC_LEVELS = [5, 10, 20, 40, 50, 60, 80, 100]  # tpch.py:238

COMMON = (None, None)  # executor_tracker.py:10 COMMON_POOL_KEY
ARRIVAL, TASK_DONE, EXEC_READY = 1, 2, 3  # event.py:9-12 (auto() order)
JOB_DONE = 4  # trace-only record kind (job completion, spark_sched_sim.py:682-697)
TO_COMMON = 5  # trace-only record kind (executor released to the common pool, spark_sched_sim.py:779-782)

GraphInstance = namedtuple("GraphInstance", ["nodes", "edges", "edge_links"])  # gymnasium.spaces.GraphInstance


# ----------------------------------------------------------------------------------------------------------
# numpy-faithful helpers that the product also precomputes (dataset packer); restated independently here
# ----------------------------------------------------------------------------------------------------------

def executor_intervals(exec_cap: int) -> np.ndarray:
    """tpch.py:237-262 — float table [exec_cap+1, 2] of (left, right) executor-count data points."""
    iv = np.zeros((exec_cap + 1, 2))
    iv[: EXEC_LEVELS[0] + 1] = EXEC_LEVELS[0]
    for i in range(len(EXEC_LEVELS) - 1):
        lo, hi = EXEC_LEVELS[i], EXEC_LEVELS[i + 1]
        iv[lo + 1: hi] = (lo, hi)
        if hi > exec_cap:
            break
        iv[hi] = hi
    if exec_cap > EXEC_LEVELS[-1]:
        iv[EXEC_LEVELS[-1] + 1: exec_cap] = EXEC_LEVELS[-1]
    return iv


def preprocess_durations(td: dict) -> None:
    """tpch.py:135-159 — drop fresh durations (as a multiset) from first_wave, then fill empty first-wave
    lists with the previous non-empty one in ascending key order. Mutates ``td`` like the reference."""
    cleaned = {}
    for key in td["first_wave"]:
        pending = {}
        for d in td["fresh_durations"][key]:
            pending[d] = pending.get(d, 0) + 1
        kept = []
        for d in td["first_wave"][key]:
            if d in pending:
                pending[d] -= 1
                if pending[d] == 0:
                    del pending[d]
            else:
                kept.append(d)
        cleaned[key] = kept
    carry = []
    for key in sorted(cleaned):
        if not cleaned[key]:
            cleaned[key] = carry
        carry = cleaned[key]
    td["first_wave"] = cleaned


def rough_duration(td: dict) -> float:
    """tpch.py:162-174 — numpy mean over fresh + (cleaned) first + rest, dict-value order."""
    flat = []
    for wave in ("fresh_durations", "first_wave", "rest_wave"):
        for lst in td[wave].values():
            flat.extend(lst)
    return np.mean(flat)


# ----------------------------------------------------------------------------------------------------------
# entity records (components/*.py); Task objects are not materialised: only task.stage_id is ever read
# ----------------------------------------------------------------------------------------------------------

class _Stage:
    __slots__ = ("job", "sid", "num_tasks", "remaining", "executing", "done", "recent", "data", "flag")

    def __init__(self, job, sid, num_tasks, rough, data):  # stage.py:5-18
        self.job, self.sid, self.num_tasks = job, sid, num_tasks
        self.remaining, self.executing, self.done = num_tasks, 0, 0
        self.recent, self.data, self.flag = rough, data, False

    @property
    def key(self):  # stage.py:28-30 pool_key
        return (self.job, self.sid)

    @property
    def completed(self):  # stage.py:36-38
        return self.done == self.num_tasks


class _Job:
    __slots__ = ("jid", "stages", "active", "frontier", "children", "parents", "edges",
                 "t_arrival", "t_completed", "local", "saturated_count", "query", "size")

    def __init__(self, jid, stages, edges, t_arrival):  # job.py:12-43
        self.jid, self.stages, self.edges, self.t_arrival = jid, stages, edges, t_arrival
        n = len(stages)
        self.children = [[] for _ in range(n)]
        self.parents = [[] for _ in range(n)]
        for u, v in edges:
            self.children[u].append(v)
            self.parents[v].append(u)
        self.active = list(range(n))
        self.t_completed = np.inf
        self.local = set()
        self.saturated_count = 0
        self.frontier = {s for s in range(n) if not self.parents[s]}  # job.py:93-111

    @property
    def saturated(self):  # job.py:52-53
        return self.saturated_count == len(self.stages)


class _Executor:
    __slots__ = ("eid", "task_stage", "job", "executing", "history")

    def __init__(self, eid):  # executor.py:5-27
        self.eid, self.task_stage, self.job, self.executing = eid, None, None, False
        self.history = [[None, -1]]  # render-only (executor.py:22-25)

    def add_history(self, wall_time, job_id):  # executor.py:34-44
        if len(self.history) > 0:
            self.history[-1][0] = wall_time
        self.history += [[None, job_id]]


class InvariantError(AssertionError):
    """An ``assert`` of the reference fired (same class of failure as the reference's AssertionError)."""


def _check(cond, where):
    if not cond:
        raise InvariantError(where)


# ----------------------------------------------------------------------------------------------------------
# the sampler (data_samplers/tpch.py)
# ----------------------------------------------------------------------------------------------------------

class TpchSamplerOracle:
    def __init__(self, cfg: dict, dataset: dict):  # tpch.py:19-49 (no download: dataset passed in)
        self.cap = cfg["job_arrival_cap"]
        self.mean_gap = 1 / cfg["job_arrival_rate"]
        self.warmup = cfg["warmup_delay"]
        self.intervals = executor_intervals(cfg["num_executors"])
        self.dataset = dataset
        self.rng = None

    def job_sequence(self, horizon):  # tpch.py:54-73
        seq, t, k = [], 0, 0
        while t < horizon and (not self.cap or k < self.cap):
            seq.append((t, self._sample_job(k, t)))
            t += self.rng.exponential(self.mean_gap)
            k += 1
        return seq

    def _sample_job(self, jid, t_arrival):  # tpch.py:176-206
        q = 1 + self.rng.integers(NUM_QUERIES)
        size = self.rng.choice(QUERY_SIZES)
        adj, tds = self.dataset[(int(q), str(size))]
        tds = copy.deepcopy(tds)  # the reference re-loads the .npy files for every job
        stages = []
        for sid in range(adj.shape[0]):
            d = tds[sid]
            k0 = next(iter(d["first_wave"]))
            nt = len(d["first_wave"][k0]) + len(d["rest_wave"][k0])
            preprocess_durations(d)
            stages.append(_Stage(jid, sid, nt, rough_duration(d), d))
        rows, cols = np.nonzero(adj)  # networkx from_numpy_array edge order = row-major nonzeros
        job = _Job(jid, stages, [(int(u), int(v)) for u, v in zip(rows, cols)], t_arrival)
        job.query, job.size = int(q), str(size)
        return job

    def _pick_key(self, data, n_local):  # tpch.py:216-235
        lo, hi = self.intervals[n_local]
        if lo == hi:
            key = lo
        else:
            pt = 1 + int(self.rng.random() * (hi - lo))
            key = lo if pt <= n_local - lo else hi
        if key not in data["first_wave"]:
            key = max(data["first_wave"])
        return key

    def _draw(self, data, wave, key, warm=False):  # tpch.py:208-214
        durations = data[wave][key]
        d = self.rng.choice(durations)
        if warm:
            d += self.warmup
        return d

    def task_duration(self, job: _Job, stage: _Stage, executor: _Executor):  # tpch.py:75-106
        n_local = len(job.local)
        _check(n_local > 0, "[task_duration]")
        data = stage.data
        key = self._pick_key(data, n_local)
        if executor.task_stage is None:
            try:
                return self._draw(data, "fresh_durations", key)
            except (ValueError, KeyError):
                return self._draw(data, "first_wave", key, warm=True)
        if executor.task_stage == stage.sid:
            try:
                return self._draw(data, "rest_wave", key)
            except (ValueError, KeyError):
                pass
        try:
            return self._draw(data, "first_wave", key)
        except (ValueError, KeyError):
            return self._draw(data, "fresh_durations", key)


# ----------------------------------------------------------------------------------------------------------
# the environment (spark_sched_sim.py + components/executor_tracker.py + components/event.py)
# ----------------------------------------------------------------------------------------------------------

class SparkSchedOracle:
    """Single-env CPU restatement. Same call surface as the reference env (reset/step)."""

    def __init__(self, env_cfg: dict, dataset: dict):  # spark_sched_sim.py:34-125
        self.N = env_cfg["num_executors"]
        self.moving_delay = env_cfg["moving_delay"]
        self.beta = env_cfg.get("beta", 0)
        self.job_arrival_cap = env_cfg.get("job_arrival_cap")
        self.sampler = TpchSamplerOracle(env_cfg, dataset)
        self.rng = None
        self.wall_time = 0
        self.duration_buff = deque(maxlen=200)
        self.stage_idx_n = 1  # action_space["stage_idx"] = Discrete(n, start=-1)
        self.trace = None  # optional event log for fixtures: list of tuples

    # ---- tracker (executor_tracker.py) ------------------------------------------------------------------
    def _tracker_reset(self):  # executor_tracker.py:32-70
        n = self.N
        self.loc = {e: COMMON for e in range(n)}
        self.pools = {None: set(), COMMON: set(range(n))}
        self.commits = {None: {}, COMMON: {}}
        self.commits_from = {None: 0, COMMON: 0}
        self.commits_to = {COMMON: 0}
        self.moving_to = {}
        self.supply = {None: 0}
        self.source = COMMON

    def _source_job(self):  # executor_tracker.py:98-102
        if not self.source or self.source is COMMON:
            return None
        return self.source[0]

    def _committable(self):  # executor_tracker.py:105-111
        n = len(self.pools[self.source]) - self.commits_from[self.source]
        _check(n >= 0, "[num_committable_execs]")
        return n

    def _add_commitment(self, n, dst):  # executor_tracker.py:146-154, 224-236
        _check(self.source, "[add_commitment]")
        src = self.source
        row = self.commits[src]
        row[dst] = row[dst] + n if dst in row else n
        self.commits_from[src] += n
        self.commits_to[dst] += n
        _check(len(self.pools[src]) >= self.commits_from[src], "[_increment_commitments]")
        if dst[0] != src[0]:
            self.supply[dst[0]] += n

    def _remove_commitment(self, e, dst):  # executor_tracker.py:156-173, 238-249
        src = self.loc[e]
        _check(src, "[remove_commitment]")
        if dst not in self.commits[src]:
            raise ValueError(f"no commitments from {src} to {dst}")
        self.commits[src][dst] -= 1
        self.commits_from[src] -= 1
        self.commits_to[dst] -= 1
        _check(self.commits_from[src] >= 0 and self.commits_to[dst] >= 0, "[_decrement_commitments]")
        if self.commits[src][dst] == 0:
            self.commits[src].pop(dst)
        if dst[0] != src[0]:
            self.supply[dst[0]] -= 1
            _check(self.supply[dst[0]] >= 0, "[remove_commitment] supply")
        return src

    def _peek_commitment(self, pool):  # executor_tracker.py:175-180
        row = self.commits.get(pool)
        if not row:
            return None
        return next(iter(row))

    def _move_to_pool(self, e, dst, send=False):  # executor_tracker.py:186-220
        if send and (not dst or dst[0] is None or dst[1] is None):
            raise ValueError("can only send executors to stages")
        old = self.loc[e]
        if old is not None:
            self.pools[old].remove(e)
            self.loc[e] = None
        if not send:
            self.loc[e] = dst
            self.pools[dst].add(e)
            return
        self.moving_to[dst] += 1
        old_job = old[0] if old is not None else None
        _check(old_job != dst[0], "[move_executor_to_pool] send")
        self.supply[dst[0]] += 1
        if old_job is not None:
            self.supply[old_job] -= 1
            _check(self.supply[old_job] >= 0, "[move_executor_to_pool] supply")

    # ---- event queue (event.py:19-49) -------------------------------------------------------------------
    def _push(self, t, kind, payload):
        heapq.heappush(self._pq, (t, next(self._counter), kind, payload))

    # ---- public API -------------------------------------------------------------------------------------
    def reset(self, seed=None, options=None):  # spark_sched_sim.py:127-186
        if seed is not None:
            self.rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        elif self.rng is None:
            self.rng = np.random.Generator(np.random.PCG64())
        options = {} if options is None else options
        limit = options.get("time_limit", np.inf)
        if limit is np.inf and not self.job_arrival_cap:
            raise ValueError("must either have a limit on job arrivals or time.")
        self.wall_time = 0
        self.sampler.rng = self.rng
        self._pq, self._counter = [], itertools.count()
        self.jobs = {}
        seq = self.sampler.job_sequence(limit)
        _check(seq[0][0] == 0, "first job must arrive at t=0")
        for t, job in seq:
            self._push(t, ARRIVAL, job)
            self.jobs[job.jid] = job
        self.job_arrival_cap = len(self.jobs)
        self.executors = [_Executor(e) for e in range(self.N)]
        self._tracker_reset()
        # _reset_edge_links (249-258): global stage index base per job, edges in job order
        self.job_base = {}
        links, base = [], 0
        for jid, job in self.jobs.items():
            self.job_base[jid] = base
            links.extend((base + u, base + v) for u, v in job.edges)
            base += len(job.stages)
        self.all_edges = np.array(links, dtype=np.int64).reshape(-1, 2)
        self.num_total_stages = base
        self.active_ids = []
        self.completed_ids = set()
        self.selected = set()
        self.sel_map = {}
        self.decisions = 0
        # _load_initial_jobs (260-273)
        while self._pq and self._pq[0][0] <= 0:
            _, seq, _, job = heapq.heappop(self._pq)
            self._log(ARRIVAL, -1, job.jid, -1, seq)
            self._on_job_arrival(job)
        self.sched = self._scan()
        return self._observe(), {"wall_time": self.wall_time}

    def step(self, action):  # spark_sched_sim.py:188-221
        self._apply_action(action)
        self.decisions += 1
        if self._committable() and self.sched:
            return self._observe(), 0, False, False, {"wall_time": self.wall_time}
        self._commit_leftovers()
        self._fulfill_from_source()
        self.source = None
        self.selected.clear()
        t0, active0 = self.wall_time, list(self.active_ids)
        self._simulate()
        reward = -self._jobtime(t0, active0)
        done = len(self.completed_ids) == len(self.jobs)
        if not done:
            _check(self._committable() and self.sched, "[step]")
        return self._observe(), reward, done, False, {"wall_time": self.wall_time}

    @property
    def terminated(self):
        return len(self.completed_ids) == len(self.jobs)

    @property
    def avg_job_duration(self):  # spark_sched_sim.py:243-245
        return np.mean(self.duration_buff).item() * 1e-3

    # ---- action (275-315) -------------------------------------------------------------------------------
    def _apply_action(self, action):
        if not _action_in_space(action, self.stage_idx_n, self.N):
            raise ValueError("invalid action: does not belong to the action space")
        if action["stage_idx"] == -1:
            self._commit_leftovers()
            return
        stage = self.sel_map[action["stage_idx"]]  # KeyError beyond the schedulable count
        if stage not in self.sched:
            raise ValueError("invalid action: stage is not currently schedulable")
        n = action["num_exec"]
        if not n:
            raise ValueError("invalid action: must commit at least one executor")
        if n > self._committable():
            raise ValueError("invalid action: too many executors requested")
        n = min(n, self._demand(stage))  # _adjust_num_executors 557-564
        _check(n > 0, "[_adjust_num_executors]")
        self._add_commitment(n, stage.key)
        self.selected.add(stage.key)
        # re-derive this job's schedulable stages and splice them in by job id (bisect, 307-315)
        ids = [s.job for s in self.sched]
        lo = bisect.bisect_left(ids, stage.job)
        hi = min(len(ids), lo + len(self.jobs[stage.job].active))
        end = bisect.bisect_right(ids, stage.job, lo=lo, hi=hi)
        self.sched = self.sched[:lo] + self._scan([stage.job]) + self.sched[end:]

    # ---- simulation loop (320-343) ----------------------------------------------------------------------
    def _simulate(self):
        found = []
        while self._pq:
            t, seq, kind, payload = heapq.heappop(self._pq)
            self.wall_time = t
            if kind == ARRIVAL:
                self._log(ARRIVAL, -1, payload.jid, -1, seq)
                self._on_job_arrival(payload)
            elif kind == EXEC_READY:
                e, st = payload
                self._log(EXEC_READY, e, st.job, st.sid, seq)
                self._on_executor_arrival(e, st)
            else:
                e, st = payload
                self._log(TASK_DONE, e, st.job, st.sid, seq)
                self._on_task_done(e, st)
            if not self._committable():
                continue
            found = self._scan()
            if found:
                break
            self._release_idle()
            self.source = None
        self.sched = found

    def _log(self, *rec):
        if self.trace is not None:
            self.trace.append((self.wall_time,) + rec)

    # ---- handlers (428-483) -----------------------------------------------------------------------------
    def _on_job_arrival(self, job):  # 428-438
        self.active_ids.append(job.jid)
        jp = (job.jid, None)
        if jp in self.pools:
            raise ValueError("job pool already exists")
        self.pools[jp], self.commits[jp], self.commits_from[jp] = set(), {}, 0
        self.supply[job.jid] = 0
        for st in job.stages:  # add_stage_pool 131-143
            k = st.key
            self.pools[k], self.commits[k], self.commits_from[k] = set(), {}, 0
            self.commits_to[k], self.moving_to[k] = 0, 0
        if self.pools[COMMON]:
            self.source = COMMON

    def _on_executor_arrival(self, e, st):  # 440-450
        job = self.jobs[st.job]
        ex = self.executors[e]
        _check(ex.task_stage is None, "[attach_executor]")
        job.local.add(e)
        ex.job = job.jid
        ex.add_history(self.wall_time, job.jid)  # :445
        self.moving_to[st.key] -= 1
        _check(self.moving_to[st.key] >= 0, "[record_executor_arrival]")
        self._move_to_pool(e, (job.jid, None))
        self._goto_stage(ex, st)

    def _on_task_done(self, e, st):  # 452-483
        job = self.jobs[st.job]
        ex = self.executors[e]
        _check(not st.completed, "[_handle_task_completion],2")
        st.executing -= 1
        st.done += 1
        ex.executing = False
        if st.remaining > 0:
            self._run_next_task(ex, st)
            return
        changed = False
        if st.completed:
            changed = self._stage_completed(job, st)
        if not job.active:
            self._job_completed(job)
        had = self._release(ex, st, changed)
        if changed:
            self.source = (st.job, None)
        elif not had:
            self.source = st.key

    # ---- helpers (487-874) ------------------------------------------------------------------------------
    def _commit_leftovers(self):  # 487-503
        n = self._committable()
        if n > 0:
            self._add_commitment(n, COMMON)

    def _scan(self, job_ids=None, source_job=None):  # _find_schedulable_stages 505-540
        if not job_ids:  # quirk Q1: [] behaves like None
            job_ids = self.active_ids
        if not source_job:  # quirk Q2: job 0 behaves like None
            source_job = self._source_job()
        keep = [j for j in job_ids if j == source_job or self.supply[j] < self.N]
        out = []
        for j in keep:
            job = self.jobs[j]
            for sid in job.active:
                st = job.stages[sid]
                if st.key not in self.selected and self._ready(job, st):
                    out.append(st)
        return out

    def _ready(self, job, st):  # 542-555
        if self._demand(st) <= 0:
            return False
        return all(self._demand(job.stages[p]) <= 0 for p in job.parents[st.sid])

    def _demand(self, st):  # 566-578
        return st.remaining - (self.moving_to[st.key] + self.commits_to[st.key])

    def _run_next_task(self, ex, st):  # 584-615
        _check(st.remaining > 0, "[_execute_next_task],1")
        _check(ex.job == st.job, "[_execute_next_task],2")
        _check(not ex.executing, "[_execute_next_task],3")
        job = self.jobs[st.job]
        st.remaining -= 1
        st.executing += 1
        if st.remaining == 0:
            job.saturated_count += 1
        dur = self.sampler.task_duration(job, st, ex)
        ex.task_stage = st.sid
        ex.executing = True
        st.recent = dur
        self._push(self.wall_time + dur, TASK_DONE, (ex.eid, st))

    def _send(self, ex, st):  # 617-637
        _check(not ex.executing, "[_send_executor],2")
        _check(ex.job != st.job, "[_send_executor],3")
        self._move_to_pool(ex.eid, st.key, send=True)
        if ex.job is not None:
            self._detach(ex)
        self._push(self.wall_time + self.moving_delay, EXEC_READY, (ex.eid, st))

    def _detach(self, ex):  # job.py:84-89
        self.jobs[ex.job].local.remove(ex.eid)
        ex.job = None
        ex.task_stage = None

    def _release(self, ex, st, changed):  # _handle_released_executor 639-660
        dst = self._peek_commitment(st.key)
        if dst is not None:
            self._fulfill(ex.eid, dst)
            return True
        ex.task_stage = None
        if changed:
            self._release_idle(st.key, [ex.eid])
        return False

    def _stage_completed(self, job, st):  # job.py:65-73, 113-128
        job.active.remove(st.sid)
        job.frontier.remove(st.sid)
        new = set()
        for c in job.children[st.sid]:
            cs = job.stages[c]
            if not cs.completed and all(job.stages[p].completed for p in job.parents[c]):
                new.add(c)
        job.frontier |= new
        return bool(new)

    def _job_completed(self, job):  # 682-697
        jp = (job.jid, None)
        if len(self.pools[jp]) > 0:
            self._release_idle(jp)
        _check(len(self.pools[jp]) == 0, "[_process_job_completion],2")
        self.active_ids.remove(job.jid)
        self.completed_ids.add(job.jid)
        job.t_completed = self.wall_time
        self.duration_buff.append(job.t_completed - job.t_arrival)
        self._log(JOB_DONE, -1, job.jid, -1, -1)

    def _fulfill(self, e, dst):  # 699-712
        src = self._remove_commitment(e, dst)
        if dst == COMMON:
            self._release_idle(src, [e])
            return
        jid, sid = dst
        self._goto_stage(self.executors[e], self.jobs[jid].stages[sid])

    def _idle_in(self, pool=None):  # 714-728
        members = self.pools[self.source].copy() if not pool else self.pools[pool].copy()
        return set(e for e in members if not self.executors[e].executing)

    def _fulfill_from_source(self):  # 730-743
        idle = self._idle_in()
        plan = self.commits[self.source].copy()
        for dst, n in plan.items():
            _check(dst and n, "[_fulfill_commitments_from_source],1")
            while n and idle:
                self._fulfill(idle.pop(), dst)
                n -= 1
        _check(not idle, "[_fulfill_commitments_from_source],2")

    def _release_idle(self, src=None, eids=None):  # _move_idle_executors 745-782
        if src is None:
            src = self.source
        _check(src is not None, "[_move_idle_executors],1")
        if src == COMMON:
            return
        if eids is None:
            eids = list(self._idle_in(src))
        _check(eids, "[_move_idle_executors],2")
        jid, sid = src
        _check(jid is not None, "[_move_idle_executors],3")
        sat = self.jobs[jid].saturated
        if sid is None and not sat:
            return
        dst = COMMON if sat else (jid, None)
        for e in eids:
            self._move_to_pool(e, dst)
            if dst == COMMON:
                self._detach_from(self.jobs[jid], self.executors[e])
                self.executors[e].add_history(self.wall_time, -1)  # :782
                self._log(TO_COMMON, e, jid, -1, -1)

    def _detach_from(self, job, ex):  # job.py:84-89 via spark_sched_sim.py:779-782
        job.local.remove(ex.eid)
        ex.job = None
        ex.task_stage = None

    def _backup(self, ex):  # _try_backup_schedule 784-797
        st = self._find_backup(ex)
        if st:
            self._goto_stage(ex, st)
            return
        self._release_idle(self.loc[ex.eid], [ex.eid])

    def _goto_stage(self, ex, st):  # _move_executor_to_stage 799-819
        if st.remaining == 0:
            self._backup(ex)
            return
        if ex.job != st.job:
            self._send(ex, st)
            return
        job = self.jobs[st.job]
        if st.sid not in job.frontier:
            ex.task_stage = None
            self._move_to_pool(ex.eid, (st.job, None))
            return
        self._move_to_pool(ex.eid, st.key)
        self._run_next_task(ex, st)

    def _find_backup(self, ex):  # 821-845
        _check(ex.job is not None, "[_find_backup_stage]")
        local = self._scan([ex.job], ex.job)
        if local:
            return local[0]
        others = [j for j in self.active_ids if j != ex.job]
        far = self._scan(others, ex.job)
        return far[0] if far else None

    def _jobtime(self, t0, active0):  # _compute_jobtime 847-874
        span = self.wall_time - t0
        if span == 0.0:
            return 0.0
        total = 0.0
        for jid in set(active0 + self.active_ids):
            job = self.jobs[jid]
            a = max(job.t_arrival, t0)
            b = min(job.t_completed, self.wall_time)
            if self.beta == 0.0:
                total += b - a
            else:
                total += np.exp(-self.beta * 1e-3 * (a - t0)) - np.exp(-self.beta * 1e-3 * (b - t0))
        if self.beta > 0.0:
            total /= self.beta
        return total

    # ---- observation (345-406, utils.py:5-22) -----------------------------------------------------------
    def _observe(self):
        self.sel_map.clear()
        for i, st in enumerate(self.sched):
            self.sel_map[i] = st
            st.flag = True
        rows, ptr, supplies = [], [0], []
        mask = np.zeros(self.num_total_stages, dtype=bool)
        src_job = self._source_job()
        src_idx = len(self.active_ids)
        for i, jid in enumerate(self.active_ids):
            job = self.jobs[jid]
            if jid == src_job:
                src_idx = i
            supplies.append(self.supply[jid])
            for sid in job.active:
                st = job.stages[sid]
                rows.append((st.remaining, st.recent, st.flag))
                st.flag = False
                mask[self.job_base[jid] + sid] = True
            ptr.append(len(rows))
        if rows:
            nodes = np.vstack(rows).astype(np.float32)
        else:
            nodes = np.zeros((0, 3), dtype=np.float32)
        keep = mask[self.all_edges[:, 0]] & mask[self.all_edges[:, 1]]
        relabel = np.zeros(mask.size, dtype=int)
        relabel[mask] = np.arange(mask.sum())
        links = relabel[self.all_edges[keep]]
        obs = {
            "dag_batch": GraphInstance(nodes, np.zeros(len(links), dtype=int), links),
            "dag_ptr": ptr,
            "num_committable_execs": self._committable(),
            "source_job_idx": src_idx,
            "exec_supplies": supplies,
        }
        self.stage_idx_n = len(rows) + 1
        return obs


def _action_in_space(action, stage_n, num_exec):
    """gymnasium 0.29.1 Dict/Discrete.contains for {"stage_idx": Discrete(n, -1), "num_exec": Discrete(N, 1)}."""
    if not isinstance(action, dict) or set(action.keys()) != {"stage_idx", "num_exec"}:
        return False

    def _in(x, start, n):
        if isinstance(x, (bool, int)):
            v = int(x)
        elif isinstance(x, (np.generic, np.ndarray)) and np.issubdtype(x.dtype, np.integer) and x.shape == ():
            v = int(x)
        else:
            return False
        return start <= v < start + n

    return _in(action["stage_idx"], -1, stage_n) and _in(action["num_exec"], 1, num_exec)


# ----------------------------------------------------------------------------------------------------------
# metrics.py
# ----------------------------------------------------------------------------------------------------------

def job_durations(env: SparkSchedOracle):  # metrics.py:4-10
    out = []
    for jid in env.active_ids + list(env.completed_ids):
        job = env.jobs[jid]
        out.append(min(job.t_completed, env.wall_time) - job.t_arrival)
    return out


def avg_job_duration(env):  # metrics.py:13-14
    return np.mean(job_durations(env))


def avg_num_jobs(env):  # metrics.py:17-18
    return sum(job_durations(env)) / env.wall_time
