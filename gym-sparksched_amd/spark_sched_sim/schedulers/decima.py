"""Batched Decima policy in PyTorch-ROCm (PyG-free): the consumer of the device observation tensors.

Restates schedulers/decima/scheduler.py (DecimaScheduler, EncoderNetwork, NodeEncoder, DagEncoder,
GlobalEncoder, StagePolicyNetwork, ExecPolicyNetwork) and the helpers it uses from
schedulers/decima/utils.py (make_mlp, sample, evaluate, collate_*) over ONE flat batch holding the
observations of all B envs of a SparkSchedSimVecEnv at once, so a decision for every env is one forward
pass instead of B Python-level calls:

  * `torch_scatter.segment_csr` -> `index_add_` over the node->DAG and DAG->env maps;
  * `torch_sparse.matmul(adj, msg)` of one message-passing level -> `index_add_` of the child messages
    into their parents (the level's edges come from the device edge-mask bit planes, csrc/decima.h);
  * `pyg.utils.softmax(ptr)` / `random.choices` -> segment softmax + per-env categorical sampling on device.

Launch-bound by design (a decision is ~150 small kernels), so the forward avoids data-dependent shapes:
one host sync per batch for the sizes, no boolean-mask indexing (every level's message pass runs over all
nodes/edges with 0/1 edge weights, stage scores over all nodes with -inf for non-schedulable ones, exec
scores on a dense [envs, N] grid with -inf beyond each DAG's commit cap).

Parameter names match the reference module tree, so a reference `state_dict` loads unchanged.

Semantics kept from the reference, including its two message-passing conventions:
  * `schedule` (one observation per call in the reference): an observation whose DAGs have no edges
    (edge_masks of depth 0) skips message passing (NodeEncoder._forward_no_mp, h = mlp_prep(x));
  * `evaluate_actions` (collated batch in the reference): if any observation of the batch has message-passing
    levels, every observation goes through the message-passing path.
Parity: tests/test_decima_policy.py compares both against the per-observation CPU fp32 restatement
(oracle/decima_gnn.py) on the oracle env's observations, within 1e-5.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any

import torch
import torch.nn as nn

from .. import _abi

from .linear import HipLinear, HipMlp3  # noqa: E402

NUM_NODE_FEATURES = 5  # env_wrapper.py:9
NUM_DAG_FEATURES = 3   # scheduler.py:34
DECIMA_PARAMS = 20802  # parameters of the decima_tpch.yaml architecture (the fused kernel's; csrc/decima_policy.h)


def make_mlp(input_dim: int, hid_dims: list[int], output_dim: int, act_cls: str,
             act_kwargs: dict[str, Any] | None = None) -> nn.Sequential:
    """schedulers/decima/utils.py:51-70."""
    act = getattr(torch.nn.modules.activation, act_cls)
    mlp = HipMlp3()  # an nn.Sequential; on the device the two-hidden-layer shapes run as one fused chain
    prev = input_dim
    dims = list(hid_dims) + [output_dim]
    for i, d in enumerate(dims):
        mlp.append(HipLinear(prev, d))  # nn.Linear; its device passes on csrc/k_linear.hip
        if i == len(dims) - 1:
            break
        mlp.append(act(**(act_kwargs or {})))
        prev = d
    return mlp


@dataclass
class DagBatch:
    """All envs' observations as one flat graph batch (node rows env-major, DAGs and edges contiguous per env)."""
    x: torch.Tensor            # f32 [Nt, 5] Decima node features
    edge_index: torch.Tensor   # i64 [2, Et] (parent, child) in flat node ids, env-major
    edge_bits: torch.Tensor    # i32 [Et]    bit l = edge in DAG-layer mask l
    max_levels: int            # max over envs of (depth - 1): message-passing levels
    env_levels: torch.Tensor   # i64 [B]     per env (depth - 1, >= 0)
    ptr: torch.Tensor          # i64 [Gt+1]  node range per DAG
    node_dag: torch.Tensor     # i64 [Nt]
    node_env: torch.Tensor     # i64 [Nt]
    dag_env: torch.Tensor      # i64 [Gt]
    obs_ptr: torch.Tensor      # i64 [B+1]   DAG range per env
    stage_mask: torch.Tensor   # bool [Nt]   schedulable
    exec_cap: torch.Tensor     # i64 [Gt]    exec_mask[g, :cap] = True
    num_stage_acts: torch.Tensor  # i64 [B]
    num_nodes: torch.Tensor       # i64 [B]
    num_edges: torch.Tensor       # i64 [B]
    num_envs: int
    max_nodes: int = 0            # max over envs of the node count (the fused policy's LDS plan)


def _excl(c: torch.Tensor) -> torch.Tensor:
    return torch.cumsum(c, 0) - c


def _ptr(c: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(c.numel() + 1, dtype=torch.long, device=c.device)
    out[1:] = torch.cumsum(c, 0)
    return out


def _expand(counts: torch.Tensor, total: int):
    """(owner row, index within owner) for `total` items laid out by `counts` (no host sync)."""
    own = torch.repeat_interleave(torch.arange(counts.numel(), device=counts.device), counts, output_size=total)
    return own, torch.arange(total, device=counts.device) - _excl(counts)[own]


def build_batch(views: dict, feats: dict, env_mask: torch.Tensor | None = None,
                envs: torch.Tensor | None = None, sizes: tuple[int, int, int, int, int] | None = None) -> DagBatch:
    """Flat batch from the obs-arena views (DeviceEngine.views) and the device Decima features
    (DeviceEngine.decima_features). `env_mask` (bool [B]) empties envs (e.g. finished ones). `envs` (i64 [K])
    builds the batch of just those envs, renumbered 0..K-1 in the given order: the same batch as
    `select_envs(build_batch(views, feats), envs)` in one pass (one host sync instead of two). `sizes`
    (total nodes, edges, DAGs, max levels, max nodes of the batch), when the caller already has them on the
    host (`live_sizes`), removes the remaining sync."""
    c = views["counts"]
    dev = c.device
    rows = None
    if envs is not None:
        rows = envs.to(dev).long()
        c = c[rows]
    B = c.shape[0]
    n = c[:, _abi.OC_NUM_NODES].long()
    ne = c[:, _abi.OC_NUM_EDGES].long()
    nj = c[:, _abi.OC_NUM_JOBS].long()
    if env_mask is not None:
        keep = env_mask.to(dev).long()
        if rows is not None:
            keep = keep[rows]
        n, ne, nj = n * keep, ne * keep, nj * keep
    depth = feats["depth"] if rows is None else feats["depth"][rows]
    levels = torch.clamp(depth.long() - 1, min=0) * (n > 0)
    if sizes is not None:
        Nt, Et, Gt, L, Nmax = sizes
    elif B == 0:
        Nt = Et = Gt = L = Nmax = 0
    else:
        Nt, Et, Gt, L, Nmax = (int(v) for v in torch.stack([n.sum(), ne.sum(), nj.sum(), levels.max(),
                                                             n.max()]).tolist())
    glob = (lambda e: e) if rows is None else (lambda e: rows[e])  # local env row -> arena row
    node_env, nl = _expand(n, Nt)
    node_base = _excl(n)
    node_src = glob(node_env)
    x = feats["node_feats"][node_src, nl]
    stage_mask = views["nodes"][node_src, nl, 2] != 0
    edge_env, el = _expand(ne, Et)
    edge_src = glob(edge_env)
    links = views["edge_links"][edge_src, el]
    edge_index = (links + node_base[edge_env][:, None]).t().contiguous()
    edge_bits = feats["edge_mask"][edge_src, el]
    dag_env, dl = _expand(nj, Gt)
    dag_src = glob(dag_env)
    dag_ptr = views["dag_ptr"].long()
    dag_counts = dag_ptr[dag_src, dl + 1] - dag_ptr[dag_src, dl]
    node_dag, _ = _expand(dag_counts, Nt)
    num_stage_acts = torch.zeros(B, dtype=torch.long, device=dev).index_add_(0, node_env, stage_mask.long())
    return DagBatch(x=x, edge_index=edge_index, edge_bits=edge_bits, max_levels=L, env_levels=levels,
                    ptr=_ptr(dag_counts), node_dag=node_dag, node_env=node_env, dag_env=dag_env, obs_ptr=_ptr(nj),
                    stage_mask=stage_mask, exec_cap=feats["commit_cap"][dag_src, dl].long(),
                    num_stage_acts=num_stage_acts, num_nodes=n, num_edges=ne, num_envs=B, max_nodes=Nmax)


def live_sizes(views: dict, feats: dict, alive: torch.Tensor):
    """One host sync for a rollout step: the live env ids (device i64, ascending, via nonzero_static) and the
    `sizes` tuple build_batch(views, feats, envs=ids) needs. Returns (ids, sizes) with ids empty if none."""
    c = views["counts"]
    st = torch.stack([alive.to(c.device).long(), c[:, _abi.OC_NUM_NODES].long(), c[:, _abi.OC_NUM_EDGES].long(),
                      c[:, _abi.OC_NUM_JOBS].long(), feats["depth"].long()]).cpu()
    live = st[0] != 0
    k = int(live.sum())
    ids = torch.nonzero_static(alive.to(c.device), size=k).squeeze(1)
    if k == 0:
        return ids, (0, 0, 0, 0, 0)
    n, ne, nj, d = st[1][live], st[2][live], st[3][live], st[4][live]
    levels = torch.clamp(d - 1, min=0) * (n > 0)
    return ids, (int(n.sum()), int(ne.sum()), int(nj.sum()), int(levels.max()), int(n.max()))


def select_envs(b: DagBatch, envs: torch.Tensor, sizes: tuple[int, int, int, int, int] | None = None) -> DagBatch:
    """Sub-batch of the observations `envs` (i64 indices into b's env rows, any order), renumbered 0..K-1
    in the given order (the rollout buffer keeps alive envs' observations this way). `sizes` (total nodes, edges,
    DAGs, max levels, max nodes of the sub-batch; minibatch_plans) removes the host sync for them."""
    dev = b.x.device
    envs = envs.to(dev).long()
    K = envs.numel()
    n, ne = b.num_nodes[envs], b.num_edges[envs]
    nd = (b.obs_ptr[1:] - b.obs_ptr[:-1])[envs]
    lv = b.env_levels[envs]
    if sizes is not None:
        Nt, Et, Gt, L, Nmax = sizes
    elif K == 0:
        Nt = Et = Gt = L = Nmax = 0
    else:
        Nt, Et, Gt, L, Nmax = (int(v) for v in torch.stack([n.sum(), ne.sum(), nd.sum(), lv.max(),
                                                             n.max()]).tolist())
    node_base_old, edge_base_old = _excl(b.num_nodes), _excl(b.num_edges)
    node_env, nl = _expand(n, Nt)
    src_node = node_base_old[envs][node_env] + nl
    edge_env, el = _expand(ne, Et)
    src_edge = edge_base_old[envs][edge_env] + el
    shift = (_excl(n) - node_base_old[envs])[edge_env]
    dag_env, dl = _expand(nd, Gt)
    src_dag = b.obs_ptr[envs][dag_env] + dl
    dag_shift = (_excl(nd) - b.obs_ptr[envs])[node_env]
    dag_counts = (b.ptr[1:] - b.ptr[:-1])[src_dag]
    return DagBatch(x=b.x[src_node], edge_index=b.edge_index[:, src_edge] + shift[None, :],
                    edge_bits=b.edge_bits[src_edge], max_levels=L, env_levels=lv, ptr=_ptr(dag_counts),
                    node_dag=b.node_dag[src_node] + dag_shift, node_env=node_env, dag_env=dag_env, obs_ptr=_ptr(nd),
                    stage_mask=b.stage_mask[src_node], exec_cap=b.exec_cap[src_dag],
                    num_stage_acts=b.num_stage_acts[envs], num_nodes=n, num_edges=ne, num_envs=K,
                    max_nodes=Nmax)


def learner_counts(b: DagBatch) -> torch.Tensor:
    """Per observation of b, the sizes of the compact learner path's index sets (NodeEncoder / scores_all with a
    plan): i64 [B, 2 + 2L] = leaves, schedulable rows, then per message-passing level l < b.max_levels the level's
    edges and its distinct parents. A sub-batch's sizes are sums over its observations, so the sizes of every
    minibatch of an epoch come from one host sync (minibatch_plans) instead of one per index set."""
    dev = b.x.device
    Nt, B, L = b.x.shape[0], b.num_envs, b.max_levels
    parent = b.edge_index[0]
    has_child = torch.zeros(Nt, dtype=torch.long, device=dev).index_add_(
        0, parent, torch.ones_like(parent)) > 0
    cols = [segment_sum((~has_child).long(), b.node_env, B), segment_sum(b.stage_mask.long(), b.node_env, B)]
    edge_env = b.node_env[parent] if parent.numel() else parent
    for lvl in range(L):
        on = ((b.edge_bits >> lvl) & 1).long()
        cols.append(segment_sum(on, edge_env, B))
        dst = torch.zeros(Nt, dtype=torch.long, device=dev).index_add_(0, parent, on) > 0
        cols.append(segment_sum(dst.long(), b.node_env, B))
    return torch.stack(cols, dim=1)


@dataclass
class LearnerPlan:
    """Host sizes of one sub-batch's compact index sets (see learner_counts)."""
    leaves: int
    sched: int
    edges: list[int]
    dsts: list[int]


def minibatch_plans(b: DagBatch, counts: torch.Tensor, groups: list[torch.Tensor]):
    """For each env-index group (a minibatch of b's observations): the select_envs `sizes` and the LearnerPlan of
    the sub-batch, all in ONE host sync. Returns [(sizes, plan)] in group order."""
    dev = b.x.device
    if not groups:
        return []
    nd = b.obs_ptr[1:] - b.obs_ptr[:-1]
    per_env = torch.cat([torch.stack([b.num_nodes, b.num_edges, nd], dim=1), counts], dim=1)  # summed columns
    gid = torch.cat([torch.full((g.numel(),), k, dtype=torch.long, device=dev) for k, g in enumerate(groups)])
    rows = torch.cat([g.to(dev).long() for g in groups])
    G = len(groups)
    sums = torch.zeros((G, per_env.shape[1]), dtype=torch.long, device=dev).index_add_(0, gid, per_env[rows])
    mx = torch.zeros((G, 2), dtype=torch.long, device=dev).scatter_reduce_(
        0, gid[:, None].expand(-1, 2), torch.stack([b.env_levels[rows], b.num_nodes[rows]], dim=1), reduce="amax",
        include_self=True)
    host = torch.cat([sums, mx], dim=1).cpu().tolist()
    out = []
    L = counts.shape[1] // 2 - 1
    for r in host:
        Nt, Et, Gt = r[0], r[1], r[2]
        c = r[3:3 + counts.shape[1]]
        Lg, Nmax = r[-2], r[-1]
        plan = LearnerPlan(leaves=c[0], sched=c[1], edges=[c[2 + 2 * l] for l in range(L)],
                           dsts=[c[3 + 2 * l] for l in range(L)])
        out.append(((Nt, Et, Gt, Lg, Nmax), plan))
    return out


def cat_batches(bs: list[DagBatch]) -> DagBatch:
    """Concatenation of batches (observations in list order). Index fields are shifted by per-element
    offsets expanded with repeat_interleave, so the cost is a fixed number of launches per field rather than
    one per batch (a rollout buffer holds thousands of per-step batches)."""
    dev = bs[0].x.device
    i64 = dict(dtype=torch.long, device=dev)
    nN = [b.x.shape[0] for b in bs]
    nE = [b.edge_index.shape[1] for b in bs]
    nG = [b.ptr.numel() - 1 for b in bs]
    nB = [b.num_envs for b in bs]

    def offsets(counts):  # exclusive prefix sums (host)
        out, t = [], 0
        for c in counts:
            out.append(t)
            t += c
        return torch.tensor(out, **i64), t

    n_off, Nt = offsets(nN)
    g_off, Gt = offsets(nG)
    e_off, Bt = offsets(nB)
    Et = sum(nE)

    def per_item(off, counts, total):  # offset of each element's batch
        return torch.repeat_interleave(off, torch.tensor(counts, **i64), output_size=total)

    zero = torch.zeros(1, **i64)
    return DagBatch(
        x=torch.cat([b.x for b in bs]),
        edge_index=torch.cat([b.edge_index for b in bs], dim=1) + per_item(n_off, nE, Et)[None, :],
        edge_bits=torch.cat([b.edge_bits for b in bs]),
        max_levels=max(b.max_levels for b in bs), env_levels=torch.cat([b.env_levels for b in bs]),
        ptr=torch.cat([bs[0].ptr[:1]] + [b.ptr[1:] for b in bs]) + torch.cat([zero, per_item(n_off, nG, Gt)]),
        node_dag=torch.cat([b.node_dag for b in bs]) + per_item(g_off, nN, Nt),
        node_env=torch.cat([b.node_env for b in bs]) + per_item(e_off, nN, Nt),
        dag_env=torch.cat([b.dag_env for b in bs]) + per_item(e_off, nG, Gt),
        obs_ptr=torch.cat([bs[0].obs_ptr[:1]] + [b.obs_ptr[1:] for b in bs]) + torch.cat([zero, per_item(g_off, nB, Bt)]),
        stage_mask=torch.cat([b.stage_mask for b in bs]), exec_cap=torch.cat([b.exec_cap for b in bs]),
        num_stage_acts=torch.cat([b.num_stage_acts for b in bs]), num_nodes=torch.cat([b.num_nodes for b in bs]),
        num_edges=torch.cat([b.num_edges for b in bs]), num_envs=int(Bt),
        max_nodes=max(b.max_nodes for b in bs))


def segment_sum(src: torch.Tensor, index: torch.Tensor, size: int) -> torch.Tensor:
    out = torch.zeros((size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    return out.index_add_(0, index, src)


def segment_max(src: torch.Tensor, index: torch.Tensor, size: int) -> torch.Tensor:
    """Per-segment max of a detached score vector; empty / all -inf segments give 0 (safe shift)."""
    mx = torch.full((size,), -torch.inf, dtype=src.dtype, device=src.device)
    mx = mx.scatter_reduce(0, index, src.detach(), reduce="amax", include_self=True)
    return torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))


def masked_softmax_stats(scores: torch.Tensor, mask: torch.Tensor, seg: torch.Tensor, nseg: int, clamp: bool):
    """pyg.utils.softmax over the masked rows of each segment (utils.py:37): probs (0 off-mask) and log-probs
    (-inf off-mask). `clamp` applies torch.distributions clamp_probs (utils.py:38) as evaluate() does."""
    mx = segment_max(torch.where(mask, scores, torch.full_like(scores, -torch.inf)), seg, nseg)
    z = torch.where(mask, scores - mx[seg], torch.zeros_like(scores))
    ex = torch.where(mask, torch.exp(z), torch.zeros_like(z))
    probs = ex / (segment_sum(ex, seg, nseg) + 1e-16)[seg]
    if clamp:
        eps = torch.finfo(probs.dtype).eps
        probs = probs.clamp(min=eps, max=1 - eps)
    logp = torch.where(mask, torch.log(torch.where(mask, probs, torch.ones_like(probs))),
                       torch.full_like(probs, -torch.inf))
    return torch.where(mask, probs, torch.zeros_like(probs)), logp


def _i64(c: int) -> int:  # a 64-bit constant as the signed value torch int64 arithmetic wraps around
    return c - (1 << 64) if c >= (1 << 63) else c


def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:  # logical shift right of int64 bit patterns
    return (x >> s) & ((1 << (64 - s)) - 1)


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 (the device policies' counter-based stream, csrc/policy.h) on int64 tensors; torch integer
    arithmetic wraps modulo 2^64 like the uint64 original."""
    x = x + _i64(0x9E3779B97F4A7C15)
    x = (x ^ _lsr(x, 30)) * _i64(0xBF58476D1CE4E5B9)
    x = (x ^ _lsr(x, 27)) * _i64(0x94D049BB133111EB)
    return x ^ _lsr(x, 31)


def counter_uniform(seed: int, counter: int, env: torch.Tensor, idx: torch.Tensor, channel: int) -> torch.Tensor:
    """Uniform (0, 1) float64 per element from a counter-based hash of (seed, decision counter, global env id,
    element index, channel): the draw of an env's element depends on nothing else, so a row samples the same
    actions whichever rank / batch position holds it (the multi-rank PPO learner relies on this)."""
    key = _mix64(env.long() * _i64(0xD1B54A32D192ED03) + _i64(counter & ((1 << 64) - 1)))
    key = _mix64(key ^ _i64(seed & ((1 << 64) - 1)) ^ _mix64(idx.long() * 2 + channel))
    return (_lsr(key, 11).double() + 0.5) * (1.0 / (1 << 53))


def gumbel_pick(logp: torch.Tensor, seg: torch.Tensor, nseg: int, generator=None,
                u: torch.Tensor | None = None) -> torch.Tensor:
    """One categorical draw per segment from log-probabilities (-inf = excluded): Gumbel-max; returns the flat
    row index per segment (-1 for segments without a candidate). `u`: the uniforms (default: torch.rand with
    `generator`)."""
    if u is None:
        u = torch.rand(logp.shape, dtype=torch.float64, device=logp.device, generator=generator)
    g = logp.double() - torch.log(-torch.log(u.clamp_min(1e-300)))
    best = torch.full((nseg,), -torch.inf, dtype=torch.float64, device=logp.device)
    best = best.scatter_reduce(0, seg, g, reduce="amax", include_self=True)
    rows = torch.arange(logp.numel(), device=logp.device)
    cand = torch.where((g == best[seg]) & torch.isfinite(g), rows, torch.full_like(rows, -1))
    out = torch.full((nseg,), -1, dtype=torch.long, device=logp.device)
    return out.scatter_reduce(0, seg, cand, reduce="amax", include_self=True)


class NodeEncoder(nn.Module):
    """scheduler.py:176-245 (reverse flow: children send to parents, deepest level first). Each level runs
    mlp_msg on every node and sums child messages into parents with the level's 0/1 edge weights: the same
    sums as the reference's masked sparse matmul, without data-dependent shapes."""

    force_dense = False  # the learner's encoder in the dense form too (tests, scripts/profile_learner.py)

    def __init__(self, num_node_features: int, embed_dim: int, mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp_prep = make_mlp(num_node_features, output_dim=embed_dim, **mlp_kwargs)
        self.mlp_msg = make_mlp(embed_dim, output_dim=embed_dim, **mlp_kwargs)
        self.mlp_update = make_mlp(embed_dim, output_dim=embed_dim, **mlp_kwargs)

    def forward(self, b: DagBatch, per_obs_no_mp: bool, plan: LearnerPlan | None = None) -> torch.Tensor:
        h_init = self.mlp_prep(b.x)
        if b.max_levels == 0:
            return h_init  # _forward_no_mp for every observation
        Nt = h_init.shape[0]
        parent, child = b.edge_index[0], b.edge_index[1]
        ones = torch.ones(parent.numel(), dtype=h_init.dtype, device=h_init.device)
        has_child = torch.zeros(Nt, dtype=h_init.dtype, device=h_init.device).index_add_(0, parent, ones) > 0
        if per_obs_no_mp or self.force_dense:  # schedule (rollouts): the dense form, whose per-row results do not
            return self._dense(b, h_init, has_child, parent, child, per_obs_no_mp)  # depend on the rest of the batch
        # evaluate_actions (the learner): the MLPs run on the rows that need them only (leaves; per level its edges'
        # children and its parents). A learner batch of J=200 observations holds millions of node rows and up to ~18
        # levels, and an MLP over every row at every level was most of the learner's time. Same values as the dense
        # form up to the GEMM shapes (the reference's masked sparse matmul sums the level's child messages into their
        # parents); rollouts keep the dense form so a row's actions and log-probs do not depend on which other rows
        # share its batch (the multi-rank learner's bit-equality with one rank).
        # With a plan (the PPO learner's minibatches) the index sets' sizes are known on the host, so the sets come
        # from nonzero_static and the forward issues no host sync.
        if plan is not None:
            leaves = torch.nonzero_static(~has_child, size=plan.leaves).squeeze(1)
        else:
            leaves = torch.nonzero(~has_child).squeeze(1)
        h = torch.zeros_like(h_init).index_put((leaves,), self.mlp_update(h_init[leaves]))
        for lvl in range(b.max_levels - 1, -1, -1):
            on = (b.edge_bits >> lvl) & 1
            if plan is not None:
                if plan.edges[lvl] == 0:
                    continue
                eidx = torch.nonzero_static(on, size=plan.edges[lvl]).squeeze(1)
            else:
                eidx = torch.nonzero(on).squeeze(1)
                if eidx.numel() == 0:
                    continue
            p, c = parent[eidx], child[eidx]
            agg = torch.zeros_like(h).index_add_(0, p, self.mlp_msg(h[c]))
            if plan is not None:  # the level's distinct parents, ascending (= torch.unique)
                hit = torch.zeros(Nt, dtype=torch.long, device=p.device).index_add_(0, p, torch.ones_like(p)) > 0
                dst = torch.nonzero_static(hit, size=plan.dsts[lvl]).squeeze(1)
            else:
                dst = torch.unique(p)
            h = h.index_put((dst,), h_init[dst] + self.mlp_update(agg[dst]))
        return h

    def _dense(self, b: DagBatch, h_init, has_child, parent, child, per_obs_no_mp: bool = True) -> torch.Tensor:
        Nt = h_init.shape[0]
        h = torch.where(has_child[:, None], torch.zeros_like(h_init), self.mlp_update(h_init))
        for lvl in range(b.max_levels - 1, -1, -1):
            w = ((b.edge_bits >> lvl) & 1).to(h.dtype)
            msg = self.mlp_msg(h)
            agg = torch.zeros_like(h).index_add_(0, parent, msg[child] * w[:, None])
            dst = torch.zeros(Nt, dtype=h.dtype, device=h.device).index_add_(0, parent, w) > 0
            h = torch.where(dst[:, None], h_init + self.mlp_update(agg), h)
        if not per_obs_no_mp:
            return h
        # schedule's convention: observations without message-passing levels keep h = mlp_prep(x)
        flat = (b.env_levels == 0)[b.node_env]
        return torch.where(flat[:, None], h_init, h)


class DagEncoder(nn.Module):
    """scheduler.py:248-262."""

    def __init__(self, num_node_features: int, embed_dim: int, mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp = make_mlp(num_node_features + embed_dim, output_dim=embed_dim, **mlp_kwargs)

    def forward(self, h_node: torch.Tensor, b: DagBatch) -> torch.Tensor:
        return segment_sum(self.mlp(torch.cat([b.x, h_node], dim=1)), b.node_dag, b.ptr.numel() - 1)


class GlobalEncoder(nn.Module):
    """scheduler.py:265-281."""

    def __init__(self, embed_dim: int, mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp = make_mlp(embed_dim, output_dim=embed_dim, **mlp_kwargs)

    def forward(self, h_dag: torch.Tensor, b: DagBatch) -> torch.Tensor:
        return segment_sum(self.mlp(h_dag), b.dag_env, b.num_envs)


class EncoderNetwork(nn.Module):
    """scheduler.py:148-173."""

    def __init__(self, num_node_features: int, embed_dim: int, mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.node_encoder = NodeEncoder(num_node_features, embed_dim, mlp_kwargs)
        self.dag_encoder = DagEncoder(num_node_features, embed_dim, mlp_kwargs)
        self.global_encoder = GlobalEncoder(embed_dim, mlp_kwargs)

    def forward(self, b: DagBatch, per_obs_no_mp: bool, plan: LearnerPlan | None = None) -> dict[str, torch.Tensor]:
        h_node = self.node_encoder(b, per_obs_no_mp, plan)
        h_dag = self.dag_encoder(h_node, b)
        return {"node": h_node, "dag": h_dag, "glob": self.global_encoder(h_dag, b)}


class StagePolicyNetwork(nn.Module):
    """scheduler.py:284-326."""

    def __init__(self, num_node_features: int, emb_dims: dict[str, int], mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp_score = make_mlp(num_node_features + emb_dims["node"] + emb_dims["dag"] + emb_dims["glob"],
                                  output_dim=1, **mlp_kwargs)

    def scores_all(self, b: DagBatch, h: dict[str, torch.Tensor], compact: bool = False,
                   plan: LearnerPlan | None = None) -> torch.Tensor:
        """Score of every node row (only schedulable rows are meaningful). compact (the learner): the MLP runs on the
        schedulable rows only, the others are 0 (their count from `plan` when given: no host sync)."""
        if not compact:
            inp = torch.cat([b.x, h["node"], h["dag"][b.node_dag], h["glob"][b.node_env]], dim=1)
            return self.mlp_score(inp).squeeze(-1)
        if plan is not None:
            idx = torch.nonzero_static(b.stage_mask, size=plan.sched).squeeze(1)
        else:
            idx = torch.nonzero(b.stage_mask).squeeze(1)
        inp = torch.cat([b.x[idx], h["node"][idx], h["dag"][b.node_dag[idx]], h["glob"][b.node_env[idx]]], dim=1)
        out = torch.zeros(b.x.shape[0], dtype=h["node"].dtype, device=b.x.device)
        return out.index_put((idx,), self.mlp_score(inp).squeeze(-1))

    def forward(self, b: DagBatch, h: dict[str, torch.Tensor]) -> torch.Tensor:
        """The reference's output: one score per schedulable node, in flat node order."""
        return self.scores_all(b, h)[b.stage_mask]


class ExecPolicyNetwork(nn.Module):
    """scheduler.py:329-385."""

    def __init__(self, num_executors: int, num_dag_features: int, emb_dims: dict[str, int],
                 mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.num_executors = num_executors
        self.num_dag_features = num_dag_features
        self.mlp_score = make_mlp(num_dag_features + emb_dims["dag"] + emb_dims["glob"] + 1, output_dim=1,
                                  **mlp_kwargs)

    def scores_grid(self, b: DagBatch, h: dict[str, torch.Tensor], dags: torch.Tensor, envs: torch.Tensor):
        """Scores of exec actions k/N for k < N, per decision (chosen DAG `dags`, its env `envs`): [K, N],
        and the validity mask k < commit cap of the DAG (the reference's exec_mask row)."""
        N = self.num_executors
        K = dags.numel()
        x_dag = b.x[b.ptr[dags], : self.num_dag_features]
        base = torch.cat([x_dag, h["dag"][dags], h["glob"][envs]], dim=1)
        scores = self.mlp_score.grid(base, N).view(K, N)  # input row (k, a) = [base[k], a / N]
        valid = torch.arange(N, device=dags.device)[None, :] < b.exec_cap[dags][:, None]
        return scores, valid

    def forward(self, b: DagBatch, h: dict[str, torch.Tensor], dags: torch.Tensor, envs: torch.Tensor):
        """The reference's output for the given decisions: scores of the valid actions (flat), their
        decision index and action k."""
        scores, valid = self.scores_grid(b, h, dags, envs)
        K, N = scores.shape
        seg = torch.arange(K, device=dags.device)[:, None].expand(K, N)
        k = torch.arange(N, device=dags.device)[None, :].expand(K, N)
        return scores[valid], seg[valid], k[valid]


class DecimaScheduler(nn.Module):
    """DecimaScheduler (scheduler.py:16-145) over all envs of a vector env at once."""

    def __init__(self, num_executors: int, embed_dim: int = 16, gnn_mlp_kwargs: dict | None = None,
                 policy_mlp_kwargs: dict | None = None, num_node_features: int = NUM_NODE_FEATURES,
                 num_dag_features: int = NUM_DAG_FEATURES, opt_cls: str | None = None, opt_kwargs: dict | None = None,
                 max_grad_norm: float | None = None, **kwargs):
        super().__init__()
        gnn_mlp_kwargs = gnn_mlp_kwargs or {"hid_dims": [32, 16], "act_cls": "LeakyReLU",
                                            "act_kwargs": {"inplace": True, "negative_slope": 0.2}}
        policy_mlp_kwargs = policy_mlp_kwargs or {"hid_dims": [64, 64], "act_cls": "Tanh"}
        self.name = "Decima"
        self.num_executors = num_executors
        self.max_grad_norm = max_grad_norm
        self.encoder = EncoderNetwork(num_node_features, embed_dim, gnn_mlp_kwargs)
        emb = {"node": embed_dim, "dag": embed_dim, "glob": embed_dim}
        self.stage_policy_network = StagePolicyNetwork(num_node_features, emb, policy_mlp_kwargs)
        self.exec_policy_network = ExecPolicyNetwork(num_executors, num_dag_features, emb, policy_mlp_kwargs)
        for name, p in self.named_parameters():  # _reset_biases (scheduler.py:65-68)
            if "bias" in name:
                p.data.zero_()
        self.optim = getattr(torch.optim, opt_cls)(self.parameters(), **(opt_kwargs or {})) if opt_cls else None

    @property
    def device(self):
        return next(self.parameters()).device

    def _sched_rows(self, b: DagBatch):
        """Per node: rank among its env's schedulable nodes (valid where stage_mask)."""
        return torch.cumsum(b.stage_mask.long(), 0) - 1 - _excl(b.num_stage_acts)[b.node_env]

    @torch.no_grad()
    def schedule(self, b: DagBatch, generator=None, stream: tuple | None = None) -> dict[str, torch.Tensor]:
        """One decision per env (envs with no schedulable stage get stage_idx -1, num_exec 1). Returns device
        tensors: stage_idx i32 [B] (index among the env's schedulable stages), num_exec i32 [B] (already
        1 + the sampled exec action, DecimaActWrapper.action), job_idx i64 [B] (DAG index within the env),
        exec_idx i64 [B], lgprob f32 [B] (utils.sample: log of the softmax probability, stage + exec).
        `stream` = (seed, counter, global env ids i64 [B]) draws the Gumbel noise from counter_uniform
        instead of `generator` (rank-independent sampling)."""
        B = b.num_envs
        dev = b.x.device
        h = self.encoder(b, per_obs_no_mp=True)
        scores = self.stage_policy_network.scores_all(b, h)
        _, logp = masked_softmax_stats(scores, b.stage_mask, b.node_env, B, clamp=False)
        u_stage = u_exec = None
        if stream is not None:
            seed, counter, env_ids = stream
            env_ids = env_ids.to(dev).long()
            local = torch.arange(b.x.shape[0], device=dev) - _excl(b.num_nodes)[b.node_env]
            u_stage = counter_uniform(seed, counter, env_ids[b.node_env], local, 0)
            N = self.num_executors
            u_exec = counter_uniform(seed, counter, env_ids[:, None].expand(B, N).reshape(-1),
                                     torch.arange(N, device=dev).repeat(B), 1)
        pick = gumbel_pick(logp, b.node_env, B, generator, u=u_stage)  # flat node row per env
        live = pick >= 0
        row = pick.clamp(min=0)
        stage_idx = torch.where(live, self._sched_rows(b)[row] if row.numel() and b.x.shape[0] else pick, -1)
        envs = torch.arange(B, device=dev)
        dags = b.node_dag[row] if b.x.shape[0] else torch.zeros(B, dtype=torch.long, device=dev)
        es, valid = self.exec_policy_network.scores_grid(b, h, dags, envs)
        elogp = torch.log_softmax(torch.where(valid, es, torch.full_like(es, -torch.inf)), dim=1)
        elogp = torch.where(valid, elogp, torch.full_like(elogp, -torch.inf))
        N = self.num_executors
        seg = torch.arange(B, device=dev)[:, None].expand(B, N).reshape(-1)
        epick = gumbel_pick(elogp.reshape(-1), seg, B, generator, u=u_exec)
        ok = live & (epick >= 0)
        exec_idx = torch.where(ok, epick - envs * N, torch.zeros_like(epick))
        lg_stage = torch.where(live, logp[row] if b.x.shape[0] else torch.zeros(B, device=dev),
                               torch.zeros(B, device=dev))
        lg_exec = torch.where(ok, elogp.reshape(-1)[epick.clamp(min=0)], torch.zeros(B, device=dev))
        return {"stage_idx": stage_idx.to(torch.int32), "num_exec": (exec_idx + 1).to(torch.int32),
                "job_idx": torch.where(live, dags - b.obs_ptr[:-1], torch.full_like(dags, -1)),
                "exec_idx": exec_idx, "lgprob": (lg_stage + lg_exec).float()}

    @torch.no_grad()
    def packed_params(self, dev) -> torch.Tensor:
        """fp32 parameters in parameters() order (nn.Linear [out][in] weights) for ssim_decima_policy /
        ssim_decima_rollout, as one contiguous device buffer."""
        return torch.cat([p.detach().reshape(-1).float() for p in self.parameters()]).to(dev).contiguous()

    @torch.no_grad()
    def schedule_fused(self, engine, feats: dict | None = None, seed: int = 0, counter: int = 0,
                       env_mask: torch.Tensor | None = None, node_cap: int | None = None,
                       with_scores: bool = False, params: torch.Tensor | None = None) -> dict[str, torch.Tensor]:
        """`schedule` for every env of a DeviceEngine in ONE kernel launch (ssim_decima_policy,
        csrc/decima_policy.h): the same forward over the obs arena and the device features, weights read
        from a packed copy of this module's parameters, sampling on a counter-based device stream of
        (seed, env, counter). Only the decima_tpch.yaml architecture (20802 parameters). Returns the same keys
        as `schedule` (int32/float32 device tensors); with_scores adds per-env stage scores [B, stage_cap]
        and exec scores [B, N]."""
        from .. import native

        eng = engine
        L = eng.layout
        B = eng.num_envs
        dev = eng.device
        if feats is None:
            feats = eng.decima_features()
        if params is None:  # callers stepping many decisions with fixed weights pass packed_params() once
            params = self.packed_params(dev)
        if node_cap is None:
            node_cap = int(eng.views["counts"][:, _abi.OC_NUM_NODES].max().item())
        i32 = dict(dtype=torch.int32, device=dev)
        out = {"stage_idx": torch.empty(B, **i32), "num_exec": torch.empty(B, **i32),
               "job_idx": torch.empty(B, **i32), "exec_idx": torch.empty(B, **i32),
               "lgprob": torch.empty(B, dtype=torch.float32, device=dev)}
        ss = es = None
        if with_scores:
            ss = torch.full((B, L.stage_cap), float("nan"), dtype=torch.float32, device=dev)
            es = torch.full((B, L.num_executors), float("nan"), dtype=torch.float32, device=dev)
        overflow = torch.zeros(1, **i32)
        m = None if env_mask is None else env_mask.to(device=dev, dtype=torch.uint8).contiguous()
        native.check(native.lib().ssim_decima_policy(
            eng.handle, feats["node_feats"].data_ptr(), feats["commit_cap"].data_ptr(), feats["edge_mask"].data_ptr(),
            feats["depth"].data_ptr(), params.data_ptr(), params.numel(), max(node_cap, 1), seed, counter,
            None if m is None else m.data_ptr(), out["stage_idx"].data_ptr(), out["num_exec"].data_ptr(),
            out["job_idx"].data_ptr(), out["exec_idx"].data_ptr(), out["lgprob"].data_ptr(),
            None if ss is None else ss.data_ptr(), None if es is None else es.data_ptr(), overflow.data_ptr(),
            eng._stream()), "ssim_decima_policy")
        self._keep = (params, m)
        out["overflow"] = overflow
        if with_scores:
            out["stage_scores"], out["exec_scores"] = ss, es
        return out

    def evaluate_actions(self, b: DagBatch, stage_idx: torch.Tensor, job_idx: torch.Tensor,
                         exec_idx: torch.Tensor, plan: LearnerPlan | None = None) -> dict[str, torch.Tensor]:
        """scheduler.py:103-145 over a batch of observations (one per env row of `b`), with grads:
        log-probabilities and normalised entropies of the given actions (utils.py:25-48, clamp_probs). `plan`
        (minibatch_plans): the compact path's index-set sizes, so the forward issues no host sync."""
        B = b.num_envs
        dev = b.x.device
        h = self.encoder(b, per_obs_no_mp=False, plan=plan)
        scores = self.stage_policy_network.scores_all(b, h, compact=True, plan=plan)
        probs, logp = masked_softmax_stats(scores, b.stage_mask, b.node_env, B, clamp=True)
        rows = torch.arange(b.x.shape[0], device=dev)
        hit = b.stage_mask & (self._sched_rows(b) == stage_idx.long()[b.node_env])
        sel = torch.full((B,), -1, dtype=torch.long, device=dev).scatter_reduce(
            0, b.node_env, torch.where(hit, rows, torch.full_like(rows, -1)), reduce="amax", include_self=True)
        s_lp = logp[sel.clamp(min=0)]
        s_ent = -segment_sum(torch.where(b.stage_mask, logp * probs, torch.zeros_like(probs)), b.node_env, B)
        envs = torch.arange(B, device=dev)
        dags = job_idx.long() + b.obs_ptr[:-1]
        es, valid = self.exec_policy_network.scores_grid(b, h, dags, envs)
        N = self.num_executors
        seg = envs[:, None].expand(B, N).reshape(-1)
        ep, elp = masked_softmax_stats(es.reshape(-1), valid.reshape(-1), seg, B, clamp=True)
        e_lp = elp[envs * N + exec_idx.long()]
        e_ent = -segment_sum(torch.where(valid.reshape(-1), elp * ep, torch.zeros_like(ep)), seg, B)
        ent = (s_ent + e_ent) / (self.num_executors * b.num_nodes).float().log()
        return {"lgprobs": s_lp + e_lp, "entropies": ent}
