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

NUM_NODE_FEATURES = 5  # env_wrapper.py:9
NUM_DAG_FEATURES = 3   # scheduler.py:34


def make_mlp(input_dim: int, hid_dims: list[int], output_dim: int, act_cls: str,
             act_kwargs: dict[str, Any] | None = None) -> nn.Sequential:
    """schedulers/decima/utils.py:51-70."""
    act = getattr(torch.nn.modules.activation, act_cls)
    mlp = nn.Sequential()
    prev = input_dim
    dims = list(hid_dims) + [output_dim]
    for i, d in enumerate(dims):
        mlp.append(nn.Linear(prev, d))
        if i == len(dims) - 1:
            break
        mlp.append(act(**(act_kwargs or {})))
        prev = d
    return mlp


@dataclass
class DagBatch:
    """All envs' observations as one flat graph batch (node rows env-major, DAGs contiguous)."""
    x: torch.Tensor            # f32 [Nt, 5] Decima node features
    edge_index: torch.Tensor   # i64 [2, Et] (parent, child) in flat node ids
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
    num_envs: int


def build_batch(views: dict, feats: dict, env_mask: torch.Tensor | None = None) -> DagBatch:
    """Flat batch from the obs-arena views (DeviceEngine.views) and the device Decima features
    (DeviceEngine.decima_features). `env_mask` (bool [B]) drops envs (e.g. finished ones)."""
    c = views["counts"]
    dev = c.device
    B, S = views["nodes"].shape[:2]
    E = views["edge_links"].shape[1]
    J = views["exec_supplies"].shape[1]
    n = c[:, _abi.OC_NUM_NODES].long()
    ne = c[:, _abi.OC_NUM_EDGES].long()
    nj = c[:, _abi.OC_NUM_JOBS].long()
    if env_mask is not None:
        keep = env_mask.to(dev)
        n, ne, nj = n * keep, ne * keep, nj * keep
    node_valid = torch.arange(S, device=dev)[None, :] < n[:, None]
    edge_valid = torch.arange(E, device=dev)[None, :] < ne[:, None]
    job_valid = torch.arange(J, device=dev)[None, :] < nj[:, None]
    x = feats["node_feats"][node_valid]
    node_base = torch.cumsum(n, 0) - n
    env_ids = torch.arange(B, device=dev)
    edge_env = torch.repeat_interleave(env_ids, ne)
    links = views["edge_links"][edge_valid]
    edge_index = (links + node_base[edge_env][:, None]).t().contiguous()
    edge_bits = feats["edge_mask"][edge_valid]
    depth = feats["depth"].long()
    env_levels = torch.clamp(depth - 1, min=0) * (n > 0)
    dag_ptr = views["dag_ptr"].long()
    dag_counts = (dag_ptr[:, 1:] - dag_ptr[:, :-1])[job_valid]
    ptr = torch.zeros(dag_counts.numel() + 1, dtype=torch.long, device=dev)
    ptr[1:] = torch.cumsum(dag_counts, 0)
    Nt, Gt = x.shape[0], dag_counts.numel()
    node_dag = torch.repeat_interleave(torch.arange(Gt, device=dev), dag_counts, output_size=Nt)
    node_env = torch.repeat_interleave(env_ids, n, output_size=Nt)
    dag_env = torch.repeat_interleave(env_ids, nj, output_size=Gt)
    obs_ptr = torch.zeros(B + 1, dtype=torch.long, device=dev)
    obs_ptr[1:] = torch.cumsum(nj, 0)
    stage_mask = views["nodes"][:, :, 2][node_valid] != 0
    num_stage_acts = torch.zeros(B, dtype=torch.long, device=dev).index_add_(0, node_env, stage_mask.long())
    return DagBatch(x=x, edge_index=edge_index, edge_bits=edge_bits, max_levels=int(env_levels.max().item()) if B else 0,
                    env_levels=env_levels, ptr=ptr, node_dag=node_dag, node_env=node_env, dag_env=dag_env,
                    obs_ptr=obs_ptr, stage_mask=stage_mask, exec_cap=feats["commit_cap"][job_valid].long(),
                    num_stage_acts=num_stage_acts, num_nodes=n, num_envs=B)


def select_envs(b: DagBatch, envs: torch.Tensor) -> DagBatch:
    """Sub-batch of the observations `envs` (i64 indices into b's env rows, any order), renumbered 0..K-1
    in the given order (the rollout buffer keeps alive envs' observations this way)."""
    dev = b.x.device
    envs = envs.to(dev).long()
    K = envs.numel()
    n_sel = b.num_nodes[envs]
    node_base_old = torch.cumsum(b.num_nodes, 0) - b.num_nodes
    node_start_new = torch.cumsum(n_sel, 0) - n_sel
    Nt = int(n_sel.sum().item()) if K else 0
    new_env_of_node = torch.repeat_interleave(torch.arange(K, device=dev), n_sel, output_size=Nt)
    src_node = node_base_old[envs][new_env_of_node] + (torch.arange(Nt, device=dev) - node_start_new[new_env_of_node])
    old2new = torch.full((b.x.shape[0],), -1, dtype=torch.long, device=dev)
    old2new[src_node] = torch.arange(Nt, device=dev)
    nd_old = b.obs_ptr[1:] - b.obs_ptr[:-1]
    nd_sel = nd_old[envs]
    Gt = int(nd_sel.sum().item()) if K else 0
    new_env_of_dag = torch.repeat_interleave(torch.arange(K, device=dev), nd_sel, output_size=Gt)
    dag_start_new = torch.cumsum(nd_sel, 0) - nd_sel
    src_dag = b.obs_ptr[envs][new_env_of_dag] + (torch.arange(Gt, device=dev) - dag_start_new[new_env_of_dag])
    dag_old2new = torch.full((b.ptr.numel() - 1,), -1, dtype=torch.long, device=dev)
    dag_old2new[src_dag] = torch.arange(Gt, device=dev)
    ekeep = old2new[b.edge_index[0]] >= 0
    ei = old2new[b.edge_index[:, ekeep]]
    eb = b.edge_bits[ekeep]
    order = torch.argsort(ei[0] * max(Nt, 1) + ei[1], stable=True) if ei.shape[1] else None
    if order is not None:  # keep edges grouped per observation in the new env order
        ei, eb = ei[:, order], eb[order]
    dag_counts = (b.ptr[1:] - b.ptr[:-1])[src_dag]
    ptr = torch.zeros(Gt + 1, dtype=torch.long, device=dev)
    ptr[1:] = torch.cumsum(dag_counts, 0)
    obs_ptr = torch.zeros(K + 1, dtype=torch.long, device=dev)
    obs_ptr[1:] = torch.cumsum(nd_sel, 0)
    lv = b.env_levels[envs]
    return DagBatch(x=b.x[src_node], edge_index=ei, edge_bits=eb, max_levels=int(lv.max().item()) if K else 0,
                    env_levels=lv, ptr=ptr, node_dag=dag_old2new[b.node_dag[src_node]], node_env=new_env_of_node,
                    dag_env=new_env_of_dag, obs_ptr=obs_ptr, stage_mask=b.stage_mask[src_node],
                    exec_cap=b.exec_cap[src_dag], num_stage_acts=b.num_stage_acts[envs], num_nodes=n_sel,
                    num_envs=K)


def cat_batches(bs: list[DagBatch]) -> DagBatch:
    """Concatenation of batches (observations in list order)."""
    dev = bs[0].x.device
    n_off = torch.tensor([0] + [b.x.shape[0] for b in bs], device=dev).cumsum(0)
    g_off = torch.tensor([0] + [b.ptr.numel() - 1 for b in bs], device=dev).cumsum(0)
    e_off = torch.tensor([0] + [b.num_envs for b in bs], device=dev).cumsum(0)
    lv = torch.cat([b.env_levels for b in bs])
    return DagBatch(
        x=torch.cat([b.x for b in bs]),
        edge_index=torch.cat([b.edge_index + n_off[i] for i, b in enumerate(bs)], dim=1),
        edge_bits=torch.cat([b.edge_bits for b in bs]),
        max_levels=max(b.max_levels for b in bs), env_levels=lv,
        ptr=torch.cat([bs[0].ptr[:1]] + [b.ptr[1:] + n_off[i] for i, b in enumerate(bs)]),
        node_dag=torch.cat([b.node_dag + g_off[i] for i, b in enumerate(bs)]),
        node_env=torch.cat([b.node_env + e_off[i] for i, b in enumerate(bs)]),
        dag_env=torch.cat([b.dag_env + e_off[i] for i, b in enumerate(bs)]),
        obs_ptr=torch.cat([bs[0].obs_ptr[:1]] + [b.obs_ptr[1:] + g_off[i] for i, b in enumerate(bs)]),
        stage_mask=torch.cat([b.stage_mask for b in bs]), exec_cap=torch.cat([b.exec_cap for b in bs]),
        num_stage_acts=torch.cat([b.num_stage_acts for b in bs]), num_nodes=torch.cat([b.num_nodes for b in bs]),
        num_envs=int(sum(b.num_envs for b in bs)))


def segment_sum(src: torch.Tensor, index: torch.Tensor, size: int) -> torch.Tensor:
    out = torch.zeros((size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    return out.index_add_(0, index, src)


def segment_log_softmax(scores: torch.Tensor, seg: torch.Tensor, nseg: int) -> torch.Tensor:
    """log of pyg.utils.softmax(scores, index=seg) (utils.py:37), without clamping."""
    mx = torch.full((nseg,), -torch.inf, dtype=scores.dtype, device=scores.device)
    mx = mx.scatter_reduce(0, seg, scores, reduce="amax", include_self=True)
    z = scores - mx[seg]
    lse = torch.log(segment_sum(torch.exp(z), seg, nseg))
    return z - lse[seg]


def segment_sample(logp: torch.Tensor, seg: torch.Tensor, nseg: int, generator=None) -> torch.Tensor:
    """One categorical draw per segment (Gumbel-max over log-probabilities); returns flat row indices
    (-1 for empty segments)."""
    u = torch.rand(logp.shape, dtype=torch.float64, device=logp.device, generator=generator)
    g = logp.double() - torch.log(-torch.log(u.clamp_min(1e-300)))
    best = torch.full((nseg,), -torch.inf, dtype=torch.float64, device=logp.device)
    best = best.scatter_reduce(0, seg, g, reduce="amax", include_self=True)
    hit = g == best[seg]
    rows = torch.arange(logp.numel(), device=logp.device)
    out = torch.full((nseg,), -1, dtype=torch.long, device=logp.device)
    return out.scatter_reduce(0, seg[hit], rows[hit], reduce="amax", include_self=True)


class NodeEncoder(nn.Module):
    """scheduler.py:176-245 (reverse flow: children send to parents, deepest level first)."""

    def __init__(self, num_node_features: int, embed_dim: int, mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp_prep = make_mlp(num_node_features, output_dim=embed_dim, **mlp_kwargs)
        self.mlp_msg = make_mlp(embed_dim, output_dim=embed_dim, **mlp_kwargs)
        self.mlp_update = make_mlp(embed_dim, output_dim=embed_dim, **mlp_kwargs)

    def forward(self, b: DagBatch, per_obs_no_mp: bool) -> torch.Tensor:
        h_init = self.mlp_prep(b.x)
        if b.max_levels == 0:
            return h_init  # _forward_no_mp for every observation
        Nt = h_init.shape[0]
        h = torch.zeros_like(h_init)
        parent, child = b.edge_index[0], b.edge_index[1]
        has_child = torch.zeros(Nt, dtype=torch.bool, device=h.device)
        has_child[parent] = True
        leaf = ~has_child
        h[leaf] = self.mlp_update(h_init[leaf])
        for lvl in range(b.max_levels - 1, -1, -1):
            sel = ((b.edge_bits >> lvl) & 1) != 0
            p, ch = parent[sel], child[sel]
            src = torch.zeros(Nt, dtype=torch.bool, device=h.device)
            src[ch] = True
            dst = torch.zeros(Nt, dtype=torch.bool, device=h.device)
            dst[p] = True
            msg = torch.zeros_like(h)
            msg[src] = self.mlp_msg(h[src])
            agg = torch.zeros_like(h).index_add_(0, p, msg[ch])
            h[dst] = h_init[dst] + self.mlp_update(agg[dst])
        if per_obs_no_mp:  # observations without message-passing levels keep h = mlp_prep(x)
            flat = (b.env_levels == 0)[b.node_env]
            h = torch.where(flat[:, None], h_init, h)
        return h


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

    def forward(self, b: DagBatch, per_obs_no_mp: bool) -> dict[str, torch.Tensor]:
        h_node = self.node_encoder(b, per_obs_no_mp)
        h_dag = self.dag_encoder(h_node, b)
        return {"node": h_node, "dag": h_dag, "glob": self.global_encoder(h_dag, b)}


class StagePolicyNetwork(nn.Module):
    """scheduler.py:284-326: one score per schedulable node (rows in flat node order)."""

    def __init__(self, num_node_features: int, emb_dims: dict[str, int], mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.mlp_score = make_mlp(num_node_features + emb_dims["node"] + emb_dims["dag"] + emb_dims["glob"],
                                  output_dim=1, **mlp_kwargs)

    def forward(self, b: DagBatch, h: dict[str, torch.Tensor]) -> torch.Tensor:
        m = b.stage_mask
        inp = torch.cat([b.x[m], h["node"][m], h["dag"][b.node_dag[m]], h["glob"][b.node_env[m]]], dim=1)
        return self.mlp_score(inp).squeeze(-1)


class ExecPolicyNetwork(nn.Module):
    """scheduler.py:329-385: scores of exec actions k/N, k < commit cap of the chosen DAG, per env."""

    def __init__(self, num_executors: int, num_dag_features: int, emb_dims: dict[str, int],
                 mlp_kwargs: dict[str, Any]):
        super().__init__()
        self.num_executors = num_executors
        self.num_dag_features = num_dag_features
        self.mlp_score = make_mlp(num_dag_features + emb_dims["dag"] + emb_dims["glob"] + 1, output_dim=1,
                                  **mlp_kwargs)

    def forward(self, b: DagBatch, h: dict[str, torch.Tensor], dags: torch.Tensor, envs: torch.Tensor):
        """dags/envs: i64 [K] chosen DAG (flat id) and its env per decision. Returns (scores [R], seg [R],
        action k [R]) with R = sum of the chosen DAGs' commit caps."""
        N = self.num_executors
        caps = b.exec_cap[dags].clamp(min=0, max=N)
        seg = torch.repeat_interleave(torch.arange(dags.numel(), device=dags.device), caps)
        start = torch.cumsum(caps, 0) - caps
        k = torch.arange(seg.numel(), device=dags.device) - start[seg]
        x_dag = b.x[b.ptr[dags], : self.num_dag_features]
        x_h_dag = torch.cat([x_dag, h["dag"][dags]], dim=1)
        acts = (torch.arange(N, device=dags.device) / N)[k].unsqueeze(1)
        inp = torch.cat([x_h_dag[seg], h["glob"][envs][seg], acts], dim=1)
        return self.mlp_score(inp).squeeze(-1), seg, k


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

    @torch.no_grad()
    def schedule(self, b: DagBatch, generator=None) -> dict[str, torch.Tensor]:
        """One decision per env (envs with no schedulable stage get stage_idx -1, num_exec 1). Returns device
        tensors: stage_idx i32 [B] (index among the env's schedulable stages), num_exec i32 [B] (already
        1 + the sampled exec action, DecimaActWrapper.action), job_idx i64 [B] (DAG index within the env),
        exec_idx i64 [B], lgprob f32 [B]."""
        B = b.num_envs
        dev = b.x.device
        h = self.encoder(b, per_obs_no_mp=True)
        scores = self.stage_policy_network(b, h)
        sched_env = b.node_env[b.stage_mask]
        logp = segment_log_softmax(scores, sched_env, B)
        pick = segment_sample(logp, sched_env, B, generator)  # flat schedulable-row index
        live = pick >= 0
        sched_base = torch.cumsum(b.num_stage_acts, 0) - b.num_stage_acts
        stage_idx = torch.where(live, pick - sched_base, torch.full_like(pick, -1))
        node_rows = torch.nonzero(b.stage_mask).squeeze(1)
        envs = torch.nonzero(live).squeeze(1)
        dags = b.node_dag[node_rows[pick[envs]]]
        escore, eseg, ek = self.exec_policy_network(b, h, dags, envs)
        elogp = segment_log_softmax(escore, eseg, envs.numel())
        epick = segment_sample(elogp, eseg, envs.numel(), generator)
        exec_idx = torch.zeros(B, dtype=torch.long, device=dev)
        lg = torch.zeros(B, dtype=torch.float32, device=dev)
        job_idx = torch.full((B,), -1, dtype=torch.long, device=dev)
        ok = epick >= 0
        exec_idx[envs[ok]] = ek[epick[ok]]
        lg[envs] = logp[pick[envs]]
        lg[envs[ok]] += elogp[epick[ok]]
        job_idx[envs] = dags - b.obs_ptr[envs]
        return {"stage_idx": stage_idx.to(torch.int32), "num_exec": (exec_idx + 1).to(torch.int32),
                "job_idx": job_idx, "exec_idx": exec_idx, "lgprob": lg}

    def evaluate_actions(self, b: DagBatch, stage_idx: torch.Tensor, job_idx: torch.Tensor,
                         exec_idx: torch.Tensor) -> dict[str, torch.Tensor]:
        """scheduler.py:103-145 over a batch of observations (one per env row of `b`), with grads:
        log-probabilities and normalised entropies of the given actions (utils.py:25-48, clamp_probs)."""
        B = b.num_envs
        dev = b.x.device
        h = self.encoder(b, per_obs_no_mp=False)
        scores = self.stage_policy_network(b, h)
        sched_env = b.node_env[b.stage_mask]
        s_lp, s_ent = _evaluate(scores, sched_env, B, stage_idx.long() + (torch.cumsum(b.num_stage_acts, 0)
                                                                           - b.num_stage_acts))
        envs = torch.arange(B, device=dev)
        dags = job_idx.long() + b.obs_ptr[:-1]
        escore, eseg, ek = self.exec_policy_network(b, h, dags, envs)
        caps = b.exec_cap[dags].clamp(min=0, max=self.num_executors)
        e_lp, e_ent = _evaluate(escore, eseg, B, exec_idx.long() + (torch.cumsum(caps, 0) - caps))
        ent = (s_ent + e_ent) / (self.num_executors * b.num_nodes).float().log()
        return {"lgprobs": s_lp + e_lp, "entropies": ent}


def _evaluate(scores: torch.Tensor, seg: torch.Tensor, nseg: int, sel: torch.Tensor):
    """utils.py:25-48: probs = clamp_probs(pyg softmax); log-prob of the selection, entropy per segment."""
    eps = torch.finfo(scores.dtype).eps
    mx = torch.full((nseg,), -torch.inf, dtype=scores.dtype, device=scores.device)
    mx = mx.scatter_reduce(0, seg, scores.detach(), reduce="amax", include_self=True)
    ex = torch.exp(scores - mx[seg])
    probs = (ex / (segment_sum(ex, seg, nseg) + 1e-16)[seg]).clamp(min=eps, max=1 - eps)
    logp = probs.log()
    ent = -segment_sum(logp * probs, seg, nseg)
    return logp[sel], ent
