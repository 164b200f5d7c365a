"""TEST INFRASTRUCTURE ONLY — CPU restatement of the Decima observation wrapper, the checker for the
device featurisation (csrc/decima.h, ssim_decima_features). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this package.

Follows schedulers/decima/env_wrapper.py:69-143 (DecimaObsWrapper.observation, _build_node_features) and
schedulers/decima/utils.py:238-267 (make_dag_layer_edge_masks) line by line with the same numpy dtypes and
the same third-party call (networkx.topological_generations, networkx 3.x: the reference pins 3.1,
requirements.txt:20; generations are a pure function of the graph, so the version does not matter here).
Parity for the float features is pinned by the reference's dtype rules: f64 quotients assigned into an f32
array for columns 0 and 2, f32 arithmetic for columns 3 and 4 (numpy value-based / NEP 50 casting agree
for a python-scalar divisor).
"""

from __future__ import annotations

import networkx as nx
import numpy as np

NUM_NODE_FEATURES = 5  # env_wrapper.py:9


def make_dag_layer_edge_masks(edge_links: np.ndarray, num_nodes: int) -> np.ndarray:
    """utils.py:238-267 (tuple input path, np_to_nx utils.py:270-274)."""
    G = nx.DiGraph()
    G.add_nodes_from(range(num_nodes))
    G.add_edges_from(edge_links)
    node_levels = list(nx.topological_generations(G))
    if len(node_levels) <= 1:
        return np.zeros((0, edge_links.shape[0]), dtype=bool)
    node_mask = np.zeros(len(G), dtype=bool)
    edge_masks = []
    for node_level in node_levels[:-1]:
        succ = set.union(*[set(G.successors(n)) for n in node_level])
        node_mask[:] = 0
        node_mask[node_level + list(succ)] = True
        edge_masks += [node_mask[edge_links[:, 0]] & node_mask[edge_links[:, 1]]]
    return np.stack(edge_masks)


def decima_observation(obs: dict, num_executors: int, num_tasks_scale: int = 200, work_scale: float = 1e5) -> dict:
    """DecimaObsWrapper.observation (env_wrapper.py:69-108) on a base observation dict."""
    dag_batch = obs["dag_batch"]
    exec_supplies = np.array(obs["exec_supplies"])
    num_committable_execs = obs["num_committable_execs"]
    gap = np.maximum(num_executors - exec_supplies, 0)
    commit_caps = np.minimum(gap, num_committable_execs)
    j_src = obs["source_job_idx"]
    num_jobs = exec_supplies.size
    if j_src < num_jobs:
        commit_caps[j_src] = num_committable_execs

    # _build_node_features (env_wrapper.py:110-143)
    num_nodes = dag_batch.nodes.shape[0]
    ptr = np.array(obs["dag_ptr"])
    node_counts = ptr[1:] - ptr[:-1]
    nodes = np.zeros((num_nodes, NUM_NODE_FEATURES), dtype=np.float32)
    nodes[:, 0] = np.repeat(commit_caps, node_counts) / num_executors
    nodes[:, 1] = -1
    if j_src < len(obs["exec_supplies"]):
        nodes[ptr[j_src]: ptr[j_src + 1], 1] = 1
    nodes[:, 2] = np.repeat(np.asarray(obs["exec_supplies"]), node_counts) / num_executors
    num_remaining_tasks = dag_batch.nodes[:, 0]
    nodes[:, 3] = num_remaining_tasks / num_tasks_scale
    most_recent_duration = dag_batch.nodes[:, 1]
    nodes[:, 4] = num_remaining_tasks * most_recent_duration / work_scale

    stage_mask = dag_batch.nodes[:, 2].astype(bool)
    exec_mask = np.zeros((num_jobs, num_executors), dtype=bool)
    for j, cap in enumerate(commit_caps):
        exec_mask[j, :cap] = True
    edge_links = np.asarray(dag_batch.edge_links, dtype=np.int64).reshape(-1, 2)
    return {
        "nodes": nodes,
        "edges": dag_batch.edges,
        "edge_links": edge_links,
        "dag_ptr": obs["dag_ptr"],
        "stage_mask": stage_mask,
        "exec_mask": exec_mask,
        "commit_caps": commit_caps,
        "edge_masks": make_dag_layer_edge_masks(edge_links, num_nodes),
    }
