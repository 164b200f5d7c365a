"""ctypes mirror of include/sparksched.h (plain C structs; shared by the device library loader)."""

from __future__ import annotations

import ctypes as ct

SSIM_RESET_SKIP, SSIM_RESET_CONTINUE, SSIM_RESET_SEED = 0, 1, 2
SSIM_CFG_FORCE_HBM = 1  # ssim_config.flags (test / diagnostic): hot blocks stay in HBM
NUM_ACC = 8  # int64 accumulators per env (ob_acc): S_act, E_act, J_act, events, decisions, episodes, 0, 0
ACC_NODES, ACC_EDGES, ACC_JOBS, ACC_EVENTS, ACC_DECISIONS, ACC_EPISODES = range(6)
SSIM_ROLLOUT_AUTORESET = 0x1
SSIM_ROLLOUT_PREEMPT = 0x2
SSIM_ROLLOUT_WARMUP = 0x4
SSIM_ROLLOUT_TEST_REJECT = 0x8  # ssim_decima_rollout test hook
SSIM_DEBUG_ENGINE, SSIM_DEBUG_DECIMA, SSIM_DEBUG_KAT_BAD = 0, 1, 2  # ssim_debug_set_trace_ex variants
SSIM_ACT_LEAKY_RELU, SSIM_ACT_TANH = 0, 1  # ssim_mlp3_* activations
SSIM_ERR_SPACE = 0x1
SSIM_ERR_KEY = 0x2
SSIM_ERR_TOO_MANY = 0x4
SSIM_ERR_PENDING = 0x8
SSIM_ERR_INVARIANT = 0x10
SSIM_ERR_CAPACITY = 0x20
SSIM_ERR_SAMPLER = 0x40
SSIM_ERR_RESET = 0x80
SSIM_ERR_STICKY = 0xF0

SSIM_POLICY_FAIR = 1
SSIM_POLICY_FIFO = 2
SSIM_POLICY_RANDOM = 3

# indices into the per-env int32 counts block
OC_NUM_NODES, OC_NUM_EDGES, OC_NUM_JOBS, OC_COMMITTABLE, OC_SOURCE_JOB_IDX, OC_NUM_SCHEDULABLE = range(6)
OC_TERMINATED, OC_TRUNCATED, OC_ERR, OC_DECISIONS, OC_EVENTS, OC_NUM_COMPLETED = range(6, 12)
OC_NUM_ARRIVED, OC_TRACE_LEN, OC_STEP_EVENTS, OC_EPISODE = range(12, 16)
NUM_COUNTS = 16
RESET_HEAD_BYTES = 64
TRACE_BYTES = 32
# trace record kinds: events (arrival, task finished, executor ready) and trace-only records
TR_ARRIVAL, TR_TASK, TR_READY, TR_JOB_DONE, TR_TO_COMMON = range(1, 6)


class SsimConfig(ct.Structure):
    _fields_ = [
        ("num_envs", ct.c_int32),
        ("num_executors", ct.c_int32),
        ("job_cap", ct.c_int32),
        ("max_stages", ct.c_int32),
        ("max_edges", ct.c_int32),
        ("trace_cap", ct.c_int32),
        ("moving_delay", ct.c_double),
        ("warmup_delay", ct.c_double),
        ("beta", ct.c_double),
        ("job_arrival_gap", ct.c_double),
        ("job_arrival_cap", ct.c_int32),
        ("flags", ct.c_int32),  # SSIM_CFG_*
    ]


class SsimDataset(ct.Structure):
    _fields_ = [
        ("num_templates", ct.c_int32),
        ("num_template_stages", ct.c_int32),
        ("tpl_stage_base", ct.c_void_p),
        ("ts_num_tasks", ct.c_void_p),
        ("ts_rough", ct.c_void_p),
        ("ts_child_base", ct.c_void_p),
        ("ts_children", ct.c_void_p),
        ("ts_parent_base", ct.c_void_p),
        ("ts_parents", ct.c_void_p),
        ("ts_fw_keymask", ct.c_void_p),
        ("ts_fw_maxlevel", ct.c_void_p),
        ("dur_off", ct.c_void_p),
        ("dur_len", ct.c_void_p),
        ("durations", ct.c_void_p),
        ("intervals", ct.c_void_p),
        ("ts_topo", ct.c_void_p),
    ]


# order of the pointer fields above = order of arrays in PackedDataset.arrays()
DATASET_ARRAYS = [
    "tpl_stage_base", "ts_num_tasks", "ts_rough", "ts_child_base", "ts_children", "ts_parent_base",
    "ts_parents", "ts_fw_keymask", "ts_fw_maxlevel", "dur_off", "dur_len", "durations", "intervals", "ts_topo",
]


class SsimResetRecord(ct.Structure):
    _fields_ = [
        ("rng_state_hi", ct.c_uint64),
        ("rng_state_lo", ct.c_uint64),
        ("rng_inc_hi", ct.c_uint64),
        ("rng_inc_lo", ct.c_uint64),
        ("rng_has_uint32", ct.c_uint32),
        ("rng_uinteger", ct.c_uint32),
        ("num_jobs", ct.c_int32),
        ("pad", ct.c_int32),
        ("time_limit", ct.c_double),
    ]


class SsimLayout(ct.Structure):
    _fields_ = [(n, ct.c_int32) for n in (
        "num_envs", "num_executors", "job_cap", "stage_cap", "edge_cap", "pool_cap", "set_cap", "commit_cap",
        "trace_cap", "lds_resident")] + [(n, ct.c_int64) for n in (
        "env_bytes", "state_bytes", "obs_bytes", "reset_bytes", "reset_stride", "scratch_bytes",
        "ob_nodes", "ob_edge_links", "ob_dag_ptr", "ob_supplies", "ob_frontier", "ob_sched_rank", "ob_counts",
        "ob_reward", "ob_wall_time", "ob_acc", "ob_trace", "lds_bytes", "lds_share", "chip_cus")]


class SsimDecimaSamples(ct.Structure):
    """ssim_decima_samples: the persistent Decima rollout's per-env sample arena (device pointers)."""
    _fields_ = [("cursor", ct.c_void_p), ("rec", ct.c_void_p), ("nodes", ct.c_void_p), ("edges", ct.c_void_p),
                ("dags", ct.c_void_p), ("cap_samples", ct.c_int32), ("cap_nodes", ct.c_int32),
                ("cap_edges", ct.c_int32), ("cap_dags", ct.c_int32)]


# ssim_decima_sample (64 B): int32 fields, then float lgprob, then f64 wall_before / reward
SAMPLE_I32 = ["num_nodes", "num_edges", "num_dags", "depth", "node_off", "edge_off", "dag_off", "stage_idx",
              "job_idx", "exec_idx", "num_exec"]
SAMPLE_BYTES = 64
SAMPLE_LGPROB = 11  # float32 word index
SAMPLE_WALL, SAMPLE_REWARD = 6, 7  # float64 word indices
CURSOR_WORDS = 8
CUR_SAMPLES, CUR_NODES, CUR_EDGES, CUR_DAGS, CUR_FULL, CUR_NEED_NODES, CUR_NEED_EDGES, CUR_NEED_DAGS = range(8)


def layout_dict(layout: SsimLayout) -> dict:
    return {name: getattr(layout, name) for name, _ in SsimLayout._fields_}
