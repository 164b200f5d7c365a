/*
 * sparksched.h — C ABI of the MI355X-native batched Spark scheduling simulator.
 *
 * Drop-in boundary for the reference's hot path (ArchieGertsman/gym-sparksched, snapshot 2025-02-22):
 *   SparkSchedSimEnv.reset/step and observation construction
 *   (spark_sched_sim/spark_sched_sim.py:127-221, 345-406) batched over many independent envs in HBM.
 *
 * Conventions: plain C types only (no torch types); every device buffer is caller-allocated device
 * memory (hipMalloc or a torch tensor); streams are passed as `void*` (hipStream_t, NULL = default).
 * Every entry point returns 0 on success or a negative SSIM_E_* code, and ssim_last_error() then holds
 * a message. Per-env failures (invalid action, reference assertion, capacity) do NOT fail the call:
 * they are reported in the per-env `err` bitmask of the observation arena (SSIM_ERR_* bits).
 * A handle is not thread-safe; all work is stream-ordered on the caller's stream.
 */
#ifndef SPARKSCHED_H
#define SPARKSCHED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ------------------------------------------------------------------------------ */
#define SSIM_OK 0
#define SSIM_E_ARG -1    /* bad argument / inconsistent sizes */
#define SSIM_E_HIP -2    /* HIP runtime error (message in ssim_last_error) */

/* ---- per-env error bits (obs arena `err` field) ------------------------------------------------- */
#define SSIM_ERR_SPACE 0x1u       /* ValueError: action not in action space (spark_sched_sim.py:276-277) */
#define SSIM_ERR_KEY 0x2u         /* KeyError: stage_idx >= #schedulable stages (spark_sched_sim.py:284) */
#define SSIM_ERR_TOO_MANY 0x4u    /* ValueError: num_exec > committable executors (:294-295) */
#define SSIM_ERR_PENDING 0x8u     /* the env's last step was preempted mid-simulation (SSIM_ROLLOUT_PREEMPT); the obs
                                     arena still holds the previous observation; any ssim_rollout_* call or
                                     ssim_step completes it (ssim_step then ignores its action for that env) */
#define SSIM_ERR_INVARIANT 0x10u  /* an `assert` of the reference fired; env frozen */
#define SSIM_ERR_CAPACITY 0x20u   /* a device capacity (commitments, trace) overflowed; env frozen */
#define SSIM_ERR_SAMPLER 0x40u    /* task_duration found no durations (reference raises); env frozen */
#define SSIM_ERR_RESET 0x80u      /* reset batch inconsistent with the config; env frozen */
#define SSIM_ERR_STICKY 0xF0u     /* bits that freeze the env until its next reset */

/* ---- device policies (action drivers; schedulers/heuristics) -------------------------------- */
#define SSIM_POLICY_FAIR 1    /* RoundRobinScheduler(dynamic_partition=True), round_robin.py:14-49 */
#define SSIM_POLICY_FIFO 2    /* RoundRobinScheduler(dynamic_partition=False) */
#define SSIM_POLICY_RANDOM 3  /* uniform-random valid action from a counter-based device RNG */

/* Env configuration (spark_sched_sim.py:37-52, tpch.py:19-49). */
typedef struct ssim_config {
  int32_t num_envs;
  int32_t num_executors;  /* N */
  int32_t job_cap;        /* max jobs per episode (job_arrival_cap, or a bound for time-limited runs) */
  int32_t max_stages;     /* max stages of any dataset template */
  int32_t max_edges;      /* max edges of any dataset template */
  int32_t trace_cap;      /* per-env event-trace records (0 = tracing off) */
  double moving_delay;    /* ms, spark_sched_sim.py:40 */
  double warmup_delay;    /* ms, tpch.py:44 */
  double beta;            /* reward discount, spark_sched_sim.py:44 */
  /* device-side job-sequence sampling (ssim_reset_sampled, rollout auto-reset; tpch.py:54-73) */
  double job_arrival_gap; /* 1 / job_arrival_rate, ms (computed by the caller, as Python does) */
  int32_t job_arrival_cap;/* 0 = no cap (time-limited episodes) */
  int32_t flags;          /* SSIM_CFG_* */
} ssim_config;

/* ssim_config.flags. SSIM_CFG_FORCE_HBM (test / diagnostic): keep every env's hot block in HBM (the kernels_hbm()
 * instantiations) even when it would fit the LDS, so small batches exercise the HBM-resident path the large
 * configurations run. */
#define SSIM_CFG_FORCE_HBM 1

/* Packed TPC-H-format dataset (device pointers). Built on the host from the raw per-query dicts by the
 * packer, which restates tpch.py:135-206 (preprocessing, num_tasks, rough duration). Template id =
 * (query_num-1)*7 + size_index. Duration lists: for template-stage ts, wave w (0 fresh_durations,
 * 1 first_wave(cleaned), 2 rest_wave) and exec level l (EXEC_LEVELS index 0..7):
 * dur_len[(ts*3+w)*8+l] = -1 if the key is missing, else the list length, at durations[dur_off[...]]. */
typedef struct ssim_dataset {
  int32_t num_templates;
  int32_t num_template_stages;
  const int32_t* tpl_stage_base;  /* [T+1] */
  const int32_t* ts_num_tasks;    /* [TS] */
  const double* ts_rough;         /* [TS] initial most_recent_duration */
  const int32_t* ts_child_base;   /* [TS+1] CSR into ts_children (local stage ids, ascending) */
  const int32_t* ts_children;
  const int32_t* ts_parent_base;  /* [TS+1] CSR into ts_parents */
  const int32_t* ts_parents;
  const int32_t* ts_fw_keymask;   /* [TS] bit l set <=> EXEC_LEVELS[l] is a first_wave key */
  const int32_t* ts_fw_maxlevel;  /* [TS] level index of max(first_wave) */
  const int32_t* dur_off;         /* [TS*3*8] */
  const int32_t* dur_len;         /* [TS*3*8] */
  const double* durations;
  const double* intervals;        /* [(N+1)*2] executor_intervals (tpch.py:237-262) */
  const uint64_t* ts_topo;        /* [TS] the same DAG as bit sets of local stage ids when every template has
                                     <= 32 stages (config max_stages <= 32): parents in bits 0-31, children in bits
                                     32-63; one load gives a stage's whole neighbourhood (the CSR takes a chain of
                                     dependent loads). Ignored for max_stages > 32. */
} ssim_dataset;

/* Per-env reset record (host-sampled job sequence; spark_sched_sim.py:127-186 / tpch.py:54-73).
 * In the reset arena each env owns `reset_stride` bytes: this record (padded to 64 B), then
 * double t_arrival[job_cap], then int32 tpl[job_cap] (template id per job, in arrival order). */
typedef struct ssim_reset_record {
  uint64_t rng_state_hi, rng_state_lo, rng_inc_hi, rng_inc_lo; /* numpy PCG64 state after sampling */
  uint32_t rng_has_uint32, rng_uinteger;
  int32_t num_jobs;    /* 0 = leave this env untouched */
  int32_t pad;
  double time_limit;   /* for the `truncated` flag (wrappers/stochastic_time_limit.py:26-31); +inf = none */
} ssim_reset_record;

/* Sizes and byte offsets. State offsets are within one env's block (stride env_bytes); obs offsets are
 * absolute within the obs arena, each field strided per env as documented. */
typedef struct ssim_layout {
  int32_t num_envs, num_executors, job_cap, stage_cap, edge_cap, pool_cap, set_cap, commit_cap, trace_cap;
  int32_t lds_resident;    /* 1: the engine kernels hold each env's hot block in LDS for a launch, 0: in HBM */
  int64_t env_bytes, state_bytes, obs_bytes, reset_bytes, reset_stride, scratch_bytes;
  /* obs arena (zero-copy views):                                           element   per-env shape   */
  int64_t ob_nodes;        /* float32  [stage_cap][3]  (remaining, most_recent_duration, schedulable) */
  int64_t ob_edge_links;   /* int64    [edge_cap][2]   */
  int64_t ob_dag_ptr;      /* int32    [job_cap+1]     */
  int64_t ob_supplies;     /* int32    [job_cap]       */
  int64_t ob_frontier;     /* uint8    [stage_cap]     node has no active parent (heuristics/utils.py:6-8) */
  int64_t ob_sched_rank;   /* int32    [stage_cap]     schedulable index of node, -1 if not schedulable */
  int64_t ob_counts;       /* int32    [16]            see SSIM_OC_* */
  int64_t ob_reward;       /* float64  [1] */
  int64_t ob_wall_time;    /* float64  [1] */
  int64_t ob_acc;          /* int64    [8]             running sums over all episodes: S_act, E_act, J_act,
                                                      events popped, decisions, finished episodes, 0, 0 */
  int64_t ob_trace;       /* float64/int32 trace records, [trace_cap] x 32 B */
  int64_t lds_bytes;       /* dynamic LDS of one engine workgroup (one env): scratch, plus the hot block if resident */
  int64_t lds_share;       /* LDS one env may hold without lowering the workgroups per CU the residency decision
                              assumed (LDS-resident: 160 KB / envs per CU, the whole CU when num_envs <= chip_cus;
                              HBM-resident: 160 KB / 16); the Decima rollout's policy plan stays within it */
  int64_t chip_cus;        /* compute units of the device the layout was computed for (current device) */
} ssim_layout;

/* indices into the per-env int32 counts block */
#define SSIM_OC_NUM_NODES 0
#define SSIM_OC_NUM_EDGES 1
#define SSIM_OC_NUM_JOBS 2        /* active jobs = len(exec_supplies) */
#define SSIM_OC_COMMITTABLE 3     /* num_committable_execs */
#define SSIM_OC_SOURCE_JOB_IDX 4
#define SSIM_OC_NUM_SCHEDULABLE 5
#define SSIM_OC_TERMINATED 6
#define SSIM_OC_TRUNCATED 7
#define SSIM_OC_ERR 8
#define SSIM_OC_DECISIONS 9       /* successful env.step calls this episode */
#define SSIM_OC_EVENTS 10         /* events popped this episode */
#define SSIM_OC_NUM_COMPLETED 11  /* completed jobs */
#define SSIM_OC_NUM_ARRIVED 12    /* arrived jobs (completed + active) */
#define SSIM_OC_TRACE_LEN 13
#define SSIM_OC_STEP_EVENTS 14    /* events popped by the last step (K of SURVEY §8d) */
#define SSIM_OC_EPISODE 15
#define SSIM_NUM_COUNTS 16

typedef struct ssim_handle ssim_handle;

/* Compute all sizes/offsets for a config. No device work. */
int ssim_layout_for(const ssim_config* cfg, ssim_layout* out);

/* Bind caller-allocated device memory: state arena (layout.state_bytes), obs arena (layout.obs_bytes),
 * reset staging (layout.reset_bytes). `dataset` holds device pointers and must outlive the handle. */
int ssim_create(const ssim_config* cfg, const ssim_dataset* dataset, void* state_arena, void* obs_arena,
                void* reset_arena, ssim_handle** out);
int ssim_destroy(ssim_handle* h);

/* Reset every env whose record in `reset_arena` has num_jobs > 0 (records written by the caller, e.g.
 * one hipMemcpyAsync of the host-packed buffer). Runs _load_initial_jobs and writes the first obs. */
int ssim_reset(ssim_handle* h, void* stream);

/* One env.step per env: stage_idx[num_envs], num_exec[num_envs] are device int32 arrays.
 * Envs that are terminated or frozen are skipped (their obs/flags stay as they are). */
int ssim_step(ssim_handle* h, const int32_t* stage_idx, const int32_t* num_exec, void* stream);

/* Device action drivers: write stage_idx/num_exec for every env from the current obs. `counter` is the
 * decision counter mixed into the random policy's counter-based stream. */
int ssim_policy(ssim_handle* h, int32_t kind, uint64_t seed, uint64_t counter, int32_t* stage_idx,
                int32_t* num_exec, void* stream);

/* Device-side reset: for every env with mode[env] != SSIM_RESET_SKIP the job sequence
 * is sampled on the device from the env's numpy Generator(PCG64) stream exactly as TPCHDataSampler.
 * job_sequence does (tpch.py:54-73: integers(22), choice(7 sizes), exponential(1/rate) by numpy's ziggurat),
 * then the env is reset as by ssim_reset (spark_sched_sim.py:127-186). Device arrays [num_envs]:
 *   mode        uint8   SSIM_RESET_SKIP | SSIM_RESET_CONTINUE (reset(seed=None): continue the env's stream)
 *                       | SSIM_RESET_SEED (reset(seed=s): Generator(PCG64(SeedSequence(seeds[env]))))
 *   seeds       uint64  (may be NULL when no env uses SSIM_RESET_SEED)
 *   time_limits float64 StochasticTimeLimit limits (+inf = none); NULL = +inf for every env.
 * Needs job_arrival_gap (and job_arrival_cap or finite limits) in the config. Uses the reset arena as
 * scratch for the sampled records. */
#define SSIM_RESET_SKIP 0
#define SSIM_RESET_CONTINUE 1
#define SSIM_RESET_SEED 2
int ssim_reset_sampled(ssim_handle* h, const uint8_t* mode, const uint64_t* seeds, const double* time_limits,
                       void* stream);

/* Fused rollout: `num_steps` x (device policy -> step) in ONE launch, obs written every step. The random
 * policy's counter is (episode << 32) + decisions of each env. `action_log` (optional, device int32
 * [num_steps][num_envs][2]) receives every action taken, for replay/parity. */
int ssim_rollout(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps, int32_t* action_log,
                 void* stream);

/* ssim_rollout with flags. SSIM_ROLLOUT_AUTORESET: an env whose episode ends (terminated, or truncated by
 * its time limit: wall_time >= limit) is reset in place on the device with reset(seed=None) semantics
 * (continuing its RNG stream, as ssim_reset_sampled SSIM_RESET_CONTINUE) and keeps stepping; the new
 * episode's limit is time_limits[env] (device float64 [num_envs], NULL = +inf). Each env's obs counts
 * carry its episode number (SSIM_OC_EPISODE). */
#define SSIM_ROLLOUT_AUTORESET 0x1
/* ssim_rollout_budget only: once the budget is spent, an env in the middle of a step stops at the next event
 * boundary instead of finishing the step (the launch ends within ~one event rather than ~the longest step);
 * the step stays pending (SSIM_ERR_PENDING) and the next launch on the handle completes it first. Decisions
 * are counted when they complete (ob_acc), so back-to-back launches count every decision exactly once. With
 * SSIM_ROLLOUT_AUTORESET an episode that ends once the budget is spent is reset at the start of the env's next
 * launch (before its next decision), so until then its observation is the terminal one. */
#define SSIM_ROLLOUT_PREEMPT 0x2
/* Same rollout, launched under the kernel symbol k_rollout_warmup instead of k_rollout, so a profiler's per-kernel
 * statistics can tell launches that are not measured (a benchmark's pre-roll and warm-up) from measured ones. */
#define SSIM_ROLLOUT_WARMUP 0x4
/* ssim_decima_rollout only, a test hook: the launch's first decision of every env asks for N + 1 executors, an action
 * the env refuses (the env freezes with SSIM_ERR_INVARIANT and the sample recorded for it is dropped). */
#define SSIM_ROLLOUT_TEST_REJECT 0x8
int ssim_rollout_ex(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps, int32_t flags,
                    const double* time_limits, int32_t* action_log, void* stream);

/* Work-conserving rollout: a shared budget of `total_decisions` decisions over all envs (each env at most
 * `max_steps`), claimed from a device counter in chunks sized to what is left. Envs whose decisions are cheap
 * take more of the budget, so the launch ends when the budget is spent rather than when the env with the most
 * expensive `num_steps` decisions finishes (cf. the reference's fixed-duration RolloutWorkerAsync,
 * trainers/rollout_worker.py:160-206, which stops each worker by wall time rather than by step count).
 * Each env's decisions are the same as in ssim_rollout_ex (its policy counter is its own decision count);
 * only how many each env takes differs. action_log rows [max_steps][num_envs][2]; rows an env did not reach
 * are left untouched. Terminated envs stop claiming unless SSIM_ROLLOUT_AUTORESET is set. */
int ssim_rollout_budget(ssim_handle* h, int32_t kind, uint64_t seed, int32_t max_steps, int64_t total_decisions,
                        int32_t flags, const double* time_limits, int32_t* action_log, void* stream);

/* ssim_rollout_ex with a per-env decision count: env i takes min(env_steps[i], max_steps) decisions (device int32
 * [num_envs]); action_log rows as ssim_rollout_ex. Used to spread a batch over the phases of its episodes (a
 * benchmark's pre-roll) or to give every env its own horizon. */
int ssim_rollout_steps(ssim_handle* h, int32_t kind, uint64_t seed, const int32_t* env_steps, int32_t max_steps,
                       int32_t flags, const double* time_limits, int32_t* action_log, void* stream);

/* Per-job results for metrics (spark_sched_sim/metrics.py): t_arrival/t_completed float64 [num_envs][job_cap]
 * and job state int32 [num_envs][job_cap] (0 not arrived, 1 active, 2 completed), any may be NULL. */
int ssim_job_times(ssim_handle* h, double* t_arrival, double* t_completed, int32_t* state, void* stream);

/* Decima observation features from the current obs (replaces DecimaObsWrapper.observation,
 * schedulers/decima/env_wrapper.py:69-143, and make_dag_layer_edge_masks, schedulers/decima/utils.py:238-267).
 * Device outputs, caller-allocated, env-major:
 *   node_feats float [num_envs][stage_cap][5]   rows < num_nodes (the reference's 5 node features)
 *   commit_cap int32 [num_envs][job_cap]         exec_mask[j, :commit_cap[j]] = True, rows < num_jobs
 *   edge_mask  uint32 [num_envs][edge_cap]       bit l = edge in message-passing mask l, l < depth - 1
 *   depth      int32 [num_envs]                  topological generations (masks are (max(depth-1,0), E))
 * Reference defaults: num_tasks_scale 200, work_scale 1e5. Requires max_stages <= 32 (SSIM_E_ARG). */
int ssim_decima_features(ssim_handle* h, float num_tasks_scale, float work_scale, float* node_feats,
                         int32_t* commit_cap, uint32_t* edge_mask, int32_t* depth, void* stream);

/* Fused Decima policy (schedulers/decima/scheduler.py:70-101 DecimaScheduler.schedule) for the
 * decima_tpch.yaml architecture (embed 16, GNN MLPs [32,16] LeakyReLU(0.2), policy MLPs [64,64] Tanh;
 * num_params must be 20802): one launch encodes every env's DAG batch from the obs arena and the
 * ssim_decima_features outputs, scores the schedulable stages and the exec actions, and samples both
 * (Gumbel-max on a counter-based stream of (seed, env, counter)). `params`: fp32 device buffer, the
 * module's parameters in DecimaScheduler.parameters() order, torch nn.Linear layout (DecimaScheduler.packed_params). `node_cap`: the per-env
 * activation plan (>= the largest env's node count; 0 = stage_cap); envs above it are skipped and counted in
 * `overflow` (device int32, optional). The plan lives in LDS when it fits a workgroup's 160 KB, else in a global
 * region the handle allocates (and grows) on demand. env_mask (optional uint8 [B]): 0 = skip the env.
 * Outputs [B]: stage_idx (index among schedulable stages, -1 none), num_exec (= 1 + exec_idx), job_idx
 * (active-job index), exec_idx, lgprob (log-probability of both choices); optional stage_scores
 * [B][stage_cap] and exec_scores [B][N] (for checking).
 * Stream use: each call repacks `params` into ONE handle-owned operand buffer on `stream` before its launch, so calls on
 * one handle must be ordered on one stream (as every call on a handle is, see ssim_create): two calls on different
 * streams could overwrite the packed weights while the earlier launch still reads them. */
int ssim_decima_policy(ssim_handle* h, const float* node_feats, const int32_t* commit_cap, const uint32_t* edge_mask,
                       const int32_t* depth, const float* params, int32_t num_params, int32_t node_cap, uint64_t seed,
                       uint64_t counter, const uint8_t* env_mask, int32_t* stage_idx, int32_t* num_exec,
                       int32_t* job_idx, int32_t* exec_idx, float* lgprob, float* stage_scores, float* exec_scores,
                       int32_t* overflow, void* stream);

/* ---- persistent Decima rollouts -------------------------------------------------
 * One launch runs, per env and per decision: the Decima features of the current observation (as
 * ssim_decima_features), the fused Decima policy (as ssim_decima_policy) and env.step with the sampled action, with
 * no host round trip and no env waiting for another (replaces the per-decision loop of
 * trainers/rollout_worker.py:135-157 RolloutWorkerSync.collect_rollout: DecimaObsWrapper.observation,
 * DecimaScheduler.schedule, env.step). The optional sample arena receives what the PPO learner needs per decision
 * (rollout_worker.py:18-46 RolloutBuffer: observation, action, log-probability, reward, wall time). */
typedef struct ssim_decima_sample { /* 64 B, one per decision */
  int32_t num_nodes, num_edges, num_dags, depth; /* observation sizes; depth as ssim_decima_features */
  int32_t node_off, edge_off, dag_off;           /* first row of the observation in the env's node / edge / DAG region */
  int32_t stage_idx, job_idx, exec_idx, num_exec;/* the action (as ssim_decima_policy's outputs) */
  float lgprob;
  double wall_before;                            /* wall time before the step */
  double reward;                                 /* the step's reward */
} ssim_decima_sample;
typedef struct ssim_decima_samples {
  int32_t* cursor;             /* device int32 [num_envs][8]: samples, node rows, edge rows, DAG rows used (the caller
                                  zeroes it before a collection); [4] = 1 when the env stopped because a region was full
                                  (grow the arena, clear the flag, launch again: the env continues where it stopped);
                                  [5..7] = the node, edge and DAG rows the observation that did not fit needs */
  ssim_decima_sample* rec;     /* [num_envs][cap_samples] */
  float* nodes;                /* [num_envs][cap_nodes][6]: the 5 Decima node features, then the schedulable flag */
  int32_t* edges;              /* [num_envs][cap_edges][4]: parent, child (node rows of the observation), edge-mask word, 0 */
  int32_t* dags;               /* [num_envs][cap_dags][2]: node count, commit cap (exec_mask[j, :cap]) */
  int32_t cap_samples, cap_nodes, cap_edges, cap_dags;
} ssim_decima_samples;

/* Bytes of the per-env workspace ssim_decima_rollout needs for this handle's layout (device memory, caller-owned). */
int64_t ssim_decima_workspace_bytes(const ssim_handle* h);

/* Dynamic LDS bytes per workgroup (one env) of this handle's ssim_decima_rollout launch: the engine's LDS plus the
 * policy plan, within the env's share of its compute unit (ssim_layout.lds_share). Diagnostic / sizing query. */
int64_t ssim_decima_rollout_lds_bytes(const ssim_handle* h);

/* Decima rollouts in one launch. `params`/`num_params` as ssim_decima_policy; num_tasks_scale / work_scale as
 * ssim_decima_features. Each env takes at most `max_steps` decisions. Sampling stream: (seed, env, counter + the env's
 * decision index in its episode), plus (episode << 32) with SSIM_ROLLOUT_AUTORESET. flags:
 *   0: collection — an env stops when its episode ends (terminated, truncated: wall_time >= its time limit);
 *   SSIM_ROLLOUT_AUTORESET: finished episodes are reset in place (time_limits as ssim_rollout_ex) and the env goes on;
 *   SSIM_ROLLOUT_PREEMPT with total_decisions > 0: a shared decision budget as ssim_rollout_budget;
 *   SSIM_ROLLOUT_WARMUP: the launch runs under the symbol k_decima_rollout_warmup (unmeasured launches).
 * total_decisions: 0 = no budget. samples: optional sample arena (NULL = none). action_log: optional int32
 * [max_steps][num_envs][2] (stage_idx, num_exec of every decision started in this launch). */
int ssim_decima_rollout(ssim_handle* h, const float* params, int32_t num_params, float num_tasks_scale,
                        float work_scale, uint64_t seed, uint64_t counter, int32_t max_steps, int64_t total_decisions,
                        int32_t flags, const double* time_limits, void* workspace, int64_t workspace_bytes,
                        const ssim_decima_samples* samples, int32_t* action_log, void* stream);

const char* ssim_last_error(void);

/* Test hook, not part of the drop-in surface: a trace of CPython-set operations (add / remove / idle order) on one
 * executor pool of env 0 through the engine's own set code, for known-answer tests against CPython
 * (tests/test_gpu_sets.py). ops: device int32 [n_ops][6] = (code, key, busy bitmap words 0..3), code 0 add, 1 remove,
 * 2 idle order (list(set(e for e in pool.copy() if not busy[e])), spark_sched_sim.py:714-728); orders: device int32
 * [n_ops][width], the set's iteration order after codes 0/1 and the idle order for code 2, -1 padded. Clobbers env 0;
 * needs 1..127 executors. */
int ssim_debug_set_trace(ssim_handle* h, const int32_t* ops, int32_t n_ops, int32_t width, int32_t* orders,
                         void* stream);
/* The same trace through a chosen engine instantiation, compiled in the translation unit (with the flags) of the kernels
 * a launch on this handle runs: SSIM_DEBUG_ENGINE = ssim_step / ssim_rollout*'s (what ssim_debug_set_trace runs),
 * SSIM_DEBUG_DECIMA = ssim_decima_rollout's, SSIM_DEBUG_KAT_BAD = a test-only instantiation that reproduces the effect
 * of the ROCm 7.2 page-assembly miscompile the engine works around (N = 100 / job cap 200, HBM-resident layouts only:
 * the KAT must fail on it). SSIM_E_ARG when the variant does not apply to the handle's layout. */
#define SSIM_DEBUG_ENGINE 0
#define SSIM_DEBUG_DECIMA 1
#define SSIM_DEBUG_KAT_BAD 2
int ssim_debug_set_trace_ex(ssim_handle* h, const int32_t* ops, int32_t n_ops, int32_t width, int32_t* orders,
                            int32_t variant, void* stream);
/* Name of the kernel translation unit a variant selects for this handle ("hbm_n100", "bench900", "dr_hbm50", ...; ""
 * when the variant does not apply). */
const char* ssim_debug_kernel_name(const ssim_handle* h, int32_t variant);

/* The PPO learner's small dense layers (widths <= 64: the Decima MLPs) on the device, replacing the nn.Linear GEMMs
 * of trainers/ppo.py's evaluate_actions passes (reference: schedulers/decima/utils.py:51-70 make_mlp, trained by
 * trainers/ppo.py:105-138). Row-major f32 device arrays; returns 0, or -1 for widths outside 1..64.
 * ssim_linear_fwd: y[r][j] = b[j] + sum_i x[r][i] * w(i, j), w(i, j) = w[j * in_dim + i] if transpose_w (nn.Linear's
 * [out][in] weight: the forward) else w[i * out_dim + j] (the input gradient, dX = dY W); b may be NULL.
 * ssim_linear_wgrad: gw[j][i] = sum_r gy[r][j] * x[r][i], gb[j] = sum_r gy[r][j] (gb may be NULL), through
 * `partial` (parts x out_dim x (in_dim + 1) floats; parts = ssim_linear_wgrad_parts(rows)), summed in chunk order:
 * deterministic. */
int ssim_linear_fwd(const float* x, const float* w, const float* b, float* y, int64_t rows, int32_t in_dim,
                    int32_t out_dim, int32_t transpose_w, void* stream);
int32_t ssim_linear_wgrad_parts(int64_t rows);
int ssim_linear_wgrad(const float* gy, const float* x, float* gw, float* gb, int64_t rows, int32_t in_dim,
                      int32_t out_dim, float* partial, int32_t parts, void* stream);

/* The Decima MLPs as one fused chain each (make_mlp with two hidden layers: Linear(d0, d1), act, Linear(d1, d2), act,
 * Linear(d2, d3); schedulers/decima/utils.py:51-70): the learner's replacement for 5 forward and ~11 backward
 * per-layer launches. Supported shapes (ssim_mlp3_supported): d0 in 1..64 and (d1, d2, d3, act) = (32, 16, 16,
 * SSIM_ACT_LEAKY_RELU) (the GNN MLPs) or (64, 64, 1, SSIM_ACT_TANH) (the score MLPs); weights in nn.Linear's
 * [out][in] layout. Input: x [rows][d0], or (x == NULL) the exec-score grid scheduler.py:355-367 builds: base
 * [rows / grid_n][d0 - 1] and row r's last column (r % grid_n) / grid_n (the action fraction), so the
 * [decisions * N][d0] input is never materialised.
 * ssim_mlp3_fwd writes y and the post-activation hidden rows h1 [rows][d1], h2 [rows][d2] the backward needs (NULL:
 * inference, not written).
 * ssim_mlp3_bwd: from gy [rows][d3] and h1 / h2, the pre-activation gradients g1 / g2 (scratch [rows][d1] / [rows][d2]),
 * the input gradient gx ([rows][d0]; in grid mode [rows / grid_n][d0 - 1], summed over each decision's actions; NULL:
 * none) and every weight / bias gradient through `partial` (ssim_mlp3_partial_floats floats; parts =
 * ssim_mlp3_parts(rows)), summed in chunk order: deterministic. Returns 0, or -1 for an unsupported shape. */
#define SSIM_ACT_LEAKY_RELU 0
#define SSIM_ACT_TANH 1
int32_t ssim_mlp3_supported(int32_t d0, int32_t d1, int32_t d2, int32_t d3, int32_t act);
int ssim_mlp3_fwd(const float* x, const float* base, int32_t grid_n, const float* w0, const float* b0,
                  const float* w1, const float* b1, const float* w2, const float* b2, float* h1, float* h2, float* y,
                  int64_t rows, int32_t d0, int32_t d1, int32_t d2, int32_t d3, int32_t act, float slope,
                  void* stream);
int32_t ssim_mlp3_parts(int64_t rows);
int64_t ssim_mlp3_partial_floats(int64_t rows, int32_t d0, int32_t d1, int32_t d2, int32_t d3);
int ssim_mlp3_bwd(const float* gy, const float* x, const float* base, int32_t grid_n, const float* w0,
                  const float* w1, const float* w2, const float* h1, const float* h2, float* g1, float* g2, float* gx,
                  float* gw0, float* gb0, float* gw1, float* gb1, float* gw2, float* gb2, int64_t rows, int32_t d0,
                  int32_t d1, int32_t d2, int32_t d3, int32_t act, float slope, float* partial, int32_t parts,
                  void* stream);

/* Continuously discounted returns (trainers/utils/returns_calculator.py:37-52): out[i][k] = r[i][k] + decay[i][k] *
 * out[i][k + 1] (out[i][cols] = 0) for row-major [rows][cols] arrays of doubles (f64 != 0) or floats, with the
 * reference's roundings (product, then sum): bit-identical to its per-column recursion. */
int ssim_discounted_returns(const void* r, const void* decay, void* out, int64_t rows, int64_t cols, int32_t f64,
                            void* stream);

/* Identity of this build: a hash of the library's kernel sources and compile definitions (__graft_entry__.build_lib).
 * bench.py quotes PMC traffic only from a PMC summary (profiles/) made with the same build. */
const char* ssim_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* SPARKSCHED_H */
