// layout.h — byte layout of the per-env state arena, obs arena and reset staging.
// Plain C++ (no HIP), shared by the device library and the test-only host build.
#pragma once
#include <stdint.h>
#include <string.h>

#include "sparksched.h"

namespace ssim {

// Per-env scalar header (first bytes of an env block). Loaded into registers at the start of a step and
// stored back at the end.
struct EnvHeader {
  double wall;            // spark_sched_sim.py:60 wall_time
  double time_limit;      // StochasticTimeLimit limit (+inf = none)
  uint64_t rng_s_hi, rng_s_lo, rng_i_hi, rng_i_lo;  // numpy PCG64
  uint32_t rng_has32, rng_u32;
  int32_t num_jobs;       // len(self.jobs) of this episode
  int32_t arrivals;       // JOB_ARRIVAL events popped so far (= next job to arrive)
  int32_t seq;            // EventQueue tie-break counter (event.py:25-29)
  int32_t n_active_jobs;  // len(active_job_ids)
  int32_t n_active_stages;
  int32_t n_completed;
  int32_t source;         // pool code of ExecutorTracker._curr_source
  int32_t commit_seq;     // insertion-order stamp for commitment dict entries
  int32_t supply_none;    // ExecutorTracker._total_executor_count[None]
  int32_t n_sched;        // len(schedulable_stages) at the last observation
  int32_t n_selected;     // len(selected_stages)
  int32_t decisions;      // successful env.step calls this episode
  int32_t events;         // events popped this episode
  int32_t terminated;
  uint32_t err;           // sticky error bits (SSIM_ERR_STICKY)
  int32_t stage_idx_n;    // action_space["stage_idx"].n
  int32_t episode;
  int32_t trace_len;
  int32_t step_events;
  int32_t pad[3];
  // running sums over observations (SURVEY.md §8d algorithmic-byte accounting)
  int64_t acc_nodes, acc_edges, acc_jobs, acc_events;
};
static_assert(sizeof(EnvHeader) % 16 == 0, "header must keep 16-B alignment");

constexpr int kNumLevels = 8;  // EXEC_LEVELS (tpch.py:238)
constexpr int kTraceBytes = 32;
constexpr int64_t kResetHeadBytes = 64;  // ssim_reset_record padded
static_assert(sizeof(ssim_reset_record) <= kResetHeadBytes, "reset record");

struct TraceRec {  // one popped event
  double t;
  int32_t kind;   // 1 arrival, 2 task finished, 3 executor ready, 4 job completed
  int32_t exec;   // executor id or -1
  int32_t job;
  int32_t stage;  // local stage id or -1
  int32_t seq;
  int32_t pad;
};
static_assert(sizeof(TraceRec) == kTraceBytes, "trace record size");

// Offsets of every per-env state field (bytes from the env block start) + scratch offsets.
struct StateOffsets {
  int64_t hdr;
  int64_t job_tpl, job_base, job_nst, job_nact, job_sat, job_local, job_supply, job_state, job_arr_dec,
      job_done_dec, job_tarr, job_tdone, active_jobs;
  int64_t st_job, st_ts, st_rem, st_exe, st_done, st_mov, st_com, st_unmet, st_sel, st_recent,
      active_stages, sched_list;
  int64_t ex_loc, ex_job, ex_task, ex_busy, ev_t, ev_seq, ev_type, ev_stage, sel_list;
  int64_t cm_src, cm_dst, cm_cnt, cm_ord;
  int64_t pool_meta, pool_cfrom, pool_tab;
  // scratch (LDS on device): offsets within one env's scratch block
  int64_t sc_row_of, sc_keys_a, sc_keys_b, sc_plan, sc_tab_a, sc_tab_b;
};

inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

inline int set_cap_for(int n) {  // smallest power of two > 4N (max CPython set table for N keys)
  int c = 8;
  while (c <= 4 * n) c <<= 1;
  return c;
}

// Computes the public layout and the private state offsets. Returns false on bad config.
inline bool compute_layout(const ssim_config& cfg, ssim_layout* L, StateOffsets* O) {
  if (cfg.num_envs <= 0 || cfg.num_executors <= 0 || cfg.num_executors > 250 || cfg.job_cap <= 0 ||
      cfg.max_stages <= 0 || cfg.max_edges < 0 || cfg.trace_cap < 0)
    return false;
  memset(L, 0, sizeof(*L));
  memset(O, 0, sizeof(*O));
  const int64_t B = cfg.num_envs, N = cfg.num_executors, J = cfg.job_cap;
  const int64_t S = J * cfg.max_stages, E = J * (cfg.max_edges > 0 ? cfg.max_edges : 1);
  const int64_t P = 1 + J + S, T = set_cap_for((int)N), C = 2 * N + 2;
  L->num_envs = (int32_t)B;
  L->num_executors = (int32_t)N;
  L->job_cap = (int32_t)J;
  L->stage_cap = (int32_t)S;
  L->edge_cap = (int32_t)E;
  L->pool_cap = (int32_t)P;
  L->set_cap = (int32_t)T;
  L->commit_cap = (int32_t)C;
  L->trace_cap = cfg.trace_cap;

  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o = align16(o + bytes);
    return r;
  };
  O->hdr = take(sizeof(EnvHeader));
  O->job_tpl = take(4 * J);
  O->job_base = take(4 * J);
  O->job_nst = take(4 * J);
  O->job_nact = take(4 * J);
  O->job_sat = take(4 * J);
  O->job_local = take(4 * J);
  O->job_supply = take(4 * J);
  O->job_state = take(4 * J);
  O->job_arr_dec = take(4 * J);
  O->job_done_dec = take(4 * J);
  O->job_tarr = take(8 * J);
  O->job_tdone = take(8 * J);
  O->active_jobs = take(4 * J);
  O->st_job = take(4 * S);
  O->st_ts = take(4 * S);
  O->st_rem = take(4 * S);
  O->st_exe = take(4 * S);
  O->st_done = take(4 * S);
  O->st_mov = take(4 * S);
  O->st_com = take(4 * S);
  O->st_unmet = take(4 * S);
  O->st_sel = take(4 * S);
  O->st_recent = take(8 * S);
  O->active_stages = take(4 * S);
  O->sched_list = take(4 * S);
  O->ex_loc = take(4 * N);
  O->ex_job = take(4 * N);
  O->ex_task = take(4 * N);
  O->ex_busy = take(4 * N);
  O->ev_t = take(8 * N);
  O->ev_seq = take(4 * N);
  O->ev_type = take(4 * N);
  O->ev_stage = take(4 * N);
  O->sel_list = take(4 * (N + 1));
  O->cm_src = take(4 * C);
  O->cm_dst = take(4 * C);
  O->cm_cnt = take(4 * C);
  O->cm_ord = take(4 * C);
  O->pool_meta = take(8 * P);
  O->pool_cfrom = take(4 * P);
  O->pool_tab = take(T * P);
  L->env_bytes = align16(o);
  L->state_bytes = 4096 + L->env_bytes * B;  // params block (engine.h kParamsReserve) + env blocks

  // scratch block per env (LDS on device)
  int64_t s = 0;
  auto stake = [&](int64_t bytes) {
    int64_t r = s;
    s = align16(s + bytes);
    return r;
  };
  O->sc_row_of = stake(4 * S);
  O->sc_keys_a = stake(4 * (N + 1));
  O->sc_keys_b = stake(4 * (N + 1));
  O->sc_plan = stake(8 * C);
  O->sc_tab_a = stake(T);
  O->sc_tab_b = stake(T);
  L->scratch_bytes = align16(s);

  // obs arena: each field is [B][per-env]
  int64_t b = 0;
  auto otake = [&](int64_t bytes) {
    int64_t r = b;
    b = align16(b + bytes);
    return r;
  };
  L->ob_nodes = otake(B * S * 3 * 4);
  L->ob_edge_links = otake(B * E * 2 * 8);
  L->ob_dag_ptr = otake(B * (J + 1) * 4);
  L->ob_supplies = otake(B * J * 4);
  L->ob_frontier = otake(B * S);
  L->ob_sched_rank = otake(B * S * 4);
  L->ob_counts = otake(B * SSIM_NUM_COUNTS * 4);
  L->ob_reward = otake(B * 8);
  L->ob_wall_time = otake(B * 8);
  L->ob_acc = otake(B * 4 * 8);
  L->ob_trace = otake(B * (int64_t)cfg.trace_cap * kTraceBytes);
  L->obs_bytes = align16(b);

  L->reset_stride = align16(kResetHeadBytes + 8 * J + 4 * J);
  L->reset_bytes = L->reset_stride * B;
  return true;
}

}  // namespace ssim
