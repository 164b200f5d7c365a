// layout.h — byte layout of the per-env state arena, obs arena and reset staging.
// Plain C++ (no HIP), shared by the device library and the test-only host build.
//
// Each env owns one block of the state arena = [hot block | cold block]:
//   hot  — everything the serial event loop touches (header, jobs, compact stage counters, executors,
//          commitments, pool metadata). Copied into LDS for the duration of a launch when it fits
//          (hot_bytes + scratch_bytes <= the per-workgroup LDS budget), else used in place in HBM.
//          Identical offsets in LDS and HBM, so the engine only swaps the base pointer.
//   cold — HBM only: the CPython-set tables of all pools (staged through LDS per set operation) and
//          most_recent_duration (read data-parallel by the observation pass).
#pragma once
#include <stdint.h>
#include <string.h>

#include "sparksched.h"

namespace ssim {

// Per-env scalar header (first bytes of the hot block). Loaded into registers at the start of a step and
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
constexpr int64_t kLdsBudget = 64 * 1024;  // dynamic LDS per workgroup without opt-in

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

// Field offsets. hot/cold offsets are relative to the start of the hot/cold block; sc_* to the scratch.
struct StateOffsets {
  int64_t hot_bytes, cold_bytes, lds_bytes;  // lds_bytes = hot + scratch when LDS-resident, else scratch
  int32_t lds_resident, pad;
  // hot: header, jobs (int16 unless noted), stages (int16), executors, commitments, pools
  int64_t hdr;
  int64_t job_tpl, job_base, job_nst, job_nact, job_sat, job_local, job_supply, job_state;
  int64_t job_arr_dec, job_done_dec;  // int32
  int64_t job_tarr, job_tdone;        // float64
  int64_t active_jobs;
  int64_t st_job, st_ts, st_rem, st_exe, st_mov, st_com, st_unmet, st_sel /*uint8*/, active_stages, sched_list;
  int64_t ex_loc, ex_job, ex_task, ex_busy, ev_type, ev_stage; /*int16*/
  int64_t ev_seq /*int32*/, ev_t /*float64*/, sel_list;
  int64_t cm_src, cm_dst, cm_cnt /*int16*/, cm_ord /*int32*/;
  int64_t pool_meta /*PySetMeta*/, pool_cfrom /*int16*/;
  // cold
  int64_t st_recent /*float64*/, pool_tab /*uint8 [P][set_cap]*/;
  // scratch (LDS)
  int64_t sc_row_of /*int16*/, sc_keys_a, sc_keys_b /*int32*/, sc_plan /*int32*/, sc_tab_a, sc_tab_b, sc_tab_p;
};

inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

inline int set_cap_for(int n) {  // smallest power of two > 4N (max CPython set table for N keys)
  int c = 8;
  while (c <= 4 * n) c <<= 1;
  return c;
}

// Computes the public layout and the private offsets. Returns false on a bad / unsupported config.
inline bool compute_layout(const ssim_config& cfg, ssim_layout* L, StateOffsets* O) {
  if (cfg.num_envs <= 0 || cfg.num_executors <= 0 || cfg.num_executors > 250 || cfg.job_cap <= 0 ||
      cfg.max_stages <= 0 || cfg.max_stages > 255 || cfg.max_edges < 0 || cfg.trace_cap < 0)
    return false;
  memset(L, 0, sizeof(*L));
  memset(O, 0, sizeof(*O));
  const int64_t B = cfg.num_envs, N = cfg.num_executors, J = cfg.job_cap;
  const int64_t S = J * cfg.max_stages, E = J * (cfg.max_edges > 0 ? cfg.max_edges : 1);
  const int64_t P = 1 + J + S, T = set_cap_for((int)N), C = 2 * N + 2;
  if (P >= 32767) return false;  // pool codes and stage indices are int16 in the hot block
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
  O->job_tpl = take(2 * J);
  O->job_base = take(2 * J);
  O->job_nst = take(2 * J);
  O->job_nact = take(2 * J);
  O->job_sat = take(2 * J);
  O->job_local = take(2 * J);
  O->job_supply = take(2 * J);
  O->job_state = take(2 * J);
  O->active_jobs = take(2 * J);
  O->job_arr_dec = take(4 * J);
  O->job_done_dec = take(4 * J);
  O->job_tarr = take(8 * J);
  O->job_tdone = take(8 * J);
  O->st_job = take(2 * S);
  O->st_ts = take(2 * S);
  O->st_rem = take(2 * S);
  O->st_exe = take(2 * S);
  O->st_mov = take(2 * S);
  O->st_com = take(2 * S);
  O->st_unmet = take(2 * S);
  O->st_sel = take(S);
  O->active_stages = take(2 * S);
  O->sched_list = take(2 * S);
  O->ex_loc = take(2 * N);
  O->ex_job = take(2 * N);
  O->ex_task = take(2 * N);
  O->ex_busy = take(2 * N);
  O->ev_type = take(2 * N);
  O->ev_stage = take(2 * N);
  O->ev_seq = take(4 * N);
  O->ev_t = take(8 * N);
  O->sel_list = take(2 * (N + 1));
  O->cm_src = take(2 * C);
  O->cm_dst = take(2 * C);
  O->cm_cnt = take(2 * C);
  O->cm_ord = take(4 * C);
  O->pool_meta = take(6 * P);
  O->pool_cfrom = take(2 * P);
  O->hot_bytes = align16(o);

  int64_t c = 0;
  auto ctake = [&](int64_t bytes) {
    int64_t r = c;
    c = align16(c + bytes);
    return r;
  };
  O->st_recent = ctake(8 * S);
  O->pool_tab = ctake(T * P);
  O->cold_bytes = align16(c);
  L->env_bytes = O->hot_bytes + O->cold_bytes;
  L->state_bytes = 4096 + L->env_bytes * B;  // params block (engine.h kParamsReserve) + env blocks

  // scratch block per env (LDS)
  int64_t s = 0;
  auto stake = [&](int64_t bytes) {
    int64_t r = s;
    s = align16(s + bytes);
    return r;
  };
  O->sc_row_of = stake(2 * S);
  O->sc_keys_a = stake(4 * (N + 1));
  O->sc_keys_b = stake(4 * (N + 1));
  O->sc_plan = stake(8 * C);
  O->sc_tab_a = stake(T);
  O->sc_tab_b = stake(T);
  O->sc_tab_p = stake(T);
  L->scratch_bytes = align16(s);
  O->lds_resident = (O->hot_bytes + L->scratch_bytes <= kLdsBudget) ? 1 : 0;
  O->lds_bytes = L->scratch_bytes + (O->lds_resident ? O->hot_bytes : 0);

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
