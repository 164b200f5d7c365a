// layout.h — byte layout of the per-env state arena, obs arena and reset staging.
// Plain C++ (no HIP), shared by the device library and the test-only host build.
//
// Each env owns one block of the state arena = [hot block | cold block]:
//   hot  — everything the serial event loop touches, as fixed-size records (one 16-byte LDS read brings
//          a whole stage / executor / pool record; ~10 section offsets instead of one per field):
//          header, JobRec[J], JobTimes[J], active-job list, StageRec[S], active-stage and schedulable
//          lists, ExecRec[N], selected list, CommitRec[C], PoolRec[P] (set metadata + the 8-slot table
//          inline). Copied into LDS for the duration of a launch when it fits (`lds_resident`), else
//          used in place in HBM. Identical offsets in LDS and HBM: the engine only swaps the base.
//   cold — HBM only: most_recent_duration per stage (read data-parallel by the observation pass) and the
//          spill area for CPython-set tables that have grown past 8 slots (staged through LDS per use).
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
  int32_t src_idx;        // obs source_job_idx at the last observation
  int32_t err_line;       // engine.h line of the check that raised the first sticky error (diagnostic)
  int32_t commit_hw;      // commitment slots used this episode: every live CommitRec has index < commit_hw
};
static_assert(sizeof(EnvHeader) % 16 == 0, "header must keep 16-B alignment");

// Running sums over observations (SURVEY.md §8d algorithmic-byte accounting), completed decisions and finished
// episodes, kept across resets. Updated in place once per decision, never held in registers. `pending` /
// `pend_t0`: a step preempted between two events of its simulation (ssim_rollout_budget with
// SSIM_ROLLOUT_PREEMPT) and the wall time its reward interval starts at; the next launch completes it.
struct EnvAcc {
  int64_t nodes, edges, jobs, events, decisions, episodes;
  double pend_t0;
  int64_t pending;
};
static_assert(sizeof(EnvAcc) % 16 == 0, "accumulator record");

// One stage (env-global index g = job base + local stage id). `done` is derived: rem + exe + done = tasks,
// so completed <=> rem == 0 && exe == 0.
struct StageRec {
  int16_t job, ts;       // owning job, template-stage index into the dataset
  int16_t rem, exe;      // Stage.num_remaining_tasks / num_executing_tasks (stage.py:5-18)
  int16_t mov, com;      // ExecutorTracker moving-to / commitments-to this stage
  int8_t unmet;          // parents not yet completed (frontier <=> unmet == 0, job.py:93-128)
  uint8_t sel;           // selected in the current round (spark_sched_sim.py:304)
  uint8_t fw_keymask;    // sampler (copied from the dataset at reset): bit l <=> EXEC_LEVELS[l] is a
  uint8_t fw_maxlevel;   //   first_wave key; level index of max(first_wave) (tpch.py:216-235)
};
static_assert(sizeof(StageRec) == 16, "stage record");

struct JobRec {
  int16_t tpl, base, nst, nact;      // template, first env stage, #stages, #active stages
  int16_t sat, local, supply, state; // saturated count, |local_executors|, exec supply, 0/1/2
  int32_t arr_dec, done_dec;         // decision counter at arrival / completion (reward union)
  int32_t pick;  // heuristics find_stage of the job at the last observation (packed min key, engine.h observe)
  int32_t pad;
};
static_assert(sizeof(JobRec) == 32, "job record");

struct JobTimes {
  double tarr, tdone;  // Job.t_arrival / t_completed
};

struct ExecRec {
  int16_t loc, job, task, busy;     // pool code, job (-1 None), last task's local stage (-1 None), executing
  int16_t ev_type, ev_stage;        // pending event (at most one per executor)
  int32_t ev_seq;                   // -1 = no pending event
  double ev_t;
  int64_t pad;
};
static_assert(sizeof(ExecRec) == 32, "executor record");

struct CommitRec {
  int16_t src, dst, cnt, pad;  // ExecutorTracker._commitments[src][dst] = cnt (deleted at 0)
  int32_t ord, pad2;           // dict insertion order stamp
};
static_assert(sizeof(CommitRec) == 16, "commitment record");

// CPython set of one pool: metadata + the table while it has 8 slots (bigger tables spill to the cold block)
struct PoolRec {
  uint16_t mask, fill, used;  // PySetMeta layout (pyset.h)
  int16_t cfrom;              // ExecutorTracker._num_commitments_from[pool]
  uint8_t tab[8];
};
static_assert(sizeof(PoolRec) == 16, "pool record");

constexpr int kNumLevels = 8;  // EXEC_LEVELS (tpch.py:238)
constexpr int kNumAcc = 8;     // int64 accumulators per env in the obs arena (ob_acc)
constexpr int kTraceBytes = 32;
constexpr int64_t kResetHeadBytes = 64;  // ssim_reset_record padded
static_assert(sizeof(ssim_reset_record) <= kResetHeadBytes, "reset record");
constexpr int64_t kLdsBudget = 64 * 1024;    // dynamic LDS per workgroup without opt-in
constexpr int64_t kLdsPerCu = 160 * 1024;     // gfx950 LDS per CU
constexpr int64_t kHbmWorkgroupsPerCu = 16;   // HBM-resident engine kernels: 4 one-wave workgroups per SIMD
// Opt-in dynamic LDS of one workgroup on gfx950 (a CU's 160 KB). The LDS-resident engine kernels use it for batches
// small enough that one env per CU costs nothing (num_envs <= kBigLdsMaxEnvs, one wave per CU), e.g. the 16 envs of a
// decima_tpch.yaml PPO iteration, whose J=200 / N=50 hot block (~146 KB) otherwise stays in HBM.
constexpr int64_t kLdsBudgetBig = 160 * 1024;
constexpr int64_t kBigLdsMaxEnvs = 256;
// Batches past what the LDS-resident kernels hold at once. Those run one wave per SIMD (one env per wave, its hot
// block in LDS: the configs[1] env's 40 KB lets 4 share a CU, 1024 on the chip's 256 CUs); a larger batch waits in
// rounds, while the HBM-resident kernels keep 4 waves per SIMD in flight and hide the memory latency the LDS saves.
// Measured on configs[1]'s env (profiles/r04/env_sweep_residency.log): LDS 3.55e7 decisions/s at every batch size
// from 1024 to 8192 envs; HBM-resident (10, 50)-specialised kernels 1.5e7 at 1024, 4.0e7 at 2048, 5.2e7 at 3072,
// 6.2e7 from 4096. So a batch above 1.5x the LDS-resident concurrency runs HBM-resident.
constexpr int64_t kChipCus = 256;  // a whole MI355X: the default when the device's CU count is not known
constexpr int64_t lds_concurrent_envs(int64_t need, int64_t chip_cus = kChipCus) {
  const int64_t per_cu = kLdsPerCu / (need > 0 ? need : 1);
  return chip_cus * (per_cu < 4 ? per_cu : 4);
}

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

// Section offsets. hot/cold offsets are relative to the start of the hot/cold block; sc_* to the scratch.
// Sections whose size depends only on (N executors, J jobs) come first, then the stage-count (S) ones, so
// a kernel specialised on (N, J) sees compile-time offsets for everything but the few S-dependent sections.
struct StateOffsets {
  int64_t hot_bytes, cold_bytes, scratch_bytes, env_bytes;
  int64_t lds_bytes;        // scratch (+ hot when LDS-resident); decided by compute_layout
  int64_t lds_share;        // LDS per env that keeps the workgroups per CU the residency decision assumed
  int32_t lds_resident, row_of_lds;  // row_of_lds: observe()'s stage -> row map in the LDS scratch (sc_row_of)
  int64_t hdr, acc, jobs, jtimes, active_jobs, execs, sel_list, commits, stages, pools, active_stages,
      sched_list;
  int64_t st_recent /*cold f64[S]*/, pool_tab /*cold uint8 [P][set_cap]*/, row_of /*cold int16[S]*/;
  int64_t sc_execs /*ExecRec[N], HBM-resident step / rollout kernels (Sim ex_lds)*/, sc_keys_a, sc_keys_b /*int32[N+1]*/, sc_plan /*int32[2C]*/, sc_tab_a, sc_tab_b, sc_tab_p /*uint8[set_cap]*/,
      sc_dcache /*uint32[N][24] when N <= kDurCacheMaxExecs*/, sc_bits /*uint32[4]*/, sc_prof /*uint64[64], diagnostic -DSSIM_PROFILE build
      only*/, sc_row_of /*int16[S], last: LDS-resident kernels only*/;
  int64_t scratch_hbm_bytes;  // the scratch without sc_row_of: what an HBM-resident kernel allocates
};

constexpr int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

constexpr int set_cap_for(int n) {  // smallest power of two > 4N (max CPython set table for N keys)
  int c = 8;
  while (c <= 4 * n) c <<= 1;
  return c;
}
constexpr int commit_cap_for(int n) { return 2 * n + 2; }
// Bytes per pool in the cold block's table area: the largest table N executors can need, in slot order (byte s =
// slot s). The device's lane-parallel set operations for 16..127 executors (engine.h "paged tables", up to 512 slots)
// load page g as the 64 bytes at 64g, so an operation reads the table's current size, not its capacity. (Round 5
// stored these tables page-major at a 512-B stride for every N, so each operation fetched 512 B whatever the size.)
constexpr int kPagedTabMax = 512;
constexpr int tab_stride_for(int n) { return set_cap_for(n); }
constexpr int64_t kDurCacheMaxExecs = 16;

// The per-env block layout as a function of (N, J, S). Single source of truth for the host layout and for
// the device engine, which re-derives it with N and J as compile-time constants where it can.
constexpr StateOffsets state_offsets(int64_t N, int64_t J, int64_t S) {
  StateOffsets O{};
  const int64_t P = 1 + J + S, T = set_cap_for((int)N), C = commit_cap_for((int)N), TS = tab_stride_for((int)N);
  int64_t o = 0;
  O.hdr = o;
  o = align16(o + (int64_t)sizeof(EnvHeader));
  O.acc = o;
  o = align16(o + (int64_t)sizeof(EnvAcc));
  O.jobs = o;
  o = align16(o + (int64_t)sizeof(JobRec) * J);
  O.jtimes = o;
  o = align16(o + (int64_t)sizeof(JobTimes) * J);
  O.active_jobs = o;
  o = align16(o + 2 * J);
  O.execs = o;
  o = align16(o + (int64_t)sizeof(ExecRec) * N);
  O.sel_list = o;
  o = align16(o + 2 * (N + 1));
  O.commits = o;
  o = align16(o + (int64_t)sizeof(CommitRec) * C);
  O.stages = o;  // last (N, J)-only offset
  o = align16(o + (int64_t)sizeof(StageRec) * S);
  O.pools = o;
  o = align16(o + (int64_t)sizeof(PoolRec) * P);
  O.active_stages = o;
  o = align16(o + 2 * S);
  O.sched_list = o;
  o = align16(o + 2 * S);
  O.hot_bytes = o;

  int64_t c = 0;
  O.st_recent = c;
  c = align16(c + 8 * S);
  O.pool_tab = c;
  c = align16(c + TS * P);
  O.row_of = c;  // observe()'s stage -> row map of the HBM-resident kernels (their LDS holds only the small scratch)
  c = align16(c + 2 * S);
  O.cold_bytes = c;
  O.env_bytes = O.hot_bytes + O.cold_bytes;

  int64_t s = 0;
  O.sc_execs = s;  // ExecRec[N]: the HBM-resident kernels' LDS copy of the executor records for a launch (Sim ex_lds)
  s = align16(s + (int64_t)sizeof(ExecRec) * N);
  O.sc_keys_a = s;
  s = align16(s + 4 * (N + 1));
  O.sc_keys_b = s;
  s = align16(s + 4 * (N + 1));
  O.sc_plan = s;
  s = align16(s + 8 * C);
  O.sc_tab_a = s;
  s = align16(s + T);
  O.sc_tab_b = s;
  s = align16(s + T);
  O.sc_tab_p = s;
  s = align16(s + T);
  O.sc_dcache = s;  // engine.h duration-descriptor cache (kernels specialised on few executors)
  s = align16(s + (N <= kDurCacheMaxExecs ? 4 * 24 * N : 0));
  O.sc_bits = s;  // uint32[4]: a set's keys as a bitmap over executor ids (paged-table operations)
  s = align16(s + (T > 64 && T <= kPagedTabMax ? 16 : 0));
  O.sc_prof = s;
#ifdef SSIM_PROFILE
  s += 8 * 64;
#endif
  O.scratch_hbm_bytes = align16(s);
  O.sc_row_of = O.scratch_hbm_bytes;
  s = align16(O.sc_row_of + 2 * S);
  O.scratch_bytes = s;
  return O;
}

// Computes the public layout and the private offsets. Returns false on a bad / unsupported config. `chip_cus`: the
// device's compute units (hipDeviceAttributeMultiprocessorCount; a partitioned device or another SKU has fewer), which
// sets how many envs the LDS-resident kernels hold at once and so the batch size above which they run HBM-resident.
inline bool compute_layout(const ssim_config& cfg, ssim_layout* L, StateOffsets* O, int64_t chip_cus = kChipCus) {
  if (cfg.num_envs <= 0 || cfg.num_executors <= 0 || cfg.num_executors > 250 || cfg.job_cap <= 0 ||
      cfg.max_stages <= 0 || cfg.max_stages > 128 /* int8 parent countdown */ || cfg.max_edges < 0 ||
      cfg.trace_cap < 0)
    return false;
  memset(L, 0, sizeof(*L));
  const int64_t B = cfg.num_envs, N = cfg.num_executors, J = cfg.job_cap;
  const int64_t S = J * cfg.max_stages, E = J * (cfg.max_edges > 0 ? cfg.max_edges : 1);
  const int64_t P = 1 + J + S, T = set_cap_for((int)N), C = commit_cap_for((int)N);
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

  *O = state_offsets(N, J, S);
  L->env_bytes = O->env_bytes;
  L->state_bytes = 4096 + L->env_bytes * B;  // params block (engine.h kParamsReserve) + env blocks
  L->scratch_bytes = O->scratch_bytes;
  // LDS per wave: [hot copy (if resident) | scratch]
  const int64_t need = O->hot_bytes + O->scratch_bytes;
  O->lds_resident = (!(cfg.flags & SSIM_CFG_FORCE_HBM) &&
                     ((need <= kLdsBudget && 2 * B <= 3 * lds_concurrent_envs(need, chip_cus)) ||
                      (need <= kLdsBudgetBig && B <= kBigLdsMaxEnvs)))
                        ? 1 : 0;
  L->lds_resident = O->lds_resident;
  // An HBM-resident kernel (4 waves per SIMD: 16 workgroups per CU) whose full scratch would not let 16 workgroups
  // share the CU's LDS keeps the stage -> row map in its cold block instead: 2 B per stage less LDS per wave
  // (configs[3]'s J=200 / N=100 shard: 11 KB -> 4 KB, occupancy 3.5 -> 4 waves per SIMD, +6.5%; the Decima rollout's
  // 9.3 KB fits and keeps the LDS map, profiles/r03/ab_row_of_cold.log).
  O->row_of_lds = (O->lds_resident || O->scratch_bytes * kHbmWorkgroupsPerCu <= kLdsPerCu) ? 1 : 0;
  O->lds_bytes = O->lds_resident ? O->hot_bytes + O->scratch_bytes
                                 : O->row_of_lds ? O->scratch_bytes : O->scratch_hbm_bytes;
  L->lds_bytes = O->lds_bytes;
  // The env's share of its CU's LDS: what may be added on top of lds_bytes (the Decima rollout's policy plan) without
  // lowering the concurrency the residency decision counted on. LDS-resident: up to 4 envs per CU (lds_concurrent_envs);
  // a batch of at most one env per CU may take the whole CU. HBM-resident: 16 one-wave workgroups per CU.
  if (O->lds_resident) {
    const int64_t per_cu = lds_concurrent_envs(need, chip_cus) / (chip_cus > 0 ? chip_cus : 1);
    O->lds_share = B <= chip_cus ? kLdsBudgetBig : kLdsPerCu / (per_cu > 1 ? per_cu : 1);
  } else {
    O->lds_share = kLdsPerCu / kHbmWorkgroupsPerCu;
  }
  L->lds_share = O->lds_share;
  L->chip_cus = chip_cus;

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
  L->ob_acc = otake(B * kNumAcc * 8);
  L->ob_trace = otake(B * (int64_t)cfg.trace_cap * kTraceBytes);
  L->obs_bytes = align16(b);

  L->reset_stride = align16(kResetHeadBytes + 8 * J + 4 * J);
  L->reset_bytes = L->reset_stride * B;
  return true;
}

}  // namespace ssim
