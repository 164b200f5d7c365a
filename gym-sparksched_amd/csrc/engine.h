// engine.h — the batched Spark-scheduling simulation step, one wavefront per env.
//
// Restates the hot path of spark_sched_sim/spark_sched_sim.py (reset 127-186, step 188-221, the event
// loop 320-343, handlers 428-483, helpers 487-874), components/executor_tracker.py and
// data_samplers/tpch.py:75-106 on device-resident structure-of-arrays state (layout.h).
//
// Execution model. Control flow is wave-uniform: every lane of the env's wavefront executes the serial
// part of the algorithm with identical values, so branches never diverge and same-address loads are
// broadcast. Data-parallel parts run across lanes through the W policy: the schedulable-stage scan
// (ballot + first-set-lane), executor event-slot argmin (min-reduce), observation rows and edges
// (ballot/prefix compaction, coalesced stores), pool-table staging. W is WaveHip on device
// (sparksched.hip); the test-only host build (tests/hostsim/) instantiates the same template with a
// one-lane W to debug the logic on CPU.
//
// Memory. The serial event loop is latency bound, so the env's hot block (header, jobs, compact stage
// counters, executors, commitments, pool metadata) is copied into LDS for the launch when it fits
// (`lds_resident`), and CPython-set tables are staged through LDS one pool at a time; HBM sees bulk
// coalesced copies, the obs stores and the read-only dataset gathers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "layout.h"
#include "pcg64.h"
#include "pyset.h"

// Diagnostic build only (-DSSIM_PROFILE, scripts/phase_profile.py): per-phase shader-clock sums per wave, kept in
// a small LDS area of the wave's scratch block (StateOffsets::sc_prof) and added to by lane 0 with no-return LDS
// atomics, so a timer costs no register array (no scratch memory) and no dependent round trip.
#ifdef SSIM_PROFILE
#define SSIM_TIC(v) const uint64_t v = W::clock()
#define SSIM_TOC(v, ph) prof_add(ph, W::clock() - (v))
#else
#define SSIM_TIC(v) (void)0
#define SSIM_TOC(v, ph) (void)0
#endif

// Diagnostic ISA-reading build only (-DSSIM_MARKERS): named asm comments delimit code regions in the .s output.
#ifdef SSIM_MARKERS
#define SSIM_MARK(name) asm volatile("; SSIM_MARK " name)
#else
#define SSIM_MARK(name) (void)0
#endif

// No floating-point contraction anywhere in the engine: the reference's float64 arithmetic rounds every product
// before the add (e.g. job arrivals t += exponential(1 / rate) = t + round(scale * e), tpch.py:70), and a fused
// multiply-add would change the last bit of the times the parity checks compare bit for bit.
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace ssim {

// Test-only wave types (the set KAT's known-bad variant, tests/test_gpu_sets.py) declare kKatBadPage = true; the paged
// set code then reproduces the effect of the ROCm 7.2 miscompile it works around (Sim::paged_set), so the KAT can be
// shown to catch it. Every shipped wave type leaves it undeclared (false).
template <class W, class = void>
struct KatBadPage {
  static constexpr bool value = false;
};
template <class W>
struct KatBadPage<W, decltype((void)W::kKatBadPage)> {
  static constexpr bool value = W::kKatBadPage;
};

// Dataset pointers are loaded from the Params block, so the compiler sees generic pointers and would emit
// FLAT loads; the cast to the global address space turns them into global_load (test host build: no-op).
#if defined(__HIP_DEVICE_COMPILE__)
#define SSIM_GLOBAL __attribute__((address_space(1)))
#else
#define SSIM_GLOBAL
#endif
template <class T>
__device__ __forceinline__ T ldg(const T* p, int64_t i) {
  return ((const SSIM_GLOBAL T*)p)[i];
}

// top-level phases (disjoint) then inclusive sub-timers (nested inside the top-level ones)
enum : int32_t { kPhPolicy = 0, kPhAction, kPhRoundCheck, kPhFulfill, kPhPop, kPhHandle, kPhPostScan, kPhObserve,
                 kPhSample, kPhPool, kPhScan, kPhLoadSave, kPhPoolBig, kPhIdleOrder, kPhDraw, kPhJobArr,
                 kPhExecArr, kPhTaskDone, kPhStageDone,
                 // whole loop iterations of the rollout (policy + step, or completing a pending step, or an auto-reset)
                 kPhIter,
                 // event counters (not cycles)
                 kCtPoolSmall, kCtPoolBig, kCtTask, kCtIdleOrder,
                 // histogram of whole-decision cycles (policy + step + auto-reset): bucket b = [2^(b+10), 2^(b+11))
                 kHist0,
                 // s_memrealtime stamps (100 MHz chip clock): wave entry, hot block loaded, loop exit, hot block saved, engine
                 // constructed, fixed sections copied
                 kTEntry = kHist0 + 16, kTLoaded, kTLoopEnd, kTSaved, kTCtor, kTCopy1,
                 // the persistent Decima rollout's action driver (decima_rollout.h): features, fused policy, sample copy
                 kPhDecFeat, kPhDecPolicy, kPhDecRecord,
                 // decima_policy_env's parts (setup, prep, message passing, summaries, stage scores, then sums of the
                 // observation sizes n, ne, levels, schedulable, then exec scores)
                 kPhDecParts,
                 // in-launch auto-resets (rollout_body): cycles, count
                 kPhReset = kPhDecParts + 10, kCtReset, kNumPhases };
#ifdef SSIM_PROFILE
#define SSIM_COUNT(ph) prof_add(ph, 1)
#else
#define SSIM_COUNT(ph) (void)0
#endif
// Diagnostic host build only (scripts/pool_stats.py): a hook per CPython-set operation (op, table size, keys).
#ifndef SSIM_POOL_STAT
#define SSIM_POOL_STAT(op, size, used) (void)0
#endif
// Diagnostic host build only (scripts/field_stats.py): a hook per wave-uniform read of a hot-block field or record, by
// section (0 stage field, 1 job field, 2 job times, 3 executor field, 4 executor event field, 5 pool cfrom, 6 stage
// recent duration, 10 pool record, 11 stage record, 12 executor record, 13 commitment scan step).
#ifndef SSIM_FIELD_STAT
#define SSIM_FIELD_STAT(sec) (void)0
#endif
enum : int32_t { kPoolNone = -1, kPoolCommon = 0 };
// trace-only kinds: a job completion (:682-697) and an executor released to the common pool (:779-782, the
// reference's Executor.add_history(wall, -1)); with the kEvReady records they give the render history.
enum : int32_t { kEvArrival = 1, kEvTask = 2, kEvReady = 3, kTrJobDone = 4, kTrToCommon = 5 };
enum : int32_t { kJobPending = 0, kJobActive = 1, kJobDone = 2 };
enum : int32_t { kScanAll = 0, kScanOnly = 1, kScanExcept = 2 };

struct StepIn {
  int32_t stage_idx, num_exec;
};

// Preemption policy of a step's simulation (Sim::simulate): `issue()` starts the (asynchronous) read of the stop
// condition, `hit(v)` tests a value issued one event earlier, so the read's latency overlaps an event's work.
// NoStop: steps always run to completion (every launch but the preemptible budget rollout).
struct NoStop {
  static constexpr bool kCan = false;
  __device__ __forceinline__ uint64_t issue() const { return 0; }
  __device__ __forceinline__ bool hit(uint64_t) const { return false; }
};
enum : int32_t { kSimIdle = 0, kSimDecision = 1, kSimPreempted = 2 };

// The launch constants the event loop reads (dataset pointers, config scalars, obs-arena offsets), filled on the
// host by fill_hot_params. On device each lane of one VGPR holds one dword (Sim::hpv) and a field read is a
// v_readlane with a constant lane: with the register pressure of the serial state machine the compiler otherwise
// re-reads Params fields with scalar loads whose latency the loop then waits on, once per event.
struct HotParams {
  const int32_t* tpl_stage_base;
  const int32_t* ts_num_tasks;
  const double* ts_rough;
  const int32_t* ts_child_base;
  const int32_t* ts_children;
  const int32_t* ts_parent_base;
  const int32_t* ts_parents;
  const int32_t* ts_fw_keymask;
  const int32_t* ts_fw_maxlevel;
  const int32_t* dur_off;
  const int32_t* dur_len;
  const double* durations;
  const uint64_t* ts_topo;
  double moving_delay, warmup_delay, beta, job_arrival_gap;
  int64_t ob_nodes, ob_edge_links, ob_dag_ptr, ob_supplies, ob_frontier, ob_sched_rank, ob_counts, ob_reward,
      ob_wall_time, ob_acc, ob_trace;
  int32_t num_templates, trace_cap, edge_cap, job_arrival_cap, topo;
  int32_t dcache;  // 1: every duration list fits the packed descriptor cache (len <= 255, offset < 2^24)
};
static_assert(sizeof(HotParams) <= 256 && sizeof(HotParams) % 8 == 0, "one dword per lane of one VGPR");

// Everything a launch needs besides the arenas. Lives at the start of the state arena (device memory),
// so kernels take one pointer and read fields through the scalar cache.
// Executor-key table per number of local executors n (tpch.py:216-235 on executor_intervals, tpch.py:237-262):
// {lo, hi, level(lo), level(hi)} — the interval's EXEC_LEVELS values (small integers) and their indices, so
// the sampler's key choice is scalar-cache reads instead of two dependent dataset loads.
constexpr int kIvRows = 256;
struct Params {
  HotParams hp;  // (first: 16-B aligned at the start of the state arena)
  ssim_layout L;
  StateOffsets O;
  ssim_dataset D;
  ssim_config C;
  uint8_t iv[kIvRows][4];
};
constexpr int64_t kParamsReserve = 4096;
// The last 2 KB of the params block hold the shared-budget rollouts' state (ssim_rollout_budget): two slots used
// alternately, each one 64-B line for the decision counter followed by kStopLines lines of the "budget spent" flag
// (env e polls line e % kStopLines, one per XCD under round-robin workgroup dispatch).
constexpr int kStopLines = 8;
constexpr int64_t kTicketOffset = kParamsReserve - 2048;
constexpr int64_t kTicketStride = 64;
constexpr int64_t kTicketSlotBytes = (1 + kStopLines) * kTicketStride;
static_assert(sizeof(Params) <= kTicketOffset, "params block");

__host__ __device__ inline int exec_level_index(double key) {  // EXEC_LEVELS index, 0xFF if not a level
  return key == 5.0 ? 0 : key == 10.0 ? 1 : key == 20.0 ? 2 : key == 40.0 ? 3 : key == 50.0 ? 4
         : key == 60.0 ? 5 : key == 80.0 ? 6 : key == 100.0 ? 7 : 0xFF;
}

// Host side: fill Params::iv from the packed executor_intervals table ((N+1) x 2 float64, host memory).
// Returns false if a value is not a small integer (the table's values are EXEC_LEVELS members).
inline bool fill_interval_table(Params* p, const double* intervals, int num_executors) {
  memset(p->iv, 0, sizeof(p->iv));
  for (int n = 0; n <= num_executors && n < kIvRows; ++n) {
    const double lo = intervals[2 * n], hi = intervals[2 * n + 1];
    if (!(lo >= 0 && lo <= 255 && hi >= 0 && hi <= 255 && lo == (double)(int)lo && hi == (double)(int)hi))
      return false;
    p->iv[n][0] = (uint8_t)lo;
    p->iv[n][1] = (uint8_t)hi;
    p->iv[n][2] = (uint8_t)exec_level_index(lo);
    p->iv[n][3] = (uint8_t)exec_level_index(hi);
  }
  return true;
}

// Host side: Params::hp from the layout, dataset and config already in *p.
inline void fill_hot_params(Params* p) {
  HotParams& h = p->hp;
  const ssim_dataset& D = p->D;
  h.tpl_stage_base = D.tpl_stage_base;
  h.ts_num_tasks = D.ts_num_tasks;
  h.ts_rough = D.ts_rough;
  h.ts_child_base = D.ts_child_base;
  h.ts_children = D.ts_children;
  h.ts_parent_base = D.ts_parent_base;
  h.ts_parents = D.ts_parents;
  h.ts_fw_keymask = D.ts_fw_keymask;
  h.ts_fw_maxlevel = D.ts_fw_maxlevel;
  h.dur_off = D.dur_off;
  h.dur_len = D.dur_len;
  h.durations = D.durations;
  h.ts_topo = D.ts_topo;
  h.moving_delay = p->C.moving_delay;
  h.warmup_delay = p->C.warmup_delay;
  h.beta = p->C.beta;
  h.job_arrival_gap = p->C.job_arrival_gap;
  const ssim_layout& L = p->L;
  h.ob_nodes = L.ob_nodes;
  h.ob_edge_links = L.ob_edge_links;
  h.ob_dag_ptr = L.ob_dag_ptr;
  h.ob_supplies = L.ob_supplies;
  h.ob_frontier = L.ob_frontier;
  h.ob_sched_rank = L.ob_sched_rank;
  h.ob_counts = L.ob_counts;
  h.ob_reward = L.ob_reward;
  h.ob_wall_time = L.ob_wall_time;
  h.ob_acc = L.ob_acc;
  h.ob_trace = L.ob_trace;
  h.num_templates = D.num_templates;
  h.trace_cap = L.trace_cap;
  h.edge_cap = L.edge_cap;
  h.job_arrival_cap = p->C.job_arrival_cap;
  h.topo = (p->C.max_stages <= 32 && D.ts_topo != nullptr) ? 1 : 0;
  h.dcache = 0;  // set by the host once it has checked the dataset's descriptors (dcache_fits)
}

// kN / kJ / kS: executor count, job cap and stage cap as compile-time constants (0 = read from the layout at
// run time). A fully specialised instantiation sees every section offset (hot block, scratch), loop bound
// and table size as a constant, so LDS accesses use immediate offsets and no SGPRs hold offsets.
template <class W, int kN = 0, int kJ = 0, int kS = 0>
struct Sim {
  using WT = W;
  const ssim_layout& L;
  const ssim_dataset& D;
  const ssim_config& C;
  const uint8_t (*IV)[4];    // Params::iv
  const int32_t NE, JC, SC;  // executors, job cap, stage cap
  const StateOffsets O;      // re-derived from (NE, JC, SC): the layout (same function as the host layout); scratch too
  uint8_t* ghot;  // this env's hot block in HBM
  uint8_t* hot;   // working copy of the hot block (LDS when resident, else == ghot)
  uint8_t* cold;  // this env's cold block in HBM
  uint8_t* scr;   // this env's scratch block (LDS)
  uint8_t* obs;   // obs arena base
  int32_t eid;    // env index
  bool res;       // hot block LDS-resident
  bool row_lds;   // observe()'s stage -> row map in the LDS scratch (else in the cold block; StateOffsets::row_of_lds)
  // ex_lds (HBM-resident step / rollout launches): the executor records live in the wave's LDS scratch (sc_execs) for
  // the launch — copied in by load_hot, back by save_hot — so their field reads (~40 per decision at N = 100) are LDS
  // round trips instead of global loads queued behind the wave's earlier stores (vmcnt counts loads and stores in
  // issue order), and their lines are not re-fetched from HBM every decision.
  bool ex_l;
  uint8_t* xb;    // ExecRec[0]: hot + O.execs, or the LDS copy
  EnvHeader h;    // register copy of the header
  Pcg64 rng;
  uint32_t iv_lane;  // Params::iv row `lane` (device: read with v_readlane instead of a scalar-cache load)
  // Executor event slots in registers (device waves): lane l of page p holds executor 64p + l's pending event, a
  // write-through copy of the ExecRec fields ev_t / ev_seq / ev_type / ev_stage (the hot block stays authoritative
  // for lane-parallel readers and across launches). The event pop then reads no memory: a DPP min over registers
  // instead of a reload of every executor record per event (an LDS round trip on the resident kernels, HBM lines on
  // the HBM-resident ones). Pages: the executor count's when it is a compile-time constant, else
  // SSIM_EV_PAGES_GENERIC (per translation unit: 2 = up to 128 executors in k_hbm.hip, 1 in k_lds.hip, where two
  // pages crash the ROCm 7.2 register allocator); more executors fall back to the record reads.
#ifndef SSIM_EV_PAGES_GENERIC
#define SSIM_EV_PAGES_GENERIC 1
#endif
#ifndef SSIM_DUR_CACHE
#define SSIM_DUR_CACHE 1
#endif
  static constexpr int kEvPages = W::kWidth == 64 ? (kN > 0 ? (kN + 63) / 64 : SSIM_EV_PAGES_GENERIC) : 0;
  struct EvRegs {
    uint32_t tlo, thi;  // ev_t bits (+inf: no event)
    int32_t seq;        // -1: no event
    int32_t ts;         // ev_type << 16 | (uint16) ev_stage
  };
  EvRegs evr[kEvPages > 0 ? kEvPages : 1];
  __device__ __forceinline__ bool ev_in_regs() const { return kEvPages > 0 && NE <= 64 * kEvPages; }
  // Duration-descriptor cache (kernels specialised on <= 16 executors): per executor, the (wave x exec-level)
  // duration-list descriptors of the stage its current task runs on (24 lanes x {len, off}, as dur_gather) in the
  // wave's LDS scratch (StateOffsets::sc_dcache). A task completion whose stage has tasks left runs the next task on
  // the same stage (spark_sched_sim.py:466-470), so the pop reads its descriptors from LDS together with the stage and
  // executor records instead of issuing the dataset gather whose latency the draw then waits on. Filled at every other
  // task start (run_next_task) and for the pending tasks when a launch starts (ev_regs_load). (Kept in LDS: as a
  // register array in the Sim object it pushed the whole object into scratch memory.)
  static constexpr bool kDurCache = W::kWidth == 64 && kN > 0 && kN <= kDurCacheMaxExecs && SSIM_DUR_CACHE;
  bool dcache_on = false;  // kDurCache and the dataset's descriptors fit the packed form (HotParams::dcache)
  __device__ __forceinline__ bool dc_on() const { return kDurCache && dcache_on; }
  const HotParams* HPp;  // host build: Params::hp read in place
  uint32_t hpv;          // device: dword `lane` of Params::hp
#ifdef SSIM_PROFILE
  uint64_t* prof;  // LDS: kNumPhases sums of this wave (lane 0 adds)
  __device__ __forceinline__ void prof_add(int ph, uint64_t v) {
    if (W::lane() == 0) W::lds_add_u64(prof + ph, v);
  }
  __device__ __forceinline__ void prof_set(int ph, uint64_t v) {
    W::sync();
    if (W::lane() == 0) prof[ph] = v;
    W::sync();
  }
#endif

  // `lds` = this wave's LDS block: [hot copy (if resident) | scratch]; resident=false keeps hot in HBM.
  // row_cold: observe()'s stage -> row map in the cold block whatever the layout says (a kernel that gives the LDS the
  // layout left for it to something else: the persistent Decima rollout's policy plan).
  __device__ __forceinline__ Sim(const Params* __restrict__ p, uint8_t* state_arena, uint8_t* lds,
                                 uint8_t* obs_arena, int32_t env_index, bool resident, bool row_cold = false,
                                 bool ex_lds = false)
      : L(p->L), D(p->D), C(p->C), IV(p->iv), NE(kN ? kN : p->L.num_executors), JC(kJ ? kJ : p->L.job_cap),
        SC(kS ? kS : p->L.stage_cap), O(state_offsets(NE, JC, SC)),
        ghot(state_arena + kParamsReserve + (int64_t)env_index * O.env_bytes),
        hot(resident ? lds : state_arena + kParamsReserve + (int64_t)env_index * O.env_bytes),
        cold(state_arena + kParamsReserve + (int64_t)env_index * O.env_bytes + O.hot_bytes),
        scr(resident ? lds + O.hot_bytes : lds), obs(obs_arena), eid(env_index), res(resident),
        row_lds(resident || (!row_cold && W::uni(p->O.row_of_lds) != 0)), ex_l(ex_lds && !resident),
        xb(ex_lds && !resident ? lds + O.sc_execs : hot + O.execs) {
    iv_lane = W::lane() < kIvRows ? *reinterpret_cast<const uint32_t*>(IV[W::lane()]) : 0u;
    dcache_on = kDurCache && W::uni(p->hp.dcache) != 0;
    HPp = &p->hp;
    hpv = (W::kWidth == 64 && W::lane() < (int)(sizeof(HotParams) / 4)) ? reinterpret_cast<const uint32_t*>(&p->hp)[W::lane()]
                                                                      : 0u;
#ifdef SSIM_PROFILE
    prof = reinterpret_cast<uint64_t*>(scr + O.sc_prof);
    for (int i = W::lane(); i < kNumPhases; i += W::kWidth) prof[i] = 0;
    W::sync();
#endif
  }
  // A HotParams field: v_readlane of hpv on device (constant lanes), the field itself in the host build.
  template <class T, int kOff>
  __device__ __forceinline__ T hp_get(const T& host_val) const {
    if constexpr (W::kWidth == 64) {
      static_assert(kOff % 4 == 0, "dword fields");
      if constexpr (sizeof(T) == 8) {
        const uint32_t lo = (uint32_t)W::bcast_i((int)hpv, kOff / 4);
        const uint32_t hi = (uint32_t)W::bcast_i((int)hpv, kOff / 4 + 1);
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
      } else {
        return __builtin_bit_cast(T, (uint32_t)W::bcast_i((int)hpv, kOff / 4));
      }
    } else {
      return host_val;
    }
  }
// HP() reads other lanes of `hpv`, so it is only ever evaluated in wave-uniform control flow (all 64 lanes
// active): a VGPR reloaded from a spill under a partial EXEC mask holds garbage in its inactive lanes. Lane-parallel
// loops and lane-0 blocks take the fields they need as locals hoisted in front of them (TopoView, the observe() and
// trace() pointers, ...); the locals are SGPRs, whose spills go to whole-wave VGPR lanes.
#define HP(f) hp_get<decltype(HotParams::f), (int)offsetof(HotParams, f)>(HPp->f)

  // ---------------------------------------------------------------- hot-block residency
  // LDS residency copies only the LIVE part of the hot block: the fixed sections (header, jobs, executors,
  // commitments, the COMMON and job pools) and, of the per-stage sections, the stage and stage-pool records of
  // the jobs from the lowest active one to the last arrived one plus the used prefix of the active-stage and
  // schedulable lists. Stages of completed jobs are never read again and those of jobs not yet arrived are
  // initialised at arrival (on_job_arrival), so nothing outside the range is read during the launch.
  // A copy issues up to kCopyBatch 16-B loads per lane before any store (one memory latency per batch).
  static constexpr int kCopyBatch = 12;
  // 16 bytes as a native vector (one dwordx4 load / store). HIP's uint4 is a struct with a union inside, and the
  // copy's array of them was placed in scratch memory (a store and a reload per element through the scratch path).
  typedef uint32_t u32x4 __attribute__((vector_size(16)));
  struct Span {
    int64_t off, n;  // byte offset in the hot block, 16-B units
  };
  template <int kSpans>
  __device__ __forceinline__ void copy_spans(uint8_t* dst, const uint8_t* src, const Span (&sp)[kSpans]) {
    W::sync();
    int64_t end[kSpans];
    int64_t total = 0;
#pragma unroll
    for (int r = 0; r < kSpans; ++r) end[r] = (total += sp[r].n);
    for (int64_t i0 = 0; i0 < total; i0 += (int64_t)W::kWidth * kCopyBatch) {
      u32x4 v[kCopyBatch];
      int64_t at[kCopyBatch];
#pragma unroll
      for (int u = 0; u < kCopyBatch; ++u) {
        const int64_t i = i0 + (int64_t)u * W::kWidth + W::lane();
        int64_t o = -1;
#pragma unroll
        for (int r = kSpans - 1; r >= 0; --r)
          if (i < end[r]) o = sp[r].off + (i - (end[r] - sp[r].n)) * 16;  // (a later r overwrites: may be < 0)
        at[u] = i < total ? o : -1;
        if (at[u] >= 0) v[u] = *reinterpret_cast<const u32x4*>(src + at[u]);
      }
#pragma unroll
      for (int u = 0; u < kCopyBatch; ++u)
        if (at[u] >= 0) *reinterpret_cast<u32x4*>(dst + at[u]) = v[u];
    }
    W::sync();
  }
  int32_t live_lo = 0;  // first stage of the live range (set by load_hot; 0 after an in-launch reset)
  // End of the live stage range: the stages of every arrived job (hot block in place).
  __device__ __forceinline__ int live_hi() const {
    const int a = h.arrivals;
    return a > 0 ? (int)job_base(a - 1) + (int)job_nst(a - 1) : 0;
  }
  __device__ __forceinline__ Span stage_span(int lo, int hi) const { return {O.stages + 16 * (int64_t)lo, hi - lo}; }
  __device__ __forceinline__ Span pool_span(int lo, int hi) const {
    return {O.pools + 16 * (int64_t)(1 + JC + lo), hi - lo};
  }
  __device__ __forceinline__ Span list_span(int64_t off, int n) const { return {off, (2 * (int64_t)n + 15) >> 4}; }
  // Lowest stage still referenced (jobs' stages are contiguous in arrival order), from the header (registers) and
  // the fixed sections: the stages of the active jobs, and stage pools / stages a completed job can still be named by
  // — an executor left in one of its stage pools (ex.loc), an executor moving to one of its stages (EXECUTOR_READY
  // ev_stage), a commitment from or to one of its stage pools, the current source pool. Capped at live_hi().
  __device__ __forceinline__ int scan_live_lo() {
    const int16_t* aj = H<int16_t>(O.active_jobs);
    constexpr int kNone = 0x7FFFFFFF;
    int lo = is_stage_pool(h.source) ? pool_stage(h.source) : kNone;
    for (int k0 = 0; k0 < h.n_active_jobs; k0 += W::kWidth) {
      const int k = k0 + W::lane();
      const int b = k < h.n_active_jobs ? (int)job(aj[k]).base : kNone;
      lo = W::min_i(b < lo ? b : lo);
    }
    for (int k0 = 0; k0 < NE; k0 += W::kWidth) {
      const int e = k0 + W::lane();
      int b = kNone;
      if (e < NE) {
        const ExecRec x = exr(e);
        if (is_stage_pool(x.loc)) b = pool_stage(x.loc);
        if (x.ev_seq >= 0 && x.ev_stage >= 0 && x.ev_stage < b) b = x.ev_stage;
      }
      lo = W::min_i(b < lo ? b : lo);
    }
    for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
      if (k0 >= h.commit_hw) break;
      const int k = k0 + W::lane();
      int b = kNone;
      if (k < h.commit_hw) {
        const CommitRec r = cm(k);
        if (r.cnt > 0) {
          if (is_stage_pool(r.src)) b = pool_stage(r.src);
          if (is_stage_pool(r.dst) && pool_stage(r.dst) < b) b = pool_stage(r.dst);
        }
      }
      lo = W::min_i(b < lo ? b : lo);
    }
    const int hi = live_hi();
    return lo < hi ? lo : hi;
  }
  __device__ __forceinline__ void load_hot() {
    SSIM_TIC(t0);
    if (hot != ghot) {
      const Span fixed[2] = {{0, O.stages >> 4}, {O.pools, 1 + JC}};
      copy_spans(hot, ghot, fixed);
#ifdef SSIM_PROFILE
      prof_set(kTCopy1, W::realtime());
#endif
      load_header();
      live_lo = scan_live_lo();
      const int hi = live_hi();
      const Span live[4] = {stage_span(live_lo, hi), pool_span(live_lo, hi), list_span(O.active_stages, h.n_active_stages),
                            list_span(O.sched_list, h.n_sched)};
      copy_spans(hot, ghot, live);
    }
    if (ex_l) copy_execs(xb, ghot + O.execs);
    ev_regs_load();
    SSIM_TOC(t0, kPhLoadSave);
  }
  // Requires the header stored (store_header) and in registers (the state after a step or a preemption).
  __device__ __forceinline__ void save_hot() {
    SSIM_TIC(t0);
    if (hot != ghot) {
      const int hi = live_hi();
      const int lo = live_lo < hi ? live_lo : hi;
      const Span spans[6] = {{0, O.stages >> 4}, {O.pools, 1 + JC}, stage_span(lo, hi), pool_span(lo, hi),
                             list_span(O.active_stages, h.n_active_stages), list_span(O.sched_list, h.n_sched)};
      copy_spans(ghot, hot, spans);
    }
    if (ex_l) copy_execs(ghot + O.execs, xb);
    SSIM_TOC(t0, kPhLoadSave);
  }
  // ExecRec[N] between HBM and the LDS copy (ex_lds): 2N 16-B units, all loads of a lane issued before its stores
  __device__ __forceinline__ void copy_execs(uint8_t* dst, const uint8_t* src) {
    constexpr int kMax = (kN > 0 ? 2 * kN + W::kWidth - 1 : 2 * 256) / W::kWidth;  // (N <= 250: compute_layout)
    const int n = 2 * NE;
    u32x4 v[kMax];
    W::sync();
#pragma unroll
    for (int u = 0; u < kMax; ++u) {
      const int i = u * W::kWidth + W::lane();
      if (i < n) v[u] = reinterpret_cast<const u32x4*>(src)[i];
    }
#pragma unroll
    for (int u = 0; u < kMax; ++u) {
      const int i = u * W::kWidth + W::lane();
      if (i < n) reinterpret_cast<u32x4*>(dst)[i] = v[u];
    }
    W::sync();
  }

  // ---------------------------------------------------------------- field access
  template <class T>
  __device__ __forceinline__ T* H(int64_t off) const {
    return reinterpret_cast<T*>(hot + off);
  }
  template <class T>
  __device__ __forceinline__ T* S(int64_t off) const {
    return reinterpret_cast<T*>(scr + off);
  }
  __device__ __forceinline__ void load_header() {
    uint32_t w[sizeof(EnvHeader) / 4];  // wave-uniform copy: the header lives in SGPRs
    __builtin_memcpy(w, H<EnvHeader>(O.hdr), sizeof(w));
    for (int i = 0; i < (int)(sizeof(EnvHeader) / 4); ++i) w[i] = W::uni(w[i]);
    __builtin_memcpy(&h, w, sizeof(w));
    rng.s_hi = h.rng_s_hi;
    rng.s_lo = h.rng_s_lo;
    rng.i_hi = h.rng_i_hi;
    rng.i_lo = h.rng_i_lo;
    rng.has32 = h.rng_has32;
    rng.u32 = h.rng_u32;
  }
  __device__ __forceinline__ void store_header() {
    h.rng_s_hi = rng.s_hi;
    h.rng_s_lo = rng.s_lo;
    h.rng_i_hi = rng.i_hi;
    h.rng_i_lo = rng.i_lo;
    h.rng_has32 = rng.has32;
    h.rng_u32 = rng.u32;
    W::sync();
    if (W::lane() == 0) *H<EnvHeader>(O.hdr) = h;
    W::sync();
  }
  // Diagnostic builds (-DSSIM_ERR_LINE=1) also record the engine.h source line of the first sticky error
  // (EnvHeader::err_line: which invariant or capacity check froze the env; scripts/diag_large.py). Off in the product
  // build: the line select at every check site kept one more SGPR live through the engine (+51 SGPR spills on the
  // bench kernel, -4.8% decisions/s).
  __device__ __forceinline__ void fail(uint32_t bits, int line = __builtin_LINE()) {
#if SSIM_ERR_LINE
    if (!frozen() && (bits & SSIM_ERR_STICKY)) h.err_line = line;
#else
    (void)line;
#endif
    h.err |= bits;
  }
  __device__ __forceinline__ bool frozen() const { return (h.err & SSIM_ERR_STICKY) != 0u; }
  __device__ __forceinline__ void check(bool ok, int line = __builtin_LINE()) {
    if (!ok) fail(SSIM_ERR_INVARIANT, line);
  }

  // Field access. Two kinds, by who is asking:
  //  * serial code (wave-uniform index): the named accessors below return a UF proxy whose reads go
  //    through W::uni, so the value lands in an SGPR and the code that uses it is scalar;
  //  * lane-parallel loops (index differs per lane): read whole records by value (stage(g), job(j),
  //    exr(e) ...) — never through UF, whose readfirstlane would broadcast lane 0's value.
  template <class T, int kSec = -1>
  struct UF {
    T* p;
    __device__ __forceinline__ operator T() const {
      SSIM_FIELD_STAT(kSec);
      return W::uni(*p);
    }
    __device__ __forceinline__ UF& operator=(T v) {
      *p = v;
      return *this;
    }
    __device__ __forceinline__ UF& operator+=(int v) {
      SSIM_FIELD_STAT(kSec);
      *p = (T)(*p + v);
      return *this;
    }
    __device__ __forceinline__ UF& operator-=(int v) {
      SSIM_FIELD_STAT(kSec);
      *p = (T)(*p - v);
      return *this;
    }
  };
  template <class T>
  __device__ __forceinline__ T ld(const T* q) const {  // uniform read of a scratch / list entry
    return W::uni(*q);
  }
  template <class T>
  __device__ __forceinline__ T ldu(const T* q, int64_t i) const {  // uniform dataset read
    return W::uni(ldg(q, i));
  }

  // Wave-uniform register copy of a whole record for serial code: one LDS access (16-B loads) and every
  // word through W::uni (SGPRs), instead of one dependent load per field; written back with `rec = copy`.
  template <class R>
  __device__ __forceinline__ R ld_rec(const R& src) const {
    static_assert(sizeof(R) % 4 == 0, "records are whole words");
    uint32_t w[sizeof(R) / 4];
    __builtin_memcpy(w, &src, sizeof(R));
    for (int i = 0; i < (int)(sizeof(R) / 4); ++i) w[i] = W::uni(w[i]);
    R r;
    __builtin_memcpy(&r, w, sizeof(R));
    return r;
  }

  // records (layout.h)
  __device__ __forceinline__ StageRec& stage(int g) const { return H<StageRec>(O.stages)[g]; }
  __device__ __forceinline__ JobRec& job(int j) const { return H<JobRec>(O.jobs)[j]; }
  __device__ __forceinline__ JobTimes& jtimes(int j) const { return H<JobTimes>(O.jtimes)[j]; }
  __device__ __forceinline__ ExecRec& exr(int e) const { return reinterpret_cast<ExecRec*>(xb)[e]; }
  __device__ __forceinline__ CommitRec& cm(int k) const { return H<CommitRec>(O.commits)[k]; }
  __device__ __forceinline__ PoolRec& pool(int p) const { return H<PoolRec>(O.pools)[p]; }
  __device__ __forceinline__ double* recent() const { return reinterpret_cast<double*>(cold + O.st_recent); }
  // stages (env-global index g = job base + local stage id); `done` is derived: rem + exe + done = tasks
  __device__ __forceinline__ UF<int16_t, 0> st_job(int g) const { return {&stage(g).job}; }
  __device__ __forceinline__ UF<int16_t, 0> st_ts(int g) const { return {&stage(g).ts}; }
  __device__ __forceinline__ UF<int16_t, 0> st_rem(int g) const { return {&stage(g).rem}; }
  __device__ __forceinline__ UF<int16_t, 0> st_exe(int g) const { return {&stage(g).exe}; }
  __device__ __forceinline__ UF<int16_t, 0> st_mov(int g) const { return {&stage(g).mov}; }
  __device__ __forceinline__ UF<int16_t, 0> st_com(int g) const { return {&stage(g).com}; }
  __device__ __forceinline__ UF<int8_t, 0> st_unmet(int g) const { return {&stage(g).unmet}; }
  __device__ __forceinline__ UF<uint8_t, 0> st_sel(int g) const { return {&stage(g).sel}; }
  __device__ __forceinline__ UF<double, 6> st_recent(int g) const { return {recent() + g}; }
  __device__ __forceinline__ bool st_completed(int g) const { return st_rem(g) == 0 && st_exe(g) == 0; }
  // jobs
  __device__ __forceinline__ UF<int16_t, 1> job_tpl(int j) const { return {&job(j).tpl}; }
  __device__ __forceinline__ UF<int16_t, 1> job_base(int j) const { return {&job(j).base}; }
  __device__ __forceinline__ UF<int16_t, 1> job_nst(int j) const { return {&job(j).nst}; }
  __device__ __forceinline__ UF<int16_t, 1> job_nact(int j) const { return {&job(j).nact}; }
  __device__ __forceinline__ UF<int16_t, 1> job_sat(int j) const { return {&job(j).sat}; }
  __device__ __forceinline__ UF<int16_t, 1> job_local(int j) const { return {&job(j).local}; }
  __device__ __forceinline__ UF<int16_t, 1> job_supply(int j) const { return {&job(j).supply}; }
  __device__ __forceinline__ UF<int16_t, 1> job_state(int j) const { return {&job(j).state}; }
  __device__ __forceinline__ UF<int32_t, 1> job_arr_dec(int j) const { return {&job(j).arr_dec}; }
  __device__ __forceinline__ UF<int32_t, 1> job_done_dec(int j) const { return {&job(j).done_dec}; }
  __device__ __forceinline__ UF<double, 2> job_tarr(int j) const { return {&jtimes(j).tarr}; }
  __device__ __forceinline__ UF<double, 2> job_tdone(int j) const { return {&jtimes(j).tdone}; }
  // executors
  __device__ __forceinline__ UF<int16_t, 3> ex_loc(int e) const { return {&exr(e).loc}; }
  __device__ __forceinline__ UF<int16_t, 3> ex_job(int e) const { return {&exr(e).job}; }
  __device__ __forceinline__ UF<int16_t, 3> ex_task(int e) const { return {&exr(e).task}; }
  __device__ __forceinline__ UF<int16_t, 3> ex_busy(int e) const { return {&exr(e).busy}; }
  __device__ __forceinline__ UF<double, 4> ev_t(int e) const { return {&exr(e).ev_t}; }
  __device__ __forceinline__ UF<int32_t, 4> ev_seq(int e) const { return {&exr(e).ev_seq}; }
  __device__ __forceinline__ UF<int16_t, 4> ev_type(int e) const { return {&exr(e).ev_type}; }
  __device__ __forceinline__ UF<int16_t, 4> ev_stage(int e) const { return {&exr(e).ev_stage}; }
  // pools: code 0 = COMMON, 1+j = job j, 1+job_cap+g = stage g, -1 = None
  __device__ __forceinline__ int32_t job_pool(int j) const { return 1 + j; }
  __device__ __forceinline__ int32_t stage_pool(int g) const { return 1 + JC + g; }
  __device__ __forceinline__ bool is_stage_pool(int p) const { return p > JC; }
  __device__ __forceinline__ int32_t pool_stage(int p) const { return p - 1 - JC; }
  __device__ __forceinline__ int32_t pool_job(int p) const {  // pool_key[0]; -1 = None
    if (p <= 0) return -1;
    if (p <= JC) return p - 1;
    return st_job(p - 1 - JC);
  }
  __device__ __forceinline__ PySetMeta* pmeta(int p) const { return reinterpret_cast<PySetMeta*>(&pool(p)); }
  __device__ __forceinline__ uint8_t* ptab(int p) const { return cold + O.pool_tab + (int64_t)p * tab_stride_for(NE); }
  __device__ __forceinline__ UF<int16_t, 5> cfrom(int p) const { return {&pool(p).cfrom}; }
  __device__ __forceinline__ int pool_size(int p) const { return p < 0 ? 0 : (int)W::uni(pool(p).used); }

  // ---------------------------------------------------------------- tracker (executor_tracker.py)
  __device__ __forceinline__ int32_t source_job() const {  // :98-102
    return (h.source <= kPoolCommon) ? -1 : pool_job(h.source);
  }
  __device__ __forceinline__ int committable() {  // :105-111 (pool None is always empty with no commitments)
    if (h.source < 0) return 0;
    SSIM_FIELD_STAT(10);
    const PoolRec pr = pool(h.source);  // size and commitments-from in one LDS round trip
    const int n = (int)W::uni(pr.used) - (int)W::uni(pr.cfrom);
    check(n >= 0);
    return n;
  }
  __device__ __forceinline__ int demand(int g) const { return st_rem(g) - (st_mov(g) + st_com(g)); }  // :566-578

  __device__ __forceinline__ void supply_add(int job, int n) {
    if (job < 0)
      h.supply_none += n;
    else
      job_supply(job) += n;
  }

  __device__ __forceinline__ void add_commitment(int n, int dst) {  // :146-154, 224-236
    const int src = h.source;
    check(src >= 0);
    if (src < 0) return;
    int hit = -1, freeslot = -1;
    SSIM_FIELD_STAT(13);
    const int hw = h.commit_hw;
    for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
      if (k0 >= hw) break;
      const int k = k0 + W::lane();
      const bool ok = k < hw;
      CommitRec r{};
      if (ok) r = cm(k);
      const uint64_t mh = W::ballot(ok && r.cnt > 0 && r.src == src && r.dst == dst);
      const uint64_t mf = W::ballot(ok && r.cnt == 0);
      if (hit < 0 && mh) hit = k0 + W::ffs(mh);
      if (freeslot < 0 && mf) freeslot = k0 + W::ffs(mf);
    }
    // slots >= commit_hw were never used this episode (cleared at reset): the first free slot of the whole array
    if (freeslot < 0 && hw < commit_cap_for(NE)) freeslot = hw;
    if (hit < 0 && freeslot >= hw) h.commit_hw = freeslot + 1;
    W::sync();
    if (hit >= 0) {
      if (W::lane() == 0) cm(hit).cnt = (int16_t)(cm(hit).cnt + n);
    } else if (freeslot >= 0) {
      if (W::lane() == 0) {
        CommitRec& r = cm(freeslot);
        r.src = (int16_t)src;
        r.dst = (int16_t)dst;
        r.cnt = (int16_t)n;
        r.ord = h.commit_seq;
      }
      h.commit_seq++;
    } else {
      fail(SSIM_ERR_CAPACITY);
      return;
    }
    W::sync();
    cfrom(src) += n;
    if (is_stage_pool(dst)) st_com(pool_stage(dst)) += n;
    check(pool_size(src) >= cfrom(src));
    const int sj = pool_job(src), dj = pool_job(dst);
    if (dj != sj) supply_add(dj, n);
  }

  __device__ __forceinline__ int find_commit(int src, int dst) {
    SSIM_FIELD_STAT(13);
    for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
      if (k0 >= h.commit_hw) break;
      const int k = k0 + W::lane();
      bool hit = false;
      if (k < h.commit_hw) {
        const CommitRec r = cm(k);
        hit = r.cnt > 0 && r.src == src && r.dst == dst;
      }
      const uint64_t m = W::ballot(hit);
      if (m) return k0 + W::ffs(m);
    }
    return -1;
  }

  __device__ __forceinline__ int remove_commitment(int e, int dst) {  // :156-173, 238-249; returns src
    const int src = ex_loc(e);
    check(src >= 0);
    const int k = src >= 0 ? find_commit(src, dst) : -1;
    if (k < 0) {
      fail(SSIM_ERR_INVARIANT);  // ValueError("no commitments from ...") in the reference
      return src;
    }
    const int left = cm(k).cnt - 1;
    W::sync();
    if (W::lane() == 0) cm(k).cnt = (int16_t)left;
    W::sync();
    cfrom(src) -= 1;
    check(cfrom(src) >= 0);
    if (is_stage_pool(dst)) {
      st_com(pool_stage(dst)) -= 1;
      check(st_com(pool_stage(dst)) >= 0);
    }
    const int sj = pool_job(src), dj = pool_job(dst);
    if (dj != sj) {
      supply_add(dj, -1);
      check(dj < 0 ? h.supply_none >= 0 : job_supply(dj) >= 0);
    }
    return src;
  }

  __device__ __forceinline__ int peek_commitment(int p) {  // :175-180: first key in insertion order, -1 = None
    int best_ord = 0x7FFFFFFF, best_dst = kPoolNone;
    SSIM_FIELD_STAT(13);
    for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
      if (k0 >= h.commit_hw) break;
      const int k = k0 + W::lane();
      int ord = 0x7FFFFFFF, dst = kPoolNone;
      if (k < h.commit_hw) {
        const CommitRec r = cm(k);
        if (r.cnt > 0 && r.src == p) {
          ord = r.ord;
          dst = r.dst;
        }
      }
      W::min_pair(ord, dst);
      if (ord < best_ord) {
        best_ord = ord;
        best_dst = dst;
      }
    }
    return best_dst;
  }

  // Snapshot of commitments[src] in insertion order into scratch plan: (dst, count) pairs.
  __device__ __forceinline__ int commit_plan(int src, int32_t* plan) {
    int n = 0, last = -1;
    for (;;) {  // selection by increasing insertion stamp (live entries <= N)
      int ord = 0x7FFFFFFF, k_best = -1;
      SSIM_FIELD_STAT(13);
      for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
        if (k0 >= h.commit_hw) break;
        const int k = k0 + W::lane();
        int o = 0x7FFFFFFF, kk = -1;
        if (k < h.commit_hw) {
          const CommitRec r = cm(k);
          if (r.cnt > 0 && r.src == src && r.ord > last) {
            o = r.ord;
            kk = k;
          }
        }
        W::min_pair(o, kk);
        if (o < ord) {
          ord = o;
          k_best = kk;
        }
      }
      if (k_best < 0) break;
      const int dst = cm(k_best).dst, cnt = cm(k_best).cnt;
      W::sync();
      if (W::lane() == 0) {
        plan[2 * n] = dst;
        plan[2 * n + 1] = cnt;
      }
      W::sync();
      n++;
      last = ord;
    }
    return n;
  }

  // CPython-set tables: an 8-slot table lives inline in the PoolRec (LDS-resident with the hot block);
  // a table that has grown past 8 slots lives in the cold block. Either way an operation stages it into
  // an LDS scratch table (capacity set_cap, so a resize fits), runs the serial probe sequence there and
  // writes it back to the home its new size dictates.
  // The two homes are separate branches (not one selected pointer) so each copy compiles to ds_* or
  // global_* instructions rather than FLAT.
  __device__ __forceinline__ uint8_t* stage_table(int p) {
    uint8_t* t = S<uint8_t>(O.sc_tab_p);
    const int size = (int)W::uni(pool(p).mask) + 1;
    W::sync();
    if (size == 8) {
      SSIM_COUNT(kCtPoolSmall);
      const uint8_t* g = pool(p).tab;
      for (int i = W::lane(); i < 8; i += W::kWidth) t[i] = g[i];
    } else {
      SSIM_COUNT(kCtPoolBig);
      SSIM_TIC(t0);
      const uint8_t* g = ptab(p);
      for (int i = W::lane(); i < size; i += W::kWidth) t[i] = g[i];
      W::sync();
      if (W::uni(t[0]) == 0xFD) t[0] = 0xFD;  // profile build only: wait for the staged bytes
      SSIM_TOC(t0, kPhPoolBig);
    }
    W::sync();
    return t;
  }
  __device__ __forceinline__ void unstage_table(int p, const uint8_t* t) {
    W::sync();
    const int size = (int)W::uni(pool(p).mask) + 1;
    if (size == 8) {
      uint8_t* g = pool(p).tab;
      for (int i = W::lane(); i < 8; i += W::kWidth) g[i] = t[i];
    } else {
      uint8_t* g = ptab(p);
      for (int i = W::lane(); i < size; i += W::kWidth) g[i] = t[i];
    }
    W::sync();
  }
  // ---- lane-parallel CPython-set operations (device waves; tables of <= 64 slots, i.e. N <= 15) ----
  // Lane i holds slot i of the table. The probe sequence of pyset.h is walked on wave-uniform 64-bit
  // ballots (EMPTY / DUMMY / key slots) with SALU bit operations, so an operation costs one lane-parallel
  // table load instead of a chain of dependent single-byte reads. Same semantics as pyset.h (whose serial
  // form the host build keeps, pinned against CPython by tests/test_kats.py); the device form is pinned by
  // the GPU parity tests' per-event executor traces.
  static constexpr bool kLaneSets = W::kWidth == 64;
  __device__ __forceinline__ bool lane_sets() const { return kLaneSets && set_cap_for(NE) <= 64; }
  __device__ __forceinline__ static uint64_t slot_bits(uint32_t mask) {
    return mask >= 63 ? ~0ull : ((1ull << (mask + 1)) - 1);
  }
  // CPython probe walk for `key` over the ballots: returns the slot holding key or -1; *empty = the EMPTY
  // slot that ended the walk, *dummy = the last DUMMY slot seen before it (-1: none) — set_add_entry's
  // freeslot. Tables without dummies and without the key give set_insert_clean's slot in *empty.
  __device__ __forceinline__ static int lt_probe(uint64_t E, uint64_t Dm, uint64_t K, uint32_t mask, uint32_t key,
                                                 int* empty, int* dummy) {
    uint32_t i = key & mask, perturb = key;
    int fd = -1;
    for (;;) {
      const uint64_t w = (i + 9u <= mask) ? (0x3FFull << i) : (1ull << i);
      const uint64_t stop = (E | K) & w;
      if (stop) {
        const int f = __builtin_ctzll(stop);
        const uint64_t d = Dm & w & ((1ull << f) - 1);
        if (d) fd = 63 - __builtin_clzll(d);
        *dummy = fd;
        if ((K >> f) & 1ull) {
          *empty = -1;
          return f;
        }
        *empty = f;
        return -1;
      }
      const uint64_t d = Dm & w;
      if (d) fd = 63 - __builtin_clzll(d);
      perturb >>= 5;
      i = (i * 5u + 1u + perturb) & mask;
    }
  }
  // A pool's metadata and (8-slot table) this lane's slot byte from ONE 16-B record read; tables past 8 slots are
  // read from the cold block.
  struct PoolView {
    uint32_t mask, fill, used;
    int v;
  };
  __device__ __forceinline__ PoolView pool_view(int p) {
    SSIM_FIELD_STAT(10);
    const PoolRec r = pool(p);
    uint32_t w[4];
    __builtin_memcpy(w, &r, sizeof(w));
    const uint32_t w0 = W::uni(w[0]), w1 = W::uni(w[1]);
    PoolView pv;
    pv.mask = w0 & 0xFFFFu;
    pv.fill = w0 >> 16;
    pv.used = w1 & 0xFFFFu;
    const int l = W::lane();
    if (pv.mask == 7) {
      const uint64_t tab = ((uint64_t)w[3] << 32) | w[2];
      pv.v = l < 8 ? (int)((tab >> (8 * l)) & 0xFFu) : kSlotEmpty;
    } else {
      pv.v = l <= (int)pv.mask ? (int)ptab(p)[l] : kSlotEmpty;
    }
    return pv;
  }
  __device__ __forceinline__ void lt_store(int p, uint32_t mask, int slot, int val) {
    W::sync();
    if (W::lane() == 0) {
      if (mask == 7)
        pool(p).tab[slot] = (uint8_t)val;
      else
        ptab(p)[slot] = (uint8_t)val;
    }
    W::sync();
  }
  __device__ __forceinline__ void lt_meta(int p, uint32_t mask, uint32_t fill, uint32_t used) {
    W::sync();
    if (W::lane() == 0) {
      PoolRec& r = pool(p);
      r.mask = (uint16_t)mask;
      r.fill = (uint16_t)fill;
      r.used = (uint16_t)used;
    }
    W::sync();
  }
  // Clean insert of the slot values of `v` (occupied slots in `occ`, table order) into a fresh table of
  // `size` slots; returns the new table (this lane's slot).
  __device__ __forceinline__ static int lt_reinsert(int v, uint64_t occ, uint32_t size) {
    const uint32_t mask = size - 1;
    uint64_t E = slot_bits(mask);
    int nv = kSlotEmpty;
    while (occ) {
      const int s = __builtin_ctzll(occ);
      occ &= occ - 1;
      const int key = W::bcast_i(v, s);
      int slot, dm;
      lt_probe(E, 0, 0, mask, (uint32_t)key, &slot, &dm);
      E &= ~(1ull << slot);
      nv = W::writelane(key, slot, nv);
    }
    return nv;
  }
  // set_table_resize(minused) of pool p whose current slots are `v`; writes the table to its new home.
  __device__ __forceinline__ void lt_resize(int p, int v, uint32_t mask, uint32_t minused) {
    const uint64_t occ = W::ballot(v < kSlotDummy) & slot_bits(mask);
    const uint32_t n = (uint32_t)W::popc(occ);
    uint32_t size = 8;
    while (size <= minused) size <<= 1;
    const int nv = lt_reinsert(v, occ, size);
    const int l = W::lane();
    if (size == 8) {
      if (l < 8) pool(p).tab[l] = (uint8_t)nv;
    } else {
      if (l < (int)size) ptab(p)[l] = (uint8_t)nv;
    }
    lt_meta(p, size - 1, n, n);
  }
  __device__ __forceinline__ void pool_add_lanes(int p, int e) {
    const PoolView pv = pool_view(p);
    const uint32_t mask = pv.mask, fill = pv.fill, used = pv.used;
    const int v = pv.v;
    const uint64_t E = W::ballot(v == kSlotEmpty) & slot_bits(mask), Dm = W::ballot(v == kSlotDummy),
                   K = W::ballot(v == e);
    int empty, dummy;
    if (lt_probe(E, Dm, K, mask, (uint32_t)e, &empty, &dummy) >= 0) return;  // already present
    if (dummy >= 0) {
      lt_store(p, mask, dummy, e);
      lt_meta(p, mask, fill, used + 1);
      return;
    }
    if ((fill + 1) * 5u >= mask * 3u) {
      lt_resize(p, W::lane() == empty ? e : v, mask, (used + 1) * 4);
      return;
    }
    lt_store(p, mask, empty, e);
    lt_meta(p, mask, fill + 1, used + 1);
  }
  __device__ __forceinline__ bool pool_remove_lanes(int p, int e) {
    const PoolView pv = pool_view(p);
    const uint32_t mask = pv.mask, fill = pv.fill, used = pv.used;
    const int v = pv.v;
    const uint64_t E = W::ballot(v == kSlotEmpty) & slot_bits(mask), K = W::ballot(v == e);
    int empty, dummy;
    const int slot = lt_probe(E, 0, K, mask, (uint32_t)e, &empty, &dummy);
    if (slot < 0) return false;
    lt_store(p, mask, slot, kSlotDummy);
    lt_meta(p, mask, fill, used - 1);
    return true;
  }
  // Keys (lane r = r-th key) in the iteration order of set(keys) built by sequential adds into a fresh set.
  __device__ __forceinline__ static int lt_build_order(int kv, int n) {
    uint32_t mask = 7, fill = 0;
    uint64_t E = 0xFFull;
    int tv = kSlotEmpty;
    for (int r = 0; r < n; ++r) {
      const int key = W::bcast_i(kv, r);
      int slot, dm;
      lt_probe(E, 0, 0, mask, (uint32_t)key, &slot, &dm);
      E &= ~(1ull << slot);
      tv = W::writelane(key, slot, tv);
      fill++;
      if (fill * 5u >= mask * 3u) {  // ps_resize(used * 4): clean re-insert in table order
        uint32_t size = 8;
        while (size <= fill * 4u) size <<= 1;
        const uint64_t occ = ~E & slot_bits(mask);
        tv = lt_reinsert(tv, occ, size);
        mask = size - 1;
        E = W::ballot(tv == kSlotEmpty) & slot_bits(mask);
      }
    }
    return W::compact(~E & slot_bits(mask), tv);
  }
  // idle_order (below) for lane-sized tables: out[0..n) = executor ids, returns n.
  __device__ __forceinline__ int idle_order_lanes(int p, int32_t* out) {
    const PoolView pv = pool_view(p);
    const uint32_t mask = pv.mask, fill = pv.fill, used = pv.used;
    const int v = pv.v;
    const uint64_t occ = W::ballot(v < kSlotDummy) & slot_bits(mask);
    int n = W::popc(occ);
    int kv = W::compact(occ, v);  // keys in table order
    // pool.copy(): same order if the fresh table has the same mask and the source no dummies
    uint32_t size = 8;
    if (n * 5 >= 21)
      while ((int)size <= n * 2) size <<= 1;
    if (n > 0 && !(size - 1 == mask && fill == used)) {
      const int tv = lt_reinsert(kv, (n >= 64 ? ~0ull : ((1ull << n) - 1)), size);
      kv = W::compact(W::ballot(tv != kSlotEmpty) & slot_bits(size - 1), tv);
    }
    // filter `not executor.is_executing`, keeping order
    const int l = W::lane();
    const bool keep = l < n && !exr(l < n ? kv : 0).busy;
    const uint64_t mk = W::ballot(keep);
    kv = W::compact(mk, kv);
    n = W::popc(mk);
    kv = lt_build_order(kv, n);
    W::sync();
    if (l < n) out[l] = kv;
    W::sync();
    return n;
  }

  // ---- paged tables (device waves; 64 < set_cap <= 512, i.e. 16..127 executors: configs[2] / [3]) ----
  // A table of up to 512 slots is held 8 slots per lane, page-major in registers: lane l holds slots l, 64 + l, ...,
  // 448 + l as the bytes of one 64-bit value (byte g = slot 64g + l). Its cold-block home keeps slot order (byte s =
  // slot s, layout.h tab_stride_for), so loading page g is one coalesced 64-B byte load per lane, a table costs its
  // current size in bytes (not the 512-B capacity) and a slot write is one byte store.
  // A probe window (<= 10 consecutive slots) lies in one page or two adjacent ones: per probe step, ballots of the
  // page's byte (EMPTY / DUMMY / key) give the window's bits with no dependent per-slot loads (the serial form staged
  // the table through LDS and walked it one byte read at a time; N = 100 makes ~18 set operations per decision).
  // Orders: a fresh table built by clean inserts (copy(), set(gen), a resize) whose keys are all below its size
  // holds every key at its home slot (hash(int) = int), so its iteration order is ascending. The remaining cases have
  // at most 64 slots (with N <= 127, copy / set(gen) / resize sizes above 64 exceed every key) and reuse the one-page
  // lane-set functions above. Same semantics as pyset.h (pinned against CPython by tests/test_kats.py); this form is
  // pinned against CPython directly by tests/test_gpu_sets.py (ssim_debug_set_trace) and by the GPU parity cases.
  static constexpr bool kPagedSets = W::kWidth == 64;
  __device__ __forceinline__ bool paged_sets() const {
    return kPagedSets && set_cap_for(NE) > 64 && set_cap_for(NE) <= kPagedTabMax;
  }
  __device__ __forceinline__ static uint32_t page_byte(uint64_t v, uint32_t g) { return (uint32_t)(v >> (8 * g)) & 0xFFu; }
  struct PagedView {
    uint32_t mask, fill, used;
    uint64_t v;  // this lane's slots (byte g = slot 64g + lane); EMPTY outside the table
  };
  __device__ __forceinline__ PagedView paged_view(int p) {
    const int l = W::lane();
    SSIM_FIELD_STAT(10);
    const PoolRec r = pool(p);
    uint32_t w[4];
    __builtin_memcpy(w, &r, sizeof(w));
    const uint32_t w0 = W::uni(w[0]), w1 = W::uni(w[1]);
    PagedView pv;
    pv.mask = w0 & 0xFFFFu;
    pv.fill = w0 >> 16;
    pv.used = w1 & 0xFFFFu;
    const uint32_t size = pv.mask + 1;
    // The cold home is read only once the record says the table lives there, and only its `size` bytes (slot order:
    // page g is the 64 contiguous bytes at 64g, so lane l's byte load of each page is one coalesced 64-B segment).
    // An inline 8-slot table (the common case: most stage and job pools) issues no cold read at all.
    if (size == 8) {
      const uint32_t b = ((l < 4 ? w[2] : w[3]) >> (8 * (l & 3))) & 0xFFu;
      pv.v = page_of(l < 8 ? (0xFFFFFF00u | b) : 0xFFFFFFFFu, 0xFFFFFFFFu);
    } else if (size <= 64) {
      const uint32_t b = l < (int)size ? (uint32_t)ptab(p)[l] : kSlotEmpty;
      pv.v = page_of(0xFFFFFF00u | b, 0xFFFFFFFFu);
    } else {  // 2, 4 or 8 pages; pages np.. are EMPTY
      const uint8_t* t = ptab(p) + l;
      const uint32_t np = size / 64;
      const uint32_t b0 = t[0], b1 = t[64];
      uint32_t lo = 0xFFFF0000u | (b1 << 8) | b0, hi = 0xFFFFFFFFu;
      if (np >= 4) lo = ((uint32_t)t[192] << 24) | ((uint32_t)t[128] << 16) | (b1 << 8) | b0;
      if (np >= 8)
        hi = ((uint32_t)t[448] << 24) | ((uint32_t)t[384] << 16) | ((uint32_t)t[320] << 8) | (uint32_t)t[256];
      pv.v = page_of(lo, hi);
    }
    return pv;
  }
  // bits r < wn of the slots i + r (one page, or two adjacent ones): EMPTY, DUMMY and `key`
  __device__ __forceinline__ static void paged_win(uint64_t v, uint32_t i, uint32_t wn, uint32_t key, uint32_t* E,
                                                   uint32_t* D, uint32_t* K) {
    const uint32_t g = i >> 6, o = i & 63u;
    const uint32_t b0 = page_byte(v, g);
    uint64_t e = W::ballot(b0 == kSlotEmpty) >> o, d = W::ballot(b0 == kSlotDummy) >> o, k = W::ballot(b0 == key) >> o;
    if (o + wn > 64u) {  // (o >= 55: the shifts below are < 64)
      const uint32_t b1 = page_byte(v, g + 1);
      e |= W::ballot(b1 == kSlotEmpty) << (64u - o);
      d |= W::ballot(b1 == kSlotDummy) << (64u - o);
      k |= W::ballot(b1 == key) << (64u - o);
    }
    const uint64_t wm = (1ull << wn) - 1ull;
    *E = (uint32_t)(e & wm);
    *D = (uint32_t)(d & wm);
    *K = (uint32_t)(k & wm);
  }
  // CPython probe walk for `key` (lt_probe on a paged table): the slot holding key or -1; *empty = the EMPTY slot that
  // ended the walk, *dummy = the last DUMMY seen before it (set_add_entry's freeslot; dummies = false: set_lookkey).
  __device__ __forceinline__ static int paged_probe(uint64_t v, uint32_t mask, uint32_t key, bool dummies, int* empty,
                                                    int* dummy) {
    uint32_t i = key & mask, perturb = key;
    int fd = -1;
    for (int it = 0;; ++it) {
      if constexpr (KatBadPage<W>::value) {  // the known-bad KAT variant may corrupt a table past any EMPTY slot:
        if (it > 4096) {                     // end its walk instead of spinning
          *empty = -1;
          *dummy = -1;
          return -1;
        }
      }
      const uint32_t wn = (i + 9u <= mask) ? 10u : 1u;
      uint32_t E, D, K;
      paged_win(v, i, wn, key, &E, &D, &K);
      if (!dummies) D = 0;
      const uint32_t stop = E | K;
      if (stop) {
        const int f = __builtin_ctz(stop);
        const uint32_t d = D & ((1u << f) - 1u);
        if (d) fd = (int)i + 31 - __builtin_clz(d);
        *dummy = fd;
        if ((K >> f) & 1u) {
          *empty = -1;
          return (int)i + f;
        }
        *empty = (int)i + f;
        return -1;
      }
      if (D) fd = (int)i + 31 - __builtin_clz(D);
      perturb >>= 5;
      i = (i * 5u + 1u + perturb) & mask;
    }
  }
  // Per-lane 64-bit pages are assembled from explicit 32-bit halves: ROCm 7.2 miscompiles the i64 form
  // `(v & ~0xFF00ull) | ((uint64_t)x << 8)` under a lane predicate in the (executors, jobs)-specialised kernels
  // (the high half came out as the shifted value's zero instead of v's, leaving key 0 in slots 256..511).
  __device__ __forceinline__ static uint64_t page_of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
  // pages 0 and 1 hold b0 / b1 (EMPTY elsewhere): the clean-insert tables whose keys are all below 128
  __device__ __forceinline__ static uint64_t page01(uint32_t b0, uint32_t b1) {
    // (the test-only KAT wave type reproduces the miscompiled result in one lane: key 0 in slot 256 of a clean-insert
    // table; the miscompile put it in every lane's pages 4..7, which leaves no bound on the walks that follow)
    return page_of(0xFFFF0000u | (b1 << 8) | b0, KatBadPage<W>::value && W::lane() == 0 ? 0xFFFFFF00u : 0xFFFFFFFFu);
  }
  __device__ __forceinline__ static uint64_t paged_set(uint64_t v, int slot, int val) {  // the register copy
    const uint32_t g = (uint32_t)(slot >> 6), sh = 8u * (g & 3u);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint32_t m = ~(0xFFu << sh), b = (uint32_t)(uint8_t)val << sh;
    if (g < 4u) lo = (lo & m) | b;
    else hi = (hi & m) | b;
    return W::lane() == (slot & 63) ? page_of(lo, hi) : v;
  }
  __device__ __forceinline__ void paged_store(int p, uint32_t mask, int slot, int val) {  // one slot at its home
    W::sync();
    if (W::lane() == 0) {
      if (mask == 7)
        pool(p).tab[slot] = (uint8_t)val;
      else
        ptab(p)[slot] = (uint8_t)val;
    }
    W::sync();
  }
  __device__ __forceinline__ void paged_write(int p, uint32_t size, uint64_t v) {  // a whole (new) table
    const int l = W::lane();
    W::sync();
    if (size == 8) {
      if (l < 8) pool(p).tab[l] = (uint8_t)v;
    } else if (size <= 64) {
      if (l < (int)size) ptab(p)[l] = (uint8_t)v;
    } else {  // page g of this lane's register copy to byte 64g + l
      uint8_t* t = ptab(p) + l;
      const uint32_t np = size / 64, lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
      t[0] = (uint8_t)lo;
      t[64] = (uint8_t)(lo >> 8);
      if (np >= 4) {
        t[128] = (uint8_t)(lo >> 16);
        t[192] = (uint8_t)(lo >> 24);
      }
      if (np >= 8) {
        t[256] = (uint8_t)hi;
        t[320] = (uint8_t)(hi >> 8);
        t[384] = (uint8_t)(hi >> 16);
        t[448] = (uint8_t)(hi >> 24);
      }
    }
    W::sync();
  }
  // the keys of a paged table as a bitmap over executor ids (k0: ids 0..63, k1: 64..127), via LDS atomics
  __device__ __forceinline__ void paged_keys(uint64_t v, uint32_t np, uint64_t* k0, uint64_t* k1) {
    uint32_t* bm = S<uint32_t>(O.sc_bits);
    W::drain();
    if (W::lane() < 4) bm[W::lane()] = 0u;
    W::drain();
    for (uint32_t g = 0; g < np; ++g) {
      const uint32_t b = page_byte(v, g);
      if (b < kSlotDummy) W::aor(bm + (b >> 5), 1u << (b & 31u));
    }
    W::drain();
    const u32x4 q = *reinterpret_cast<const u32x4*>(bm);
    *k0 = ((uint64_t)W::uni((uint32_t)q[1]) << 32) | W::uni((uint32_t)q[0]);
    *k1 = ((uint64_t)W::uni((uint32_t)q[3]) << 32) | W::uni((uint32_t)q[2]);
  }
  __device__ __forceinline__ static int bits_max(uint64_t k0, uint64_t k1) {  // highest set bit, -1 if none
    return k1 ? 127 - __builtin_clzll(k1) : k0 ? 63 - __builtin_clzll(k0) : -1;
  }
  // the ids of a bitmap in ascending order into out[] (lane-parallel); returns the count
  __device__ __forceinline__ static int out_ascending(uint64_t k0, uint64_t k1, int32_t* out) {
    const int l = W::lane(), n0 = W::popc(k0);
    W::drain();
    if ((k0 >> l) & 1ull) out[W::rank(k0)] = l;
    if ((k1 >> l) & 1ull) out[n0 + W::rank(k1)] = 64 + l;
    W::drain();
    return n0 + W::popc(k1);
  }
  // the keys of a paged table in iteration (slot) order into out[], those with keep(key) only; returns the count
  template <class Keep>
  __device__ __forceinline__ static int paged_order(uint64_t v, uint32_t np, int32_t* out, const Keep& keep) {
    int n = 0;
    W::drain();
    for (uint32_t g = 0; g < np; ++g) {
      const uint32_t b = page_byte(v, g);
      const bool in = b < kSlotDummy && keep(b);
      const uint64_t m = W::ballot(in);
      if (in) out[n + W::rank(m)] = (int32_t)b;
      n += W::popc(m);
    }
    W::drain();
    return n;
  }
  __device__ __forceinline__ static uint32_t pages_of(uint32_t size) { return size > 64 ? size / 64 : 1; }
  // size of a fresh set after n sequential adds (pyset.h ps_add's resizes to > 4 * used: 8, 32, 128, 512)
  __device__ __forceinline__ static uint32_t build_size(uint32_t n) {
    return n <= 4 ? 8u : n <= 18 ? 32u : n <= 76 ? 128u : 512u;
  }
  __device__ __forceinline__ static uint32_t copy_size(uint32_t n) {  // set.copy()'s table (ps_copy_order)
    uint32_t size = 8;
    if (n * 5 >= 21)
      while (size <= n * 2) size <<= 1;
    return size;
  }
  // set_table_resize(minused) of pool p whose slots are `v` (n keys): clean re-insert in table order, to the new home
  __device__ __forceinline__ void paged_resize(int p, uint64_t v, uint32_t mask, uint32_t n, uint32_t minused) {
    uint32_t size = 8;
    while (size <= minused) size <<= 1;
    const uint32_t np = pages_of(mask + 1);
    uint64_t k0, k1;
    paged_keys(v, np, &k0, &k1);
    const int l = W::lane();
    uint64_t nv;
    if (bits_max(k0, k1) < (int)size) {  // every key at its home slot (pages 0 and 1: ids < 128)
      const bool in0 = l < (int)size && ((k0 >> l) & 1ull), in1 = 64 + l < (int)size && ((k1 >> l) & 1ull);
      nv = page01(in0 ? (uint32_t)l : kSlotEmpty, in1 ? (uint32_t)(64 + l) : kSlotEmpty);
    } else {  // size <= 64 (n <= 15): the one-page clean re-insert
      int32_t* tmp = S<int32_t>(O.sc_keys_b);
      const int nn = paged_order(v, np, tmp, [](uint32_t) { return true; });
      const int src = l < nn ? tmp[l] : (int)kSlotEmpty;
      const int tv = lt_reinsert(src, nn >= 64 ? ~0ull : ((1ull << nn) - 1ull), size);
      nv = page_of(0xFFFFFF00u | (uint32_t)(uint8_t)tv, 0xFFFFFFFFu);
    }
    paged_write(p, size, nv);
    lt_meta(p, size - 1, n, n);
  }
  __device__ __forceinline__ void pool_add_paged(int p, int e) {
    const PagedView pv = paged_view(p);
    int empty, dummy;
    if (paged_probe(pv.v, pv.mask, (uint32_t)e, true, &empty, &dummy) >= 0) return;  // already present
    if (dummy >= 0) {
      paged_store(p, pv.mask, dummy, e);
      lt_meta(p, pv.mask, pv.fill, pv.used + 1);
      return;
    }
    if ((pv.fill + 1) * 5u >= pv.mask * 3u) {
      paged_resize(p, paged_set(pv.v, empty, e), pv.mask, pv.used + 1, (pv.used + 1) * 4);
      return;
    }
    paged_store(p, pv.mask, empty, e);
    lt_meta(p, pv.mask, pv.fill + 1, pv.used + 1);
  }
  __device__ __forceinline__ bool pool_remove_paged(int p, int e) {
    const PagedView pv = paged_view(p);
    int empty, dummy;
    const int slot = paged_probe(pv.v, pv.mask, (uint32_t)e, false, &empty, &dummy);
    if (slot < 0) return false;
    paged_store(p, pv.mask, slot, kSlotDummy);
    lt_meta(p, pv.mask, pv.fill, pv.used - 1);
    return true;
  }
  // idle_order (below) of a paged table: out[0..n) = executor ids, returns n
  __device__ __forceinline__ int idle_order_paged(int p, int32_t* out) {
    const PagedView pv = paged_view(p);
    const uint32_t size = pv.mask + 1, np = pages_of(size);
    uint64_t k0, k1;
    paged_keys(pv.v, np, &k0, &k1);
    const int l = W::lane();
    const bool x0 = l < NE && exr(l).busy != 0, x1 = 64 + l < NE && exr(64 + l).busy != 0;
    const uint64_t b0 = W::ballot(x0), b1 = W::ballot(x1);
    const uint64_t f0 = k0 & ~b0, f1 = k1 & ~b1;
    const int nf = W::popc(f0) + W::popc(f1);
    if (nf == 0) return 0;
    // set(gen) of the idle keys: a fresh set whose final size exceeds every key holds them in ascending order,
    // whatever order the copy() yields them in
    if (bits_max(f0, f1) < (int)build_size((uint32_t)nf)) return out_ascending(f0, f1, out);
    // nf <= 18 from here (every larger set(gen) ends at 128 slots): the copy's order, filtered, then the adds
    const auto idle = [&](uint32_t b) { return ((((b < 64u) ? b0 : b1) >> (b & 63u)) & 1ull) == 0ull; };
    int32_t* tmp = S<int32_t>(O.sc_keys_b);
    const uint32_t sc = copy_size(pv.used);
    int kv;
    if (sc == size && pv.fill == pv.used) {  // copy() is a slot copy: the source's order
      paged_order(pv.v, np, tmp, idle);
      kv = l < nf ? tmp[l] : (int)kSlotEmpty;
    } else if (bits_max(k0, k1) < (int)sc) {  // copy() re-inserts at the home slots: ascending
      out_ascending(f0, f1, tmp);
      kv = l < nf ? tmp[l] : (int)kSlotEmpty;
    } else {  // copy() of <= 31 keys into <= 64 slots: the one-page clean re-insert in the source's order
      const int nn = paged_order(pv.v, np, tmp, [](uint32_t) { return true; });
      const int src = l < nn ? tmp[l] : (int)kSlotEmpty;
      const int tv = lt_reinsert(src, nn >= 64 ? ~0ull : ((1ull << nn) - 1ull), sc);
      const bool keep = tv != (int)kSlotEmpty && idle((uint32_t)tv);
      kv = W::compact(W::ballot(keep), tv);
    }
    kv = lt_build_order(kv, nf);
    W::drain();
    if (l < nf) out[l] = kv;
    W::drain();
    return nf;
  }
  // set(range(N)) built by sequential adds (reset's COMMON pool): every key at its home slot
  __device__ __forceinline__ void paged_init_range(int p, int n) {
    const uint32_t size = build_size((uint32_t)n);
    const int l = W::lane();
    const bool in0 = l < n && l < (int)size, in1 = 64 + l < n && 64 + l < (int)size;
    paged_write(p, size, page01(in0 ? (uint32_t)l : kSlotEmpty, in1 ? (uint32_t)(64 + l) : kSlotEmpty));
    lt_meta(p, size - 1, (uint32_t)n, (uint32_t)n);
  }
  // the keys of pool p in iteration order into out[] (diagnostic / the set known-answer test); returns the count
  __device__ __forceinline__ int table_keys(int p, int32_t* out) {
    if constexpr (kPagedSets) {
      if (paged_sets()) {
        const PagedView pv = paged_view(p);
        return paged_order(pv.v, pages_of(pv.mask + 1), out, [](uint32_t) { return true; });
      }
    }
    if constexpr (kLaneSets) {
      if (lane_sets()) {
        const PoolView pv = pool_view(p);
        const uint64_t occ = W::ballot(pv.v < kSlotDummy) & slot_bits(pv.mask);
        const int kv = W::compact(occ, pv.v);
        W::sync();
        if (W::lane() < W::popc(occ)) out[W::lane()] = kv;
        W::sync();
        return W::popc(occ);
      }
    }
    const uint8_t* t = stage_table(p);
    const int n = ps_keys<W>(pmeta(p), t, out);
    W::sync();
    return n;
  }

  __device__ __forceinline__ void pool_add(int p, int e) {
    SSIM_POOL_STAT(0, (int)W::uni(pool(p).mask) + 1, pool_size(p));
    SSIM_TIC(t0);
    if constexpr (kPagedSets) {
      if (paged_sets()) {
        pool_add_paged(p, e);
        SSIM_TOC(t0, kPhPool);
        return;
      }
    }
    if constexpr (kLaneSets) {
      if (lane_sets()) {
        pool_add_lanes(p, e);
        SSIM_TOC(t0, kPhPool);
        return;
      }
    }
    uint8_t* t = stage_table(p);
    ps_add<W>(pmeta(p), t, (uint32_t)e, S<int32_t>(O.sc_keys_b));
    unstage_table(p, t);
    SSIM_TOC(t0, kPhPool);
  }
  __device__ __forceinline__ void pool_remove(int p, int e) {
    SSIM_POOL_STAT(1, (int)W::uni(pool(p).mask) + 1, pool_size(p));
    SSIM_TIC(t0);
    if constexpr (kPagedSets) {
      if (paged_sets()) {
        check(pool_remove_paged(p, e));
        SSIM_TOC(t0, kPhPool);
        return;
      }
    }
    if constexpr (kLaneSets) {
      if (lane_sets()) {
        check(pool_remove_lanes(p, e));
        SSIM_TOC(t0, kPhPool);
        return;
      }
    }
    uint8_t* t = stage_table(p);
    const bool ok = ps_remove<W>(pmeta(p), t, (uint32_t)e);
    unstage_table(p, t);
    check(ok != 0);
    SSIM_TOC(t0, kPhPool);
  }

  __device__ __forceinline__ void move_to_pool(int e, int dst, bool send) {  // :186-220
    const int old = ex_loc(e);
    if (old >= 0) {
      pool_remove(old, e);
      ex_loc(e) = kPoolNone;
    }
    if (!send) {
      ex_loc(e) = (int16_t)dst;
      pool_add(dst, e);
      return;
    }
    const int g = pool_stage(dst);
    st_mov(g) += 1;
    const int oj = old >= 0 ? pool_job(old) : -1;
    const int nj = st_job(g);
    check(oj != nj);
    job_supply(nj) += 1;
    if (oj >= 0) {
      job_supply(oj) -= 1;
      check(job_supply(oj) >= 0);
    }
  }

  // Table order of set(e for e in pool.copy() if not busy) — _get_idle_source_executors (:714-728).
  __device__ __forceinline__ int idle_order(int p, int32_t* out) {
    if (p < 0) return 0;
    SSIM_POOL_STAT(2, (int)W::uni(pool(p).mask) + 1, pool_size(p));
    SSIM_COUNT(kCtIdleOrder);
    SSIM_TIC(t0);
    if constexpr (kPagedSets) {
      if (paged_sets()) {
        const int n = idle_order_paged(p, out);
        SSIM_TOC(t0, kPhPool);
        SSIM_TOC(t0, kPhIdleOrder);
        return n;
      }
    }
    if constexpr (kLaneSets) {
      if (lane_sets()) {
        const int n = idle_order_lanes(p, out);
        SSIM_TOC(t0, kPhPool);
        SSIM_TOC(t0, kPhIdleOrder);
        return n;
      }
    }
    const uint8_t* t = stage_table(p);
    const PySetMeta* m = pmeta(p);
    int n = ps_keys<W>(m, t, out);
    ps_copy_order<W>(m, out, n, S<uint8_t>(O.sc_tab_a));
    int k = 0;
    for (int i = 0; i < n; ++i) {
      const int e = ld(out + i);
      if (!ex_busy(e)) out[k++] = e;
    }
    n = k;
    ps_build_order<W>(out, n, S<uint8_t>(O.sc_tab_b), S<int32_t>(O.sc_keys_b));
    W::sync();
    SSIM_TOC(t0, kPhPool);
    SSIM_TOC(t0, kPhIdleOrder);
    return n;
  }

  // ---------------------------------------------------------------- events (event.py)
  // Register event slots (evr): (re)loaded from the executor records after the hot block is in place, and updated
  // together with the records by every writer of an event field (push_event, run_next_task_rec, pop_event, reset).
  __device__ __forceinline__ void ev_regs_load() {
    if constexpr (kEvPages > 0) {
#pragma unroll
      for (int p = 0; p < kEvPages; ++p) {
        const int e = 64 * p + W::lane();
        ExecRec r{};
        r.ev_seq = -1;
        r.ev_t = __builtin_inf();
        if (e < NE) r = exr(e);
        const uint64_t b = __builtin_bit_cast(uint64_t, r.ev_seq >= 0 ? r.ev_t : __builtin_inf());
        evr[p].tlo = (uint32_t)b;
        evr[p].thi = (uint32_t)(b >> 32);
        evr[p].seq = r.ev_seq >= 0 ? r.ev_seq : -1;
        evr[p].ts = ((int32_t)r.ev_type << 16) | (uint16_t)r.ev_stage;
      }
    }
    if (dc_on()) {  // the pending tasks' descriptors (independent gathers, one latency)
      for (int e = 0; e < kN; ++e) {
        const ExecRec x = ld_rec(exr(e));
        const bool task = x.ev_seq >= 0 && x.ev_type == kEvTask && x.ev_stage >= 0;
        const int ts = task ? (int)W::uni(stage(x.ev_stage).ts) : 0;
        dcache_store(e, dur_gather(ts));
      }
    }
  }
  __device__ __forceinline__ void ev_regs_set(int e, double t, int seq, int type, int g) {
    if constexpr (kEvPages > 0) {
      const uint64_t b = __builtin_bit_cast(uint64_t, t);
      const int l = e & 63, pg = e >> 6;
#pragma unroll
      for (int p = 0; p < kEvPages; ++p) {
        if (p == pg) {  // (uniform)
          evr[p].tlo = (uint32_t)W::writelane((int)(uint32_t)b, l, (int)evr[p].tlo);
          evr[p].thi = (uint32_t)W::writelane((int)(uint32_t)(b >> 32), l, (int)evr[p].thi);
          evr[p].seq = W::writelane(seq, l, evr[p].seq);
          evr[p].ts = W::writelane((type << 16) | (g & 0xFFFF), l, evr[p].ts);
        }
      }
    }
  }
  __device__ __forceinline__ void ev_regs_clear(int e) {
    if constexpr (kEvPages > 0) {
      const uint64_t b = __builtin_bit_cast(uint64_t, (double)__builtin_inf());
      const int l = e & 63, pg = e >> 6;
#pragma unroll
      for (int p = 0; p < kEvPages; ++p) {
        if (p == pg) {
          evr[p].tlo = (uint32_t)W::writelane((int)(uint32_t)b, l, (int)evr[p].tlo);
          evr[p].thi = (uint32_t)W::writelane((int)(uint32_t)(b >> 32), l, (int)evr[p].thi);
          evr[p].seq = W::writelane(-1, l, evr[p].seq);
        }
      }
    }
  }
  __device__ __forceinline__ void push_event(int e, double t, int type, int g) {
    check(ev_seq(e) < 0);  // at most one pending event per executor (DESIGN.md §Event queue)
    const int sq = h.seq++;
    ev_t(e) = t;
    ev_seq(e) = sq;
    ev_type(e) = (int16_t)type;
    ev_stage(e) = (int16_t)g;
    ev_regs_set(e, t, sq, type, g);
  }

  __device__ __forceinline__ void trace(double t, int kind, int e, int job, int sid, int seq) {
    const int cap = HP(trace_cap);
    if (cap == 0) return;  // tracing off: no bookkeeping at all
    TraceRec* const base = reinterpret_cast<TraceRec*>(obs + HP(ob_trace)) + (int64_t)eid * cap;
    if (h.trace_len < cap && W::lane() == 0) {
      TraceRec* r = base + h.trace_len;
      r->t = t;
      r->kind = kind;
      r->exec = e;
      r->job = job;
      r->stage = sid;
      r->seq = seq;
      r->pad = 0;
    }
    h.trace_len++;
  }

  // ---------------------------------------------------------------- sampler (tpch.py:75-106, 208-235)
  // The (wave x exec-level) duration-list descriptors of stage template `ts`: on device one lane-parallel
  // gather (lane l < 24 holds wave l/8, level l%8) issued together with the key metadata, so a task
  // launch pays two dependent dataset round trips (descriptors, then the drawn duration).
  struct DurDesc {
    int len, off;  // this lane's descriptor (device) — unused by a 1-lane build
  };
  // packed: offset << 8 | length (a missing list, length -1, stores 0: both mean "no draw")
  __device__ __forceinline__ void dcache_store(int e, const DurDesc& d) {
    if (W::lane() < 24)
      S<uint32_t>(O.sc_dcache)[e * 24 + W::lane()] = d.len > 0 ? ((uint32_t)d.off << 8) | (uint32_t)d.len : 0u;
  }
  __device__ __forceinline__ DurDesc dcache_load(int e) const {
    DurDesc d{0, 0};
    if (W::lane() < 24) {
      const uint32_t v = S<uint32_t>(O.sc_dcache)[e * 24 + W::lane()];
      d.len = (int)(v & 0xFFu);
      d.off = (int)(v >> 8);
    }
    return d;
  }
  __device__ __forceinline__ DurDesc dur_gather(int ts) const {
    DurDesc d{0, 0};
    if (W::kWidth >= 24) {
      const int32_t* const dlen = HP(dur_len);  // (uniform reads, before the lane-divergent loads)
      const int32_t* const doff = HP(dur_off);
      const int l = W::lane();
      if (l < 24) {
        const int idx = (ts * 3 + (l >> 3)) * kNumLevels + (l & 7);
        d.len = ldg(dlen, idx);
        d.off = ldg(doff, idx);
      }
    }
    return d;
  }
  __device__ __forceinline__ bool draw(int ts, const DurDesc& dd, int wave, int level, double* out) {
    int len, off;
    if (W::kWidth >= 24) {
      len = W::bcast_i(dd.len, wave * 8 + level);
      off = W::bcast_i(dd.off, wave * 8 + level);
    } else {
      const int idx = (ts * 3 + wave) * kNumLevels + level;
      len = ldu(HP(dur_len), idx);
      off = ldu(HP(dur_off), idx);
    }
    if (len <= 0) return false;  // KeyError (missing) or ValueError (empty): no RNG consumed
    SSIM_TIC(t0);
    const uint32_t k = rng.bounded((uint32_t)len);
    *out = ldu(HP(durations), off + (int)k);
    SSIM_TOC(t0, kPhDraw);
    return true;
  }

  // n_local = len(job.local_executors), ts = the stage's template stage, last = the executor's last task's
  // local stage (-1 = None), lid = this stage's local id, keymask / maxlevel = the stage record's copies of
  // the template stage's first_wave key set. The only dataset loads are the descriptor gather (issued first,
  // independent of the RNG) and the drawn duration; the executor key comes from Params::iv (scalar cache).
  __device__ __forceinline__ double task_duration(int n_local, int ts, int last, int lid, int keymask,
                                                  int maxlevel) {
    return task_duration_dd(n_local, ts, last, lid, keymask, maxlevel, dur_gather(ts));
  }
  // task_duration with the descriptor gather already issued (the task-completion path issues it when the
  // event is popped, so its latency overlaps the handler's LDS work)
  __device__ __forceinline__ double task_duration_dd(int n_local, int ts, int last, int lid, int keymask,
                                                     int maxlevel, const DurDesc& dd) {
    check(n_local > 0 && n_local < kIvRows);
    const int row = n_local < kIvRows ? n_local : 0;
    const uint32_t iv = (W::kWidth == 64 && row < 64) ? (uint32_t)W::bcast_i((int)iv_lane, row)
                                                      : W::uni(*reinterpret_cast<const uint32_t*>(IV[row]));
    const int lo = (int)(iv & 0xFF), hi = (int)((iv >> 8) & 0xFF);
    int level = (int)((iv >> 16) & 0xFF);  // key = lo
    if (lo != hi) {  // _sample_executor_key (tpch.py:216-235): one random() draw
      const int pt = 1 + (int)(rng.random() * (double)(hi - lo));
      if (!(pt <= n_local - lo)) level = (int)(iv >> 24);  // key = hi
    }
    if (level >= kNumLevels || !((keymask >> level) & 1)) level = maxlevel;
    double d = 0.0;
    if (last < 0) {
      if (draw(ts, dd, 0, level, &d)) return d;
      if (draw(ts, dd, 1, level, &d)) return d + HP(warmup_delay);
      fail(SSIM_ERR_SAMPLER);
      return 0.0;
    }
    if (last == lid) {
      if (draw(ts, dd, 2, level, &d)) return d;
    }
    if (draw(ts, dd, 1, level, &d)) return d;
    if (draw(ts, dd, 0, level, &d)) return d;
    fail(SSIM_ERR_SAMPLER);
    return 0.0;
  }

  // ---------------------------------------------------------------- schedulable-stage search (:505-555)
  // The dataset's DAG tables, read from HP in uniform control flow by the callers of the lane-parallel predicates.
  struct TopoView {
    const uint64_t* ts_topo;
    const int32_t *parent_base, *parents, *child_base, *children;
    bool bits;  // templates of <= 32 stages: parents / children as bit sets (ts_topo)
  };
  __device__ __forceinline__ TopoView topo_view() const {
    TopoView v{nullptr, nullptr, nullptr, nullptr, nullptr, HP(topo) != 0};
    if (v.bits) {  // (a uniform branch: only the tables the path uses are read)
      v.ts_topo = HP(ts_topo);
    } else {
      v.parent_base = HP(ts_parent_base);
      v.parents = HP(ts_parents);
      v.child_base = HP(ts_child_base);
      v.children = HP(ts_children);
    }
    return v;
  }
  __device__ __forceinline__ bool stage_pred(int g, int mode, int jx, int src_job, const TopoView& tv) const {
    const StageRec s = stage(g);  // one 16-B record read
    const int j = s.job;
    if (mode == kScanOnly && j != jx) return false;
    if (mode == kScanExcept && j == jx) return false;
    const JobRec& jr = job(j);
    if (!(j == src_job || jr.supply < NE)) return false;
    if (s.sel) return false;
    if (s.rem - (s.mov + s.com) <= 0) return false;
    const int base = jr.base;
    if (tv.bits) {  // one dataset load for all parents, then their records
      uint32_t pm = (uint32_t)ldg(tv.ts_topo, s.ts);
      while (pm) {
        const StageRec ps = stage(base + __builtin_ctz(pm));
        pm &= pm - 1;
        if (ps.rem - (ps.mov + ps.com) > 0) return false;
      }
      return true;
    }
    for (int k = ldg(tv.parent_base, s.ts); k < ldg(tv.parent_base, s.ts + 1); ++k) {
      const StageRec ps = stage(base + ldg(tv.parents, k));
      if (ps.rem - (ps.mov + ps.com) > 0) return false;
    }
    return true;
  }

  // Templates of <= 32 stages: the DAG neighbourhood of a stage as bit sets (ssim_dataset.ts_topo)
  __device__ __forceinline__ bool topo_masks() const { return HP(topo) != 0; }

  // first schedulable stage in node order, or -1
  __device__ __forceinline__ int scan_first(int mode, int jx, int src_job) {
    SSIM_TIC(t0);
    const int n = h.n_active_stages;
    const int16_t* act = H<int16_t>(O.active_stages);
    const TopoView tv = topo_view();
    int found = -1;
    for (int i0 = 0; i0 < n; i0 += W::kWidth) {
      const int i = i0 + W::lane();
      const int g = i < n ? act[i] : -1;
      const uint64_t m = W::ballot(g >= 0 && stage_pred(g, mode, jx, src_job, tv));
      if (m) {
        found = W::bcast_i(g, W::ffs(m));
        break;
      }
    }
    SSIM_TOC(t0, kPhScan);
    return found;
  }
  __device__ __forceinline__ bool any_schedulable() { return scan_first(kScanAll, -1, source_job()) >= 0; }

  __device__ __forceinline__ int find_backup(int e) {  // :821-845 (quirks Q1/Q2)
    const int jx = ex_job(e);
    check(jx >= 0);
    const int sj = (jx == 0 || jx < 0) ? source_job() : jx;  // `if not source_job_id`
    int g = scan_first(kScanOnly, jx, sj);
    if (g >= 0) return g;
    const bool others = h.n_active_jobs > ((jx >= 0 && job_state(jx) == kJobActive) ? 1 : 0);
    return scan_first(others ? kScanExcept : kScanAll, jx, sj);  // `if not job_ids`: [] -> all
  }

  // ---------------------------------------------------------------- list maintenance
  __device__ __forceinline__ void list_remove(int16_t* list, int n, int value) {  // ordered removal by wave shift
    int pos = -1;
    for (int i0 = 0; i0 < n && pos < 0; i0 += W::kWidth) {
      const int i = i0 + W::lane();
      const uint64_t m = W::ballot(i < n && list[i] == value);
      if (m) pos = i0 + W::ffs(m);
    }
    check(pos >= 0);
    if (pos < 0) return;
    for (int i0 = pos; i0 < n - 1; i0 += W::kWidth) {
      const int i = i0 + W::lane();
      const int16_t v = (i < n - 1) ? list[i + 1] : (int16_t)0;
      W::sync();
      if (i < n - 1) list[i] = v;
      W::sync();
    }
  }

  // ---------------------------------------------------------------- movement state machine
  __device__ __forceinline__ void detach(int j, int e) {  // job.py:84-89
    check(ex_job(e) == j);
    job_local(j) -= 1;
    ex_job(e) = -1;
    ex_task(e) = -1;
  }

  // _execute_next_task (:584-615) on register copies of the stage and executor records (ld_rec), which the
  // caller writes back: the task-completion path then costs one LDS access per record, not one per field.
  __device__ __forceinline__ void run_next_task_rec(int e, int g, StageRec& s, ExecRec& x) {
    run_next_task_rec(e, g, s, x, dur_gather(s.ts));
  }
  __device__ __forceinline__ void run_next_task_rec(int e, int g, StageRec& s, ExecRec& x, const DurDesc& dd) {
    const int j = s.job;
    check(s.rem > 0);
    check(x.job == j);
    check(!x.busy);
    s.rem = (int16_t)(s.rem - 1);
    s.exe = (int16_t)(s.exe + 1);
    const JobRec jr = ld_rec(job(j));
    if (s.rem == 0) job_sat(j) = (int16_t)(jr.sat + 1);
    SSIM_TIC(t_smp);
    SSIM_COUNT(kCtTask);
    const int lid = g - jr.base;
    SSIM_MARK("sample_begin");
    const double dur = task_duration_dd(jr.local, s.ts, x.task, lid, s.fw_keymask, s.fw_maxlevel, dd);
    SSIM_MARK("sample_end");
    SSIM_TOC(t_smp, kPhSample);
    x.task = (int16_t)lid;
    x.busy = 1;
    st_recent(g) = dur;
    check(x.ev_seq < 0);  // at most one pending event per executor
    x.ev_t = h.wall + dur;
    x.ev_seq = h.seq++;
    x.ev_type = (int16_t)kEvTask;
    x.ev_stage = (int16_t)g;
    ev_regs_set(e, x.ev_t, x.ev_seq, kEvTask, g);
  }
  __device__ __forceinline__ void run_next_task(int e, int g) {  // :584-615
    SSIM_FIELD_STAT(11);
    const StageRec sraw = stage(g);  // both records in one LDS round trip
    const ExecRec xraw = exr(e);
    StageRec s = ld_rec(sraw);
    ExecRec x = ld_rec(xraw);
    const DurDesc dd = dur_gather(s.ts);
    if (dc_on()) dcache_store(e, dd);
    run_next_task_rec(e, g, s, x, dd);
    stage(g) = s;
    exr(e) = x;
  }

  __device__ __forceinline__ void send(int e, int g) {  // :617-637
    check(!ex_busy(e));
    check(ex_job(e) != st_job(g));
    move_to_pool(e, stage_pool(g), true);
    if (ex_job(e) >= 0) detach(ex_job(e), e);
    push_event(e, h.wall + HP(moving_delay), kEvReady, g);
  }

  // _move_idle_executors (:745-782) with an explicit executor list (n ids in `ids`).
  __device__ __forceinline__ void release_idle_list(int src, const int32_t* ids, int n) {
    if (src < 0) src = h.source;
    check(src >= 0);
    if (src <= kPoolCommon) return;
    check(n > 0);
    const int j = pool_job(src);
    const bool sat = job_sat(j) == job_nst(j);
    if (!is_stage_pool(src) && !sat) return;
    const int dst = sat ? kPoolCommon : job_pool(j);
    for (int k = 0; k < n; ++k) {
      const int e = ld(ids + k);
      move_to_pool(e, dst, false);
      if (dst == kPoolCommon) {
        detach(j, e);
        if (HP(trace_cap) > 0) trace(h.wall, kTrToCommon, e, j, -1, -1);
      }
    }
  }
  __device__ __forceinline__ void release_idle_one(int src, int e) {
    int32_t one = e;
    release_idle_list(src, &one, 1);
  }
  __device__ __forceinline__ void release_idle_all(int src) {
    if (src < 0) src = h.source;
    check(src >= 0);
    if (src <= kPoolCommon) return;
    int32_t* ids = S<int32_t>(O.sc_keys_a);
    const int n = idle_order(src, ids);
    release_idle_list(src, ids, n);
  }

  __device__ __forceinline__ void goto_stage(int e, int g) {  // _move_executor_to_stage :799-819 (+ backup loop)
    for (int guard = 0; guard < 4 * SC + 8; ++guard) {
      SSIM_FIELD_STAT(11);
      const StageRec sraw = stage(g);  // the stage record and the executor's job in one LDS round trip
      const int16_t xjob = exr(e).job;
      const StageRec sr = ld_rec(sraw);
      if (sr.rem == 0) {  // _try_backup_schedule :784-797
        const int b = find_backup(e);
        if (b >= 0) {
          g = b;
          continue;
        }
        release_idle_one(ex_loc(e), e);
        return;
      }
      const int j = sr.job;
      if (W::uni(xjob) != j) {
        send(e, g);
        return;
      }
      if (sr.unmet != 0) {  // not in job.frontier_stages
        ex_task(e) = -1;
        move_to_pool(e, job_pool(j), false);
        return;
      }
      move_to_pool(e, stage_pool(g), false);
      run_next_task(e, g);
      return;
    }
    fail(SSIM_ERR_INVARIANT);
  }

  __device__ __forceinline__ void fulfill(int e, int dst) {  // :699-712
    const int src = remove_commitment(e, dst);
    if (dst == kPoolCommon) {
      release_idle_one(src, e);
      return;
    }
    goto_stage(e, pool_stage(dst));
  }

  __device__ __forceinline__ void fulfill_from_source() {  // :730-743
    int32_t* idle = S<int32_t>(O.sc_keys_a);
    int32_t* plan = S<int32_t>(O.sc_plan);
    const int n_idle = idle_order(h.source, idle);
    const int n_plan = h.source >= 0 ? commit_plan(h.source, plan) : 0;
    int k = 0;
    for (int c = 0; c < n_plan; ++c) {
      const int dst = ld(plan + 2 * c);
      int n = ld(plan + 2 * c + 1);
      check(dst >= 0 && n > 0);
      while (n > 0 && k < n_idle && !frozen()) {
        const int e = ld(idle + k++);
        fulfill(e, dst);
        n--;
      }
    }
    check(k == n_idle);
  }

  __device__ __forceinline__ void commit_leftovers() {  // :487-503
    const int n = committable();
    if (n > 0) add_commitment(n, kPoolCommon);
  }

  __device__ __forceinline__ bool release(int e, int g, bool changed) {  // _handle_released_executor :639-660
    const int dst = peek_commitment(stage_pool(g));
    if (dst != kPoolNone) {
      fulfill(e, dst);
      return true;
    }
    ex_task(e) = -1;
    if (changed) release_idle_one(stage_pool(g), e);
    return false;
  }

  // ---------------------------------------------------------------- event handlers (:428-483)
  __device__ __forceinline__ void on_job_arrival(int j) {
    job_state(j) = kJobActive;
    job_arr_dec(j) = h.decisions;
    int16_t* aj = H<int16_t>(O.active_jobs);
    int16_t* as = H<int16_t>(O.active_stages);
    if (W::lane() == 0) aj[h.n_active_jobs] = (int16_t)j;
    const int base = job_base(j), n = job_nst(j), tsb = ldu(HP(tpl_stage_base), (int)job_tpl(j));
    const int32_t* const nt = HP(ts_num_tasks);  // (uniform reads, before the lane-divergent block)
    const int32_t* const pb = HP(ts_parent_base);
    const int32_t* const fwk = HP(ts_fw_keymask);
    const int32_t* const fwm = HP(ts_fw_maxlevel);
    const double* const rough = HP(ts_rough);
    for (int k0 = 0; k0 <= n; k0 += W::kWidth) {  // stage records, pools of the job and its stages, active list
      const int k = k0 + W::lane();
      if (k <= n) {
        const int p = (k == n) ? job_pool(j) : stage_pool(base + k);
        ps_init(pmeta(p), pool(p).tab);
        cfrom(p) = 0;
        if (k < n) {
          const int g = base + k, ts = tsb + k;
          StageRec r;
          r.job = (int16_t)j;
          r.ts = (int16_t)ts;
          r.rem = (int16_t)ldg(nt, ts);
          r.exe = 0;
          r.mov = 0;
          r.com = 0;
          r.unmet = (int8_t)(ldg(pb, ts + 1) - ldg(pb, ts));
          r.sel = 0;
          r.fw_keymask = (uint8_t)ldg(fwk, ts);
          r.fw_maxlevel = (uint8_t)ldg(fwm, ts);
          stage(g) = r;
          recent()[g] = ldg(rough, ts);
          as[h.n_active_stages + k] = (int16_t)g;
        }
      }
    }
    W::sync();
    h.n_active_jobs += 1;
    h.n_active_stages += n;
    if (pool_size(kPoolCommon) > 0) h.source = kPoolCommon;
  }

  __device__ __forceinline__ void on_executor_arrival(int e, int g) {  // :440-450
    SSIM_FIELD_STAT(11);
    const StageRec sraw = stage(g);  // stage and executor records in one LDS round trip
    const ExecRec xraw = exr(e);
    const StageRec sr = ld_rec(sraw);
    const int j = sr.job;
    check(W::uni(xraw.task) < 0);  // Job.attach_executor asserts executor.task is None
    job_local(j) += 1;
    ex_job(e) = (int16_t)j;
    st_mov(g) = (int16_t)(sr.mov - 1);
    check(sr.mov - 1 >= 0);
    move_to_pool(e, job_pool(j), false);
    goto_stage(e, g);
  }

  __device__ __forceinline__ bool stage_completed(int j, int g) {  // Job.record_stage_completion (job.py:65-73,113-128)
    check(st_unmet(g) == 0);  // frontier_stages.remove(stage)
    list_remove(H<int16_t>(O.active_stages), h.n_active_stages, g);
    h.n_active_stages -= 1;
    job_nact(j) -= 1;
    const int ts = st_ts(g), base = job_base(j);
    bool changed = false;
    if (topo_masks()) {
      uint32_t cm = (uint32_t)(ldu(HP(ts_topo), ts) >> 32);
      while (cm) {
        const int c = base + __builtin_ctz(cm);
        cm &= cm - 1;
        st_unmet(c) -= 1;
        if (st_unmet(c) == 0 && !st_completed(c)) changed = true;
      }
      return changed;
    }
    const int kb = ldu(HP(ts_child_base), ts), ke = ldu(HP(ts_child_base), ts + 1);
    for (int k = kb; k < ke; ++k) {
      const int c = base + ldu(HP(ts_children), k);
      st_unmet(c) -= 1;
      if (st_unmet(c) == 0 && !st_completed(c)) changed = true;
    }
    return changed;
  }

  __device__ __forceinline__ void job_completed(int j) {  // :682-697
    if (pool_size(job_pool(j)) > 0) release_idle_all(job_pool(j));
    check(pool_size(job_pool(j)) == 0);
    list_remove(H<int16_t>(O.active_jobs), h.n_active_jobs, j);
    h.n_active_jobs -= 1;
    h.n_completed += 1;
    job_state(j) = kJobDone;
    job_tdone(j) = h.wall;
    job_done_dec(j) = h.decisions;
    trace(h.wall, kTrJobDone, -1, j, -1, -1);
  }

  // `s` = the stage record (read when the event was popped), `dd` = its duration descriptors, in flight
  __device__ __forceinline__ void on_task_done(int e, int g, StageRec s, ExecRec x, const DurDesc& dd) {  // :452-483
    SSIM_MARK("task_done_begin");
    const int j = s.job;
    check(!(s.rem == 0 && s.exe == 0));
    s.exe = (int16_t)(s.exe - 1);
    x.busy = 0;
    if (s.rem > 0) {  // the common case: the executor takes the stage's next task
      run_next_task_rec(e, g, s, x, dd);
      stage(g) = s;
      exr(e) = x;
      SSIM_MARK("task_done_fast_end");
      return;
    }
    stage(g) = s;
    exr(e) = x;
    SSIM_TIC(t_sd);
    bool changed = false;
    if (st_completed(g)) changed = stage_completed(j, g);
    SSIM_TOC(t_sd, kPhStageDone);
    if (job_nact(j) == 0) job_completed(j);
    const bool had = release(e, g, changed);
    if (changed)
      h.source = job_pool(j);
    else if (!had)
      h.source = stage_pool(g);
  }

  // Pops the min (t, seq) event: arrival cursor vs. per-executor slots. Returns false when empty.
  // Each lane loads its executor's record; one wave argmin (W::argmin_event: DPP min of t, ties by seq)
  // picks the winner, whose type / stage / seq are read from the winning lane's registers.
  __device__ __forceinline__ bool pop_event(double* t, int* kind, int* e, int* g, int* seq) {
    constexpr int kSpan = W::kWidth < 16 ? W::kWidth : (kN > 0 && kN <= 16) ? 16 : 64;
    double bt = 0.0;
    int bseq = 0x7FFFFFFF, be = -1, btype = 0, bstage = -1;
    const bool have_arr = h.arrivals < h.num_jobs;
    // the next arrival's time: read per lane and made uniform only where it is compared, so its LDS read is in
    // flight together with the executor records' instead of being waited on first (+1%; also fetching the job
    // record with the stage's and executor's, its id taken from the pop, measured -0.5%: profiles/r02/ab_lds_overlap.log)
    const double ta_lane = have_arr ? jtimes(h.arrivals).tarr : 0.0;
    bool scanned = false;
    if constexpr (kEvPages > 0) {
      if (ev_in_regs()) {  // the register event slots: no memory read
        scanned = true;
#pragma unroll
        for (int p = 0; p < kEvPages; ++p) {
          if (64 * p >= NE) break;
          const EvRegs r = evr[p];
          const double tv = __builtin_bit_cast(double, ((uint64_t)r.thi << 32) | r.tlo);
          double tt;
          const int l = W::template argmin_event<kSpan>(tv, r.seq, r.seq >= 0, &tt);
          if (l < 0) continue;
          const int ss = W::bcast_i(r.seq, l);
          if (be < 0 || tt < bt || (tt == bt && ss < bseq)) {
            bt = tt;
            bseq = ss;
            be = 64 * p + l;
            const int ts = W::bcast_i(r.ts, l);
            btype = ts >> 16;
            bstage = (int16_t)(ts & 0xFFFF);
          }
        }
      }
    }
    for (int k0 = 0; !scanned && k0 < NE; k0 += kSpan) {
      const int k = k0 + W::lane();
      ExecRec r{};
      r.ev_seq = -1;
      if (k < NE && W::lane() < kSpan) r = exr(k);
      double tt;
      const int l = W::template argmin_event<kSpan>(r.ev_t, r.ev_seq, r.ev_seq >= 0, &tt);
      if (l < 0) continue;
      const int ss = W::bcast_i(r.ev_seq, l);
      if (be < 0 || tt < bt || (tt == bt && ss < bseq)) {
        bt = tt;
        bseq = ss;
        be = k0 + l;
        btype = W::bcast_i(r.ev_type, l);
        bstage = W::bcast_i(r.ev_stage, l);
      }
    }
    if (have_arr) {
      const double ta = W::uni(ta_lane);
      const int sa = h.arrivals;  // arrivals were pushed first with seq 0..J-1
      if (be < 0 || ta < bt || (ta == bt && sa < bseq)) {
        *t = ta;
        *kind = kEvArrival;
        *e = -1;
        *g = h.arrivals;  // job id
        *seq = sa;
        h.arrivals++;
        return true;
      }
    }
    if (be < 0) return false;
    *t = bt;
    *kind = btype;
    *e = be;
    *g = bstage;
    *seq = bseq;
    ev_seq(be) = -1;
    ev_regs_clear(be);
    return true;
  }

  // kSimDecision when it stopped at a decision point (committable executors and a schedulable stage), kSimIdle
  // when the queue ran dry (or the env froze), kSimPreempted when `stop` fired between two events (the state is
  // then exactly the reference's between those events; a later call continues the loop).
  // The stop condition is a read of one shared word (TicketStop): polled every kStopEvery-th event, issued one
  // event before it is tested so its latency hides behind that event. A launch ends when its last wave has seen the
  // flag, so the poll interval is the launch's tail. Round 6 (50 timed 20-step launches per run, low-noise,
  // `profiles/r06/ab_stop_poll/`): every event 3.21·10⁷ vs every 8th 3.12·10⁷ decisions/s on the driver's window,
  // +0.9% at 300 steps, +1.1% on configs[3], configs[2] within noise (round 2's and 5's single-window A/Bs could not
  // resolve it).
#ifndef SSIM_STOP_EVERY
#define SSIM_STOP_EVERY 1
#endif
  static constexpr int kStopEvery = SSIM_STOP_EVERY;  // a power of two
  template <class Stop>
  __device__ __forceinline__ int simulate(const Stop& stop) {  // _resume_simulation :320-343
    uint64_t tk = 0;
    int n = 0;
    for (;;) {
      if (frozen()) return kSimIdle;
      if (Stop::kCan) {
        const int ph = n++ & (kStopEvery - 1);
        if (ph == 0 && n > 1 && stop.hit(tk)) return kSimPreempted;  // the value issued one event ago
        if (ph == kStopEvery - 1) tk = stop.issue();
      }
      double t;
      int kind, e, g, seq;
      SSIM_TIC(t_pop);
      SSIM_MARK("pop_begin");
      const bool have = pop_event(&t, &kind, &e, &g, &seq);
      SSIM_MARK("pop_end");
      SSIM_TOC(t_pop, kPhPop);
      if (!have) return kSimIdle;
      SSIM_TIC(t_h);
      h.wall = t;
      h.events++;
      h.step_events++;
      if (kind == kEvArrival) {
        if (HP(trace_cap) > 0) trace(t, kind, -1, g, -1, seq);
        SSIM_TIC(t_a);
        on_job_arrival(g);
        SSIM_TOC(t_a, kPhJobArr);
      } else {
        if (HP(trace_cap) > 0) {
          const int j = st_job(g);
          trace(t, kind, e, j, g - job_base(j), seq);
        }
        SSIM_TIC(t_x);
        if (kind == kEvReady) {
          on_executor_arrival(e, g);
          SSIM_TOC(t_x, kPhExecArr);
        } else {
          // the stage and executor records (and the cached duration descriptors) are read together (one LDS round
          // trip), then made uniform
          SSIM_FIELD_STAT(11);
          const StageRec sraw = stage(g);
          const ExecRec xraw = exr(e);
          DurDesc ddc{0, 0};
          if (dc_on()) ddc = dcache_load(e);
          const StageRec sr = ld_rec(sraw);
          if (!dc_on() && sr.rem > 0) ddc = dur_gather(sr.ts);
          // the next task's duration descriptors (if the stage has tasks left): issued now, used after the job
          // record read
          on_task_done(e, g, sr, ld_rec(xraw), ddc);
          SSIM_TOC(t_x, kPhTaskDone);
        }
      }
      SSIM_TOC(t_h, kPhHandle);
      SSIM_TIC(t_s);
      if (committable() == 0) {
        SSIM_TOC(t_s, kPhPostScan);
        continue;
      }
      const bool found = any_schedulable();
      if (!found) {
        release_idle_all(kPoolNone);
        h.source = kPoolNone;
      }
      SSIM_TOC(t_s, kPhPostScan);
      if (found) return kSimDecision;
    }
  }

  __device__ __forceinline__ double jobtime(double t0, int dec) {  // _compute_jobtime :847-874
    const double span = h.wall - t0;
    if (span == 0.0) return 0.0;
    double part = 0.0;
    const double beta = HP(beta);
    for (int j0 = 0; j0 < h.arrivals; j0 += W::kWidth) {
      const int j = j0 + W::lane();
      if (j < h.arrivals) {
        const JobRec jr = job(j);
        const JobTimes jt = jtimes(j);
        const int st = jr.state;
        const bool in_union = st == kJobActive || (st == kJobDone && jr.done_dec == dec && jr.arr_dec < dec);
        if (in_union) {
          const double ta = jt.tarr;
          const double a = ta > t0 ? ta : t0;
          const double tc = st == kJobDone ? jt.tdone : h.wall;
          const double b = tc < h.wall ? tc : h.wall;
          if (beta == 0.0)
            part += b - a;
          else
            part += exp(-beta * 1e-3 * (a - t0)) - exp(-beta * 1e-3 * (b - t0));
        }
      }
    }
    double total = W::sum_d(part);
    if (beta > 0.0) total /= beta;
    return total;
  }

  // ---------------------------------------------------------------- observation (:345-406, utils.py)
  // Observation-arena stores. SSIM_NT_OBS=1 makes them non-temporal (they are never read back by the kernel); measured
  // on every workload it changed no rate and tripled the HBM write bytes (partial-line streaming writes), so it is off.
#ifndef SSIM_NT_OBS
#define SSIM_NT_OBS 0
#endif
  template <class T>
  __device__ __forceinline__ static void obs_st(T* p, T v) {
    if constexpr (SSIM_NT_OBS && W::kWidth == 64)
      W::st_nt(p, v);
    else
      *p = v;
  }
  __device__ __forceinline__ void observe(double reward) {
    const int n = h.n_active_stages;
    const int src_job = source_job();
    const int16_t* act = H<int16_t>(O.active_stages);
    int16_t* sched = H<int16_t>(O.sched_list);
    int16_t* row_of = row_lds ? S<int16_t>(O.sc_row_of) : reinterpret_cast<int16_t*>(cold + O.row_of);
    float* nodes = reinterpret_cast<float*>(obs + HP(ob_nodes)) + (int64_t)eid * SC * 3;
    uint8_t* front = obs + HP(ob_frontier) + (int64_t)eid * SC;
    int32_t* srank = reinterpret_cast<int32_t*>(obs + HP(ob_sched_rank)) + (int64_t)eid * SC;
    const TopoView tv = topo_view();
    const int ecap = HP(edge_cap);
    // picks[j] (job id j): heuristics/utils.py find_stage of the job, packed as a min key over its
    // schedulable nodes: (frontier ? 0 : 1 << 16) | schedulable rank; INT32_MAX = none. Nodes of a job are
    // contiguous in node order and ranks grow with node order, so the min is the first frontier stage,
    // else the first schedulable one.
    const int16_t* ajl = H<int16_t>(O.active_jobs);
    for (int k0 = 0; k0 < h.n_active_jobs; k0 += W::kWidth) {
      const int k = k0 + W::lane();
      if (k < h.n_active_jobs) job(ajl[k]).pick = 0x7FFFFFFF;
    }
    W::sync();
    int nsched = 0;
    for (int i0 = 0; i0 < n; i0 += W::kWidth) {
      const int i = i0 + W::lane();
      const bool ok = i < n;
      const int g = ok ? act[i] : -1;
      const bool s = ok && stage_pred(g, kScanAll, -1, src_job, tv);
      const uint64_t m = W::ballot(s);
      const int r = nsched + W::rank(m);
      if (ok) {
        const StageRec sr = stage(g);
        obs_st(nodes + 3 * i + 0, (float)sr.rem);
        obs_st(nodes + 3 * i + 1, (float)recent()[g]);
        obs_st(nodes + 3 * i + 2, s ? 1.0f : 0.0f);
        obs_st(front + i, (uint8_t)(sr.unmet == 0 ? 1 : 0));
        obs_st(srank + i, s ? r : -1);
        row_of[g] = (int16_t)i;
        if (s) {
          sched[r] = (int16_t)g;
          W::amin(&job(sr.job).pick, (sr.unmet == 0 ? 0 : 0x10000) | r);
        }
      }
      nsched += W::popc(m);
    }
    W::sync();
    // jobs: dag_ptr, exec_supplies, source_job_idx
    const int nj = h.n_active_jobs;
    const int16_t* aj = H<int16_t>(O.active_jobs);
    int32_t* ptr = reinterpret_cast<int32_t*>(obs + HP(ob_dag_ptr)) + (int64_t)eid * (JC + 1);
    int32_t* sup = reinterpret_cast<int32_t*>(obs + HP(ob_supplies)) + (int64_t)eid * JC;
    int src_idx = nj, run = 0;
    for (int k0 = 0; k0 < nj; k0 += W::kWidth) {
      const int k = k0 + W::lane();
      const bool ok = k < nj;
      const int j = ok ? aj[k] : -1;
      const JobRec jr = ok ? job(j) : JobRec{};
      const int cnt = ok ? jr.nact : 0;
      int total = 0;
      const int ex = W::excl_scan(cnt, &total);
      if (ok) {
        obs_st(ptr + k, run + ex);
        obs_st(sup + k, (int32_t)jr.supply);
      }
      const uint64_t ms = W::ballot(ok && j == src_job);
      if (ms) src_idx = k0 + W::ffs(ms);
      run += total;
    }
    if (W::lane() == 0) obs_st(ptr + nj, run);
    check(run == n);
    // edges: (row(u), row(v)) for active u, child v active; order = node order, children ascending
    int64_t* links = reinterpret_cast<int64_t*>(obs + HP(ob_edge_links)) + (int64_t)eid * ecap * 2;
    int ne = 0;
    for (int i0 = 0; i0 < n; i0 += W::kWidth) {
      const int i = i0 + W::lane();
      const bool ok = i < n;
      const int g = ok ? act[i] : -1;
      int cnt = 0, cb = 0, ce = 0, base = 0;
      uint32_t live = 0;  // (bit-set path) the children that are not completed, ascending local id
      if (ok) {
        const StageRec sr = stage(g);
        base = job(sr.job).base;
        if (tv.bits) {
          uint32_t cm = (uint32_t)(ldg(tv.ts_topo, sr.ts) >> 32);
          while (cm) {
            const int b = __builtin_ctz(cm);
            cm &= cm - 1;
            const StageRec c = stage(base + b);
            if (!(c.rem == 0 && c.exe == 0)) live |= 1u << b;
          }
          cnt = __builtin_popcount(live);
        } else {
          cb = ldg(tv.child_base, sr.ts);
          ce = ldg(tv.child_base, sr.ts + 1);
          for (int k = cb; k < ce; ++k) {
            const StageRec c = stage(base + ldg(tv.children, k));
            if (!(c.rem == 0 && c.exe == 0)) cnt++;
          }
        }
      }
      int total = 0;
      const int ex = W::excl_scan(cnt, &total);
      if (ok) {
        int o = ne + ex;
        if (tv.bits) {
          while (live && o < ecap) {
            const int c = base + __builtin_ctz(live);
            live &= live - 1;
            obs_st(links + 2 * o + 0, (int64_t)i);
            obs_st(links + 2 * o + 1, (int64_t)row_of[c]);
            o++;
          }
        } else {
          for (int k = cb; k < ce; ++k) {
            const int c = base + ldg(tv.children, k);
            const StageRec cr = stage(c);
            if (!(cr.rem == 0 && cr.exe == 0) && o < ecap) {
              obs_st(links + 2 * o + 0, (int64_t)i);
              obs_st(links + 2 * o + 1, (int64_t)row_of[c]);
              o++;
            }
          }
        }
      }
      ne += total;
    }
    if (ne > ecap) fail(SSIM_ERR_CAPACITY);
    h.n_sched = nsched;
    h.src_idx = src_idx;
    h.stage_idx_n = n + 1;
    EnvAcc a = ld_rec(*H<EnvAcc>(O.acc));
    a.nodes += n;
    a.edges += ne;
    a.jobs += nj;
    a.events += h.step_events;
    *H<EnvAcc>(O.acc) = a;
    int64_t* const acc = reinterpret_cast<int64_t*>(obs + HP(ob_acc)) + (int64_t)eid * kNumAcc;
    int32_t* const cnts = reinterpret_cast<int32_t*>(obs + HP(ob_counts)) + (int64_t)eid * SSIM_NUM_COUNTS;
    double* const rew = reinterpret_cast<double*>(obs + HP(ob_reward)) + eid;
    double* const wall = reinterpret_cast<double*>(obs + HP(ob_wall_time)) + eid;
    const int ncommit = committable();
    W::sync();
    if (W::lane() == 0) {
      acc[0] = a.nodes;
      acc[1] = a.edges;
      acc[2] = a.jobs;
      acc[3] = a.events;
      acc[4] = a.decisions;
      acc[5] = a.episodes;
      acc[6] = 0;
      acc[7] = 0;
      cnts[SSIM_OC_NUM_NODES] = n;
      cnts[SSIM_OC_NUM_EDGES] = ne;
      cnts[SSIM_OC_NUM_JOBS] = nj;
      cnts[SSIM_OC_COMMITTABLE] = ncommit;
      cnts[SSIM_OC_SOURCE_JOB_IDX] = src_idx;
      cnts[SSIM_OC_NUM_SCHEDULABLE] = nsched;
      cnts[SSIM_OC_TERMINATED] = h.terminated;
      cnts[SSIM_OC_TRUNCATED] = h.wall >= h.time_limit ? 1 : 0;
      cnts[SSIM_OC_ERR] = (int32_t)h.err;
      cnts[SSIM_OC_DECISIONS] = h.decisions;
      cnts[SSIM_OC_EVENTS] = h.events;
      cnts[SSIM_OC_NUM_COMPLETED] = h.n_completed;
      cnts[SSIM_OC_NUM_ARRIVED] = h.arrivals;
      cnts[SSIM_OC_TRACE_LEN] = h.trace_len;
      cnts[SSIM_OC_STEP_EVENTS] = h.step_events;
      cnts[SSIM_OC_EPISODE] = h.episode;
      *rew = reward;
      *wall = h.wall;
    }
    W::sync();
  }

  __device__ __forceinline__ void write_err_only(uint32_t transient) {
    int32_t* const cnts = reinterpret_cast<int32_t*>(obs + HP(ob_counts)) + (int64_t)eid * SSIM_NUM_COUNTS;
    W::sync();
    if (W::lane() == 0) {
      cnts[SSIM_OC_ERR] = (int32_t)(h.err | transient);
    }
    W::sync();
  }

  // ---------------------------------------------------------------- step (:188-221, :275-315)
  // Requires the hot block in place (load_hot() by the caller for LDS residency).
  __device__ __forceinline__ void step(StepIn a) {
    load_header();
    step_loaded(a);
  }
  __device__ __forceinline__ bool idle() const { return h.terminated || frozen() || h.num_jobs == 0; }
  __device__ __forceinline__ EnvAcc& acc() const { return *H<EnvAcc>(O.acc); }
  __device__ __forceinline__ bool pending() const { return W::uni(acc().pending) != 0; }
  __device__ __forceinline__ void count_decision() {  // a step completed (its observation is written)
    UF<int64_t> d{&acc().decisions};
    d = (int64_t)d + 1;
  }
  // The end of a step from its simulation on: returns false if `stop` preempted it (pending, see EnvAcc).
  template <class Stop>
  __device__ __forceinline__ bool finish_step(double t0, const Stop& stop) {
    const int r = simulate(stop);
    if (Stop::kCan && r == kSimPreempted) {
      W::sync();
      if (W::lane() == 0) {
        acc().pend_t0 = t0;
        acc().pending = 1;
      }
      store_header();
      write_err_only(SSIM_ERR_PENDING);
      return false;
    }
    const double reward = -jobtime(t0, h.decisions);
    h.terminated = (h.n_completed == h.num_jobs) ? 1 : 0;
    // step's `assert committable and schedulable_stages` (:212-215): simulate() stopped at a decision
    // point (state untouched since) unless the queue ran dry
    if (!h.terminated) check(r == kSimDecision);
    count_decision();  // before observe(), which publishes the accumulators to the obs arena
    SSIM_TIC(t_o);
    observe(reward);
    SSIM_TOC(t_o, kPhObserve);
    store_header();
    return true;
  }
  // The pending step's reward-interval start; clears the pending mark (the caller then runs finish_step).
  __device__ __forceinline__ double take_pending() {
    const double t0 = W::uni(acc().pend_t0);
    W::sync();
    if (W::lane() == 0) acc().pending = 0;
    W::sync();
    return t0;
  }
  // Completes a step preempted by an earlier launch (header loaded); true if none was pending or it completed.
  template <class Stop>
  __device__ __forceinline__ bool resume(const Stop& stop) {
    if (!pending()) return true;
    return finish_step(take_pending(), stop);
  }
  // The last step_begin refused its action (ValueError / KeyError in the reference): the state is untouched and no
  // observation was written, only the error bits of the obs arena.
  bool rejected = false;
  // step() with the header already in registers. Returns false when `stop` preempted the step's simulation (the
  // step stays pending until resume()).
  template <class Stop = NoStop>
  __device__ __forceinline__ bool step_loaded(StepIn a, const Stop& stop = Stop()) {
    double t0;
    if (!step_begin(a, &t0)) return true;
    return finish_step(t0, stop);
  }
  // The first part of a step: the action (:275-315) and, if the round continues, the observation. Returns true
  // when the step goes on to simulate (finish_step from *t0), false when it is complete (or rejected / idle).
  // The fused rollout calls step_begin and finish_step from one loop, so finish_step (the event loop, the
  // observation) is inlined once whether a launch starts a step or completes a preempted one.
  __device__ __forceinline__ bool step_begin(StepIn a, double* t0) {
    rejected = false;
    if (h.terminated || frozen() || h.num_jobs == 0) return false;
    SSIM_TIC(t_act);
    const int idx = a.stage_idx, nx = a.num_exec;
    // Discrete(n, start=-1) holds -1 .. n-2; Discrete(N, start=1) holds 1 .. N
    if (idx < -1 || idx > h.stage_idx_n - 2 || nx < 1 || nx > NE) {
      write_err_only(SSIM_ERR_SPACE);
      rejected = true;
      return false;
    }
    if (idx == -1) {
      commit_leftovers();
    } else {
      if (idx >= h.n_sched) {
        write_err_only(SSIM_ERR_KEY);
        rejected = true;
        return false;
      }
      const int g = ld(H<int16_t>(O.sched_list) + idx);
      if (nx > committable()) {
        write_err_only(SSIM_ERR_TOO_MANY);
        rejected = true;
        return false;
      }
      const int d = demand(g);
      const int n = nx < d ? nx : d;  // _adjust_num_executors
      check(n > 0);
      add_commitment(n, stage_pool(g));
      st_sel(g) = 1;
      if (h.n_selected <= NE) {
        if (W::lane() == 0) H<int16_t>(O.sel_list)[h.n_selected] = (int16_t)g;
        h.n_selected++;
      } else {
        fail(SSIM_ERR_CAPACITY);
      }
      W::sync();
    }
    h.decisions++;
    h.step_events = 0;
    SSIM_TOC(t_act, kPhAction);
    SSIM_TIC(t_rc);
    const bool round_continues = committable() > 0 && any_schedulable();
    SSIM_TOC(t_rc, kPhRoundCheck);
    if (round_continues) {
      count_decision();
      SSIM_TIC(t_o);
      observe(0.0);
      SSIM_TOC(t_o, kPhObserve);
      store_header();
      return false;
    }
    SSIM_TIC(t_f);
    commit_leftovers();
    fulfill_from_source();
    SSIM_TOC(t_f, kPhFulfill);
    h.source = kPoolNone;
    {  // selected_stages.clear()
      const int16_t* sl = H<int16_t>(O.sel_list);
      for (int k0 = 0; k0 < h.n_selected; k0 += W::kWidth) {
        const int k = k0 + W::lane();
        if (k < h.n_selected) st_sel(sl[k]) = 0;
      }
      h.n_selected = 0;
      W::sync();
    }
    *t0 = h.wall;
    return true;
  }

  // ---------------------------------------------------------------- device-side reset sampling
  // TPCHDataSampler.job_sequence (tpch.py:54-73) on the env's RNG `rng`: per job integers(22) + 1 (query),
  // choice(QUERY_SIZES) (= integers(0, 7)), arrival t, then t += exponential(1 / rate) (drawn after every
  // job, the last included), while t < time_limit and under the arrival cap. Writes the arrival times and
  // template ids of the env's reset record (HBM, lane 0) and returns the job count (-1: over job_cap).
  __device__ __forceinline__ int sample_job_sequence(double time_limit, uint8_t* rec_base) {
    double* tarr = reinterpret_cast<double*>(rec_base + kResetHeadBytes);
    int32_t* tpl = reinterpret_cast<int32_t*>(rec_base + kResetHeadBytes + 8 * (int64_t)JC);
    const int cap = HP(job_arrival_cap);
    double t = 0.0;
    int k = 0;
    while (t < time_limit && (cap == 0 || k < cap)) {
      if (k >= JC) return -1;
      const int q = 1 + (int)rng.bounded(22);
      const int sz = (int)rng.bounded(7);
      if (W::lane() == 0) {
        tpl[k] = (q - 1) * 7 + sz;
        tarr[k] = t;
      }
      t += HP(job_arrival_gap) * rng.std_exponential();
      k++;
    }
    return k;
  }

  // reset(seed=None | seed) with the job sequence sampled on the device; then reset() from the record.
  // `mode`: SSIM_RESET_CONTINUE continues the env's current stream (header loaded), SSIM_RESET_SEED
  // reseeds it as Generator(PCG64(SeedSequence(seed))).
  __device__ __forceinline__ void reset_sampled(int mode, uint64_t seed, double time_limit, uint8_t* rec_base) {
    if (mode == SSIM_RESET_SEED) {
      rng = Pcg64::from_seed(seed);
    } else if (h.num_jobs == 0 && h.episode == 0) {  // no stream to continue: never reset before
      fail(SSIM_ERR_RESET);
      store_header();
      return;
    }
    int n = 0;
    if (!(time_limit == __builtin_inf() && HP(job_arrival_cap) == 0) && HP(job_arrival_gap) > 0.0)
      n = sample_job_sequence(time_limit, rec_base);
    ssim_reset_record* rec = reinterpret_cast<ssim_reset_record*>(rec_base);
    if (W::lane() == 0) {
      rec->rng_state_hi = rng.s_hi;
      rec->rng_state_lo = rng.s_lo;
      rec->rng_inc_hi = rng.i_hi;
      rec->rng_inc_lo = rng.i_lo;
      rec->rng_has_uint32 = rng.has32;
      rec->rng_uinteger = rng.u32;
      rec->num_jobs = n > 0 ? n : JC + 1;  // over-capacity / empty sequences make reset() fail the env
      rec->time_limit = time_limit;
    }
    W::gsync();  // lane 0's global stores before every lane reads the record back
    reset(rec_base);
  }

  // ---------------------------------------------------------------- reset (:127-186, :260-273)
  // Runs with the hot block in HBM (hot == ghot).
  __device__ __forceinline__ void reset(const uint8_t* rec_base) {
    const ssim_reset_record* rec = reinterpret_cast<const ssim_reset_record*>(rec_base);
    const double* tarr = reinterpret_cast<const double*>(rec_base + kResetHeadBytes);
    const int32_t* tpl = reinterpret_cast<const int32_t*>(rec_base + kResetHeadBytes + 8 * (int64_t)JC);
    const int nj = rec->num_jobs;
    if (nj <= 0) return;
    const EnvHeader* prev = H<EnvHeader>(O.hdr);
    const int prev_episode = W::uni(prev->episode);
    if (W::uni(prev->num_jobs) > 0) {  // the previous episode ends here (accumulators persist, EnvAcc)
      UF<int64_t> eps{&H<EnvAcc>(O.acc)->episodes};
      eps = (int64_t)eps + 1;
    }
    {  // a step preempted in the previous episode is abandoned with it
      UF<int64_t> pend{&H<EnvAcc>(O.acc)->pending};
      pend = (int64_t)0;
    }
    h = EnvHeader();
    h.episode = prev_episode + 1;
    h.time_limit = rec->time_limit;
    rng.s_hi = rec->rng_state_hi;
    rng.s_lo = rec->rng_state_lo;
    rng.i_hi = rec->rng_inc_hi;
    rng.i_lo = rec->rng_inc_lo;
    rng.has32 = rec->rng_has_uint32;
    rng.u32 = rec->rng_uinteger;
    h.num_jobs = nj;
    h.seq = nj;
    h.source = kPoolCommon;
    h.commit_seq = 0;
    if (nj > JC) {
      fail(SSIM_ERR_RESET);
      h.num_jobs = 0;
      observe(0.0);
      store_header();
      return;
    }
    // jobs: template, stage base (exclusive scan of stage counts)
    int run = 0;
    bool bad = false;
    const int ntpl = HP(num_templates);
    const int32_t* const tsb = HP(tpl_stage_base);
    for (int j0 = 0; j0 < nj; j0 += W::kWidth) {
      const int j = j0 + W::lane();
      const bool ok = j < nj;
      const int t = ok ? tpl[j] : 0;
      const bool tb = ok && (t < 0 || t >= ntpl);
      const int ns = (ok && !tb) ? ldg(tsb, t + 1) - ldg(tsb, t) : 0;
      int total = 0;
      const int ex = W::excl_scan(ns, &total);
      if (ok) {
        job_tpl(j) = (int16_t)t;
        job_base(j) = (int16_t)(run + ex);
        job_nst(j) = (int16_t)ns;
        job_nact(j) = (int16_t)ns;
        job_sat(j) = 0;
        job_local(j) = 0;
        job_supply(j) = 0;
        job_state(j) = kJobPending;
        job_arr_dec(j) = -1;
        job_done_dec(j) = -1;
        job_tarr(j) = tarr[j];
        job_tdone(j) = __builtin_inf();
      }
      if (W::ballot(tb)) bad = true;
      run += total;
    }
    if (bad || run > SC) {
      fail(SSIM_ERR_RESET);
      h.num_jobs = 0;
      observe(0.0);
      store_header();
      return;
    }
    W::sync();
    // stage records are initialised at arrival (on_job_arrival)
    live_lo = 0;
    // executors, commitments, COMMON pool = set(range(N))
    for (int k0 = 0; k0 < NE; k0 += W::kWidth) {
      const int e = k0 + W::lane();
      if (e < NE) {
        ex_loc(e) = kPoolCommon;
        ex_job(e) = -1;
        ex_task(e) = -1;
        ex_busy(e) = 0;
        ev_seq(e) = -1;
        ev_t(e) = 0.0;
        ev_type(e) = 0;
        ev_stage(e) = -1;
      }
    }
    for (int k0 = 0; k0 < commit_cap_for(NE); k0 += W::kWidth) {
      const int k = k0 + W::lane();
      if (k < commit_cap_for(NE)) cm(k) = CommitRec{};
    }
    W::sync();
    ev_regs_load();
    if (paged_sets()) {
      paged_init_range(kPoolCommon, NE);
    } else {
      uint8_t* t = S<uint8_t>(O.sc_tab_p);
      ps_init(pmeta(kPoolCommon), t);
      for (int e = 0; e < NE; ++e) ps_add<W>(pmeta(kPoolCommon), t, (uint32_t)e, S<int32_t>(O.sc_keys_b));
      unstage_table(kPoolCommon, t);
    }
    cfrom(kPoolCommon) = 0;
    W::sync();
    // _load_initial_jobs: arrivals with t <= 0 (wall_time stays 0)
    while (h.arrivals < h.num_jobs && job_tarr(h.arrivals) <= 0.0) {
      const int j = h.arrivals++;
      h.events++;
      trace(0.0, kEvArrival, -1, j, -1, j);
      on_job_arrival(j);
    }
    if (h.num_jobs > 0) check(job_tarr(0) == 0.0);  // "first job must arrive at t=0"
    observe(0.0);
    store_header();
  }
};

}  // namespace ssim
