// kernels.h — the Sim-based step / rollout kernels (templates) shared by the kernel translation units.
//
// Each instantiation of the engine is a large kernel, so they are compiled in separate translation units
// (k_*.hip, built in parallel) that each return the kernel pointers of one layout specialisation
// (KernelSet); sparksched.hip picks one per launch from the layout.
#pragma once
#include <hip/hip_runtime.h>

#include "sparksched.h"
#include "engine.h"
#include "policy.h"
#include "rollout.h"
#include "wave_hip.h"

using namespace ssim;

extern __shared__ __attribute__((aligned(16))) uint8_t g_smem[];

// An env whose header says terminated / frozen / never reset is skipped without touching LDS.
__device__ __forceinline__ bool env_idle(const Params* __restrict__ P, const uint8_t* state, int eid) {
  const EnvHeader* gh =
      reinterpret_cast<const EnvHeader*>(state + kParamsReserve + (int64_t)eid * P->L.env_bytes + P->O.hdr);
  return gh->terminated || (gh->err & SSIM_ERR_STICKY) || gh->num_jobs == 0;
}

// kRes: hot block LDS-resident. A compile-time flag (not a runtime select between an LDS and an HBM pointer)
// so every hot-block access compiles to ds_read/ds_write rather than FLAT instructions.
// Waves per SIMD the HBM-resident (kRes = false) kernels are compiled for. Their state lives in HBM, so the
// event loop is bound by memory latency and occupancy hides it; the LDS-resident ones run one wave per SIMD
// by LDS budget anyway. Register caps: 2 waves -> 256 VGPRs, 4 -> 128. Measured on the configs[3] shard (4096
// envs, J=200, N=100): 8.9M decisions/s at 1 wave (266 VGPRs), 15.2M at 2, 17.3M at 4 (despite scratch spills).
#ifndef SSIM_HBM_ROLLOUT_WAVES
#define SSIM_HBM_ROLLOUT_WAVES 4
#endif
#ifndef SSIM_HBM_STEP_WAVES
#define SSIM_HBM_STEP_WAVES 4
#endif
constexpr int32_t kFlagTicketSlot = 0x100;  // internal k_rollout flag: use the second budget counter

// The budget rollout's decision counter and "budget spent" flag. Claims take chunks of decisions from one atomic
// counter (tens of claims per microsecond over the whole chip); the wave whose claim finds the budget spent raises
// the flag on kStopLines lines, and with SSIM_ROLLOUT_PREEMPT every running step polls its own line
// (env % kStopLines) every few events, so the polls spread over eight lines instead of queueing on the counter.
// `issue` starts a poll one event before `hit` tests it (Sim::simulate), hiding its latency.
struct TicketStop {
  static constexpr bool kCan = true;
  uint8_t* base;   // this launch's slot (null: no budget)
  int64_t total;   // the launch's budget
  int line;        // this wave's flag line
  bool on;         // preemption enabled
  __device__ __forceinline__ unsigned long long* word(int l) const {
    return reinterpret_cast<unsigned long long*>(base + kTicketStride * l);
  }
  // Decisions granted to this wave (0: the budget is spent). The chunk follows what is left per env: 8 early,
  // 1 at the end (guided self-scheduling). `last` = the counter at this wave's previous claim.
  __device__ __forceinline__ int64_t claim(int64_t num_envs, int64_t& last) const {
    int64_t c = (total - last) / (4 * num_envs);
    c = c < 1 ? 1 : c > 8 ? 8 : c;
    unsigned long long t = 0;
    if (WaveHip::lane() == 0) t = atomicAdd(word(0), (unsigned long long)c);
    last = (int64_t)WaveHip::uni((uint64_t)t);
    if (last < total) return total - last < c ? total - last : c;
    if (WaveHip::lane() < kStopLines)  // the budget is spent: stop the steps still simulating
      __hip_atomic_store(word(1 + WaveHip::lane()), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  // Returns `n` decisions granted to this wave but not taken, so other waves of the launch can still claim them.
  __device__ __forceinline__ void give_back(int64_t n) const {
    if (WaveHip::lane() == 0) atomicAdd(word(0), (unsigned long long)(-n));
  }
  __device__ __forceinline__ uint64_t issue() const {
    return on ? __hip_atomic_load(word(1 + line), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
  }
  __device__ __forceinline__ bool hit(uint64_t v) const { return on && WaveHip::uni(v) != 0; }
};

template <bool kRes, int kN, int kJ, int kS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(kRes ? 1 : SSIM_HBM_STEP_WAVES))) void k_step(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                             const int32_t* __restrict__ stage_idx,
                                             const int32_t* __restrict__ num_exec) {
  const int eid = blockIdx.x;
  if (env_idle(P, state, eid)) return;
  Sim<WaveHip, kN, kJ, kS> s(P, state, g_smem, obs, eid, kRes, false, /*ex_lds=*/!kRes);
  StepIn a;
  a.stage_idx = stage_idx[eid];
  a.num_exec = num_exec[eid];
  s.load_hot();
  s.load_header();
  if (s.pending()) {  // a preempted step completes first; this call's action (chosen on a stale obs) is dropped
    s.resume(NoStop());
    s.write_err_only(SSIM_ERR_PENDING);
  } else {
    s.step_loaded(a);
  }
  s.save_hot();
}

// row_cold: the engine keeps observe()'s row map in the cold block (Sim), leaving the layout's LDS for the row map to
// the action driver (the Decima rollout's policy plan).
template <bool kRes, int kN, int kJ, int kS, class Pol>
__device__ __forceinline__ void rollout_body(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                                const Pol& pol, int num_steps, int flags,
                                                const double* __restrict__ limits, uint8_t* reset,
                                                int32_t* action_log, uint64_t* prof_out, int64_t budget,
                                                const int32_t* __restrict__ env_steps, bool row_cold = false,
                                                bool ex_lds = true) {
  const int eid = blockIdx.x;
  const int B = P->L.num_envs;
  if (budget > 0 && eid == 0 && WaveHip::lane() <= kStopLines)  // the next budget launch's slot (TicketStop)
    *reinterpret_cast<unsigned long long*>(state + kTicketOffset + ((flags & kFlagTicketSlot) ? 0 : kTicketSlotBytes) +
                                           kTicketStride * WaveHip::lane()) = 0ull;
  if (env_steps != nullptr) {  // per-env decision counts (ssim_rollout_steps), capped by num_steps
    const int n = env_steps[eid];
    num_steps = n < num_steps ? n : num_steps;
    if (num_steps <= 0) return;
  }
  const bool autoreset = (flags & SSIM_ROLLOUT_AUTORESET) != 0;
  if (!autoreset && action_log == nullptr && env_idle(P, state, eid)) return;
  // Shared budget (budget > 0): decisions are claimed from one device counter in chunks sized to what is
  // left (guided self-scheduling: 8 early, 1 at the end), so the launch ends within ~one decision of the
  // budget running out instead of waiting for the env with the most expensive K decisions. With
  // SSIM_ROLLOUT_PREEMPT it ends within ~one EVENT: a step still simulating when the budget runs out stops at
  // its next event boundary and stays pending for the next launch.
  // Two slots used alternately (kFlagTicketSlot): this launch's starts zeroed because the previous budget launch
  // zeroed it, and this launch zeroes the other for the next (launches on a stream are ordered), so no memset
  // launch precedes a budget launch.
  const int slot = (flags & kFlagTicketSlot) ? 1 : 0;
  const TicketStop stop{budget > 0 ? state + kTicketOffset + kTicketSlotBytes * slot : nullptr, budget,
                        eid % kStopLines, budget > 0 && (flags & SSIM_ROLLOUT_PREEMPT) != 0};
  RolloutCursor c{0, 0, 0};
  const double limit = limits != nullptr ? limits[eid] : __builtin_inf();
  uint8_t* rec = reset + (int64_t)eid * P->L.reset_stride;
#ifdef SSIM_PROFILE
  const uint64_t rt_entry = WaveHip::realtime();
#endif
  Sim<WaveHip, kN, kJ, kS> s(P, state, g_smem, obs, eid, kRes, row_cold, ex_lds && !kRes);
#ifdef SSIM_PROFILE
  s.prof_set(kTCtor, WaveHip::realtime());
#endif
  s.load_hot();
#ifdef SSIM_PROFILE
  s.prof_set(kTEntry, rt_entry);
  s.prof_set(kTLoaded, WaveHip::realtime());
#endif
  const auto reset_in_place = [&](Sim<WaveHip, kN, kJ, kS>& x) {
    x.reset_sampled(SSIM_RESET_CONTINUE, 0ull, limit, rec);
  };
  rollout_loop(s, pol, stop, c, B, eid, num_steps, autoreset, action_log, reset_in_place);
  if (c.granted > 0) stop.give_back(c.granted);  // a chunk the wave could not use (its step cap or episode end)
#ifdef SSIM_PROFILE
  s.prof_set(kTLoopEnd, WaveHip::realtime());
#endif
  s.save_hot();
#ifdef SSIM_PROFILE
  s.prof_set(kTSaved, WaveHip::realtime());
  WaveHip::sync();
  if (prof_out != nullptr)
    for (int p = WaveHip::lane(); p < kNumPhases; p += 64) prof_out[(int64_t)eid * kNumPhases + p] = s.prof[p];
#else
  (void)prof_out;
#endif
}

#define SSIM_ROLLOUT_ARGS                                                                                       \
  const Params *__restrict__ P, uint8_t *state, uint8_t *obs, int kind, uint64_t seed, int num_steps, int flags, \
      const double *__restrict__ limits, uint8_t *reset, int32_t *action_log, uint64_t *prof_out, int64_t budget, \
      const int32_t *__restrict__ env_steps
#define SSIM_ROLLOUT_WAVES(kRes) ((kRes) ? 1 : SSIM_HBM_ROLLOUT_WAVES)
template <bool kRes, int kN, int kJ, int kS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(SSIM_ROLLOUT_WAVES(kRes)))) void k_rollout(SSIM_ROLLOUT_ARGS) {
  rollout_body<kRes, kN, kJ, kS, HeuristicPolicy>(P, state, obs, HeuristicPolicy{kind, seed}, num_steps, flags, limits,
                                                  reset, action_log, prof_out, budget, env_steps);
}
// The same rollout under its own symbol for launches that are not measured (SSIM_ROLLOUT_WARMUP: a benchmark's
// pre-roll and warm-up), so a profiler's per-kernel statistics of k_rollout cover the timed launches only.
template <bool kRes, int kN, int kJ, int kS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(SSIM_ROLLOUT_WAVES(kRes)))) void k_rollout_warmup(SSIM_ROLLOUT_ARGS) {
  rollout_body<kRes, kN, kJ, kS, HeuristicPolicy>(P, state, obs, HeuristicPolicy{kind, seed}, num_steps, flags, limits,
                                                  reset, action_log, prof_out, budget, env_steps);
}

// Test hook (ssim_debug_set_trace_ex, tests/test_gpu_sets.py): a trace of CPython-set operations on one pool (job 0's)
// of env 0 through the set code of the engine instantiation `Sim<WV, kN, kJ, kS>` with residency kRes — the template
// instantiation a translation unit's shipped kernels inline, compiled in that unit with its flags (kTag keeps one
// copy per unit; the linker would otherwise fold identical instantiations of different units into one). The set path
// is the one the layout selects (one-page lane sets for <= 15 executors, paged tables for 16..127). ops: int32
// [n_ops][6] = (code, key, busy bitmap words 0..3); code 0 add(key), 1 remove(key), 2 idle order:
// list(set(e for e in s.copy() if not busy[e])) with the executors' busy flags from the bitmap. orders [n_ops][width]:
// the set's iteration order after an add / remove, the idle order for code 2; -1 padded. Clobbers env 0.
// Compiled under the rollout kernels' occupancy attribute (the same register budget), but as its own kernel: it pins
// the set code's logic per unit and its codegen at that budget, not the inlined codegen inside k_rollout /
// k_decima_rollout (those are pinned end to end by the replay tests).
template <class WV, bool kRes, int kN, int kJ, int kS, int kTag>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(SSIM_ROLLOUT_WAVES(kRes)))) void k_set_trace(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                                  const int32_t* __restrict__ ops, int n_ops, int width,
                                                  int32_t* orders) {
  Sim<WV, kN, kJ, kS> s(P, state, g_smem, obs, 0, kRes);
  if constexpr (kRes) s.load_hot();
  const int p = s.job_pool(0);
  ps_init(s.pmeta(p), s.pool(p).tab);
  int32_t* out = s.template S<int32_t>(s.O.sc_keys_a);
  for (int k = 0; k < n_ops; ++k) {
    const int code = WV::uni(ops[6 * k]), key = WV::uni(ops[6 * k + 1]);
    int n = 0;
    if (code == 2) {
      for (int e = WV::lane(); e < s.NE; e += 64)
        s.exr(e).busy = (int16_t)((ops[6 * k + 2 + (e >> 5)] >> (e & 31)) & 1);
      WV::sync();
      n = s.idle_order(p, out);
    } else {
      if (code == 0)
        s.pool_add(p, key);
      else
        s.pool_remove(p, key);
      n = s.table_keys(p, out);
    }
    WV::sync();
    for (int i = WV::lane(); i < width; i += 64) orders[(int64_t)k * width + i] = i < n ? out[i] : -1;
    WV::sync();
  }
}
// The known-bad wave type of the KAT (engine.h KatBadPage): test-only, never used by a shipped kernel.
struct WaveHipKatBadPage : WaveHip {
  static constexpr bool kKatBadPage = true;
};

using StepFn = void (*)(const Params*, uint8_t*, uint8_t*, const int32_t*, const int32_t*);
using RolloutFn = void (*)(const Params*, uint8_t*, uint8_t*, int, uint64_t, int, int, const double*, uint8_t*,
                          int32_t*, uint64_t*, int64_t, const int32_t*);
using SetTraceFn = void (*)(const Params*, uint8_t*, uint8_t*, const int32_t*, int, int, int32_t*);
struct KernelSet {
  StepFn step;
  RolloutFn rollout, rollout_warmup;
  SetTraceFn set_trace;  // the set KAT through this unit's engine instantiation (k_set_trace)
  const char* name;      // the translation unit (ssim_debug_kernel_name)
};
template <bool kRes, int kN, int kJ, int kS, int kTag>
inline KernelSet kernel_set(const char* name) {
  return {k_step<kRes, kN, kJ, kS>, k_rollout<kRes, kN, kJ, kS>, k_rollout_warmup<kRes, kN, kJ, kS>,
          k_set_trace<WaveHip, kRes, kN, kJ, kS, kTag>, name};
}
// Translation-unit tags of k_set_trace (one per k_*.hip)
enum : int { kTagBench900 = 1, kTagBench, kTagLds, kTagHbm, kTagHbmN100, kTagHbmN10, kTagHbmN50, kTagDrHbm, kTagDrHbm50,
             kTagDrLds, kTagKatBad, kTagDrLds50 };
SetTraceFn set_trace_kat_bad();  // k_hbm_n100.hip: the N = 100 / J = 200 instantiation on WaveHipKatBadPage
// one per translation unit
KernelSet kernels_bench900();  // k_bench900.hip: LDS-resident, 10 executors / 50 jobs / stage cap 900
KernelSet kernels_bench();     // k_bench.hip: LDS-resident, 10 executors / 50 jobs, stage cap at run time
KernelSet kernels_lds();       // k_lds.hip: LDS-resident, any shape
KernelSet kernels_hbm();       // k_hbm.hip: hot block in HBM, any shape
KernelSet kernels_hbm_n100();  // k_hbm_n100.hip: hot block in HBM, 100 executors / 200 jobs (configs[3] shard)
KernelSet kernels_hbm_n10();   // k_hbm_n10.hip: hot block in HBM, 10 executors / 50 jobs (configs[1] env, large batches)
KernelSet kernels_hbm_n50();   // k_hbm_n50.hip: hot block in HBM, 50 executors / 200 jobs (decima_tpch.yaml env)
