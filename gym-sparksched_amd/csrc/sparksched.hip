// sparksched.hip — gfx950 kernels and the C ABI (include/sparksched.h).
//
// One 64-lane wavefront per env (one workgroup = one wave; no workgroup barriers needed). Per-env state
// lives in the caller's state arena in HBM (env-major SoA, layout.h); per-launch scratch (node row map,
// temporary CPython-set tables, commitment plan) lives in LDS. Kernels:
//   k_reset   : env init from a host-sampled job sequence + _load_initial_jobs + first observation
//   k_step    : one env.step per env from device action arrays (obs written to the obs arena)
//   k_policy  : device action driver (fair / FIFO / random) reading the obs arena
//   k_rollout : `num_steps` x (policy -> step) fused into one launch (no host round trips)
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdlib.h>

#include <mutex>
#include <stdio.h>
#include <string.h>

#include "kernels.h"
#include "decima.h"
#include "decima_policy.h"
#include "decima_rollout.h"

// ------------------------------------------------------------------------------------------ kernels

__global__ __launch_bounds__(64) void k_reset(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                              const uint8_t* __restrict__ reset) {
  const int eid = blockIdx.x;
  Sim<WaveHip> s(P, state, g_smem, obs, eid, false);
  s.reset(reset + (int64_t)eid * P->L.reset_stride);
}

// Device-sampled reset of the envs with mode != SSIM_RESET_SKIP (hot block in HBM, like k_reset).
__global__ __launch_bounds__(64) void k_reset_sampled(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                                      uint8_t* reset, const uint8_t* __restrict__ mode,
                                                      const uint64_t* __restrict__ seeds,
                                                      const double* __restrict__ limits) {
  const int eid = blockIdx.x;
  const int m = mode[eid];
  if (m == SSIM_RESET_SKIP) return;
  Sim<WaveHip> s(P, state, g_smem, obs, eid, false);
  s.load_header();
  s.reset_sampled(m, seeds != nullptr ? seeds[eid] : 0ull, limits != nullptr ? limits[eid] : __builtin_inf(),
                  reset + (int64_t)eid * P->L.reset_stride);
}

__global__ __launch_bounds__(64) void k_policy(const Params* __restrict__ P, const uint8_t* obs, int kind,
                                               uint64_t seed, uint64_t counter, int32_t* stage_idx,
                                               int32_t* num_exec) {
  const int eid = blockIdx.x;
  PolicyView<WaveHip> v{P->L, obs, eid};
  const StepIn a = v.act(kind, seed, counter);
  if (WaveHip::lane() == 0) {
    stage_idx[eid] = a.stage_idx;
    num_exec[eid] = a.num_exec;
  }
}

__global__ __launch_bounds__(64) void k_decima(const Params* __restrict__ P, const uint8_t* obs, float nts,
                                               float ws, float* feats, int32_t* ccap, uint32_t* emask,
                                               int32_t* depth) {
  DecimaView<WaveHip> v{P->L, obs, (int)blockIdx.x};
  v.run(nts, ws, g_smem, feats, ccap, emask, depth);
}

// The policy parameters (DecimaScheduler.parameters() order, nn.Linear layout) into the matrix cores' packed layout
// (decima_policy.h Mlp3P); one thread per packed float.
__global__ __launch_bounds__(256) void k_decima_pack(const float* __restrict__ params, float* __restrict__ packed) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= 4 * kDpPacked) return;
  const int src = dp_pack_src(f);
  packed[f] = src >= 0 ? params[src] : 0.0f;
}

// `plan` null: the plan in LDS (dynamic shared memory); else a per-env region of global memory (stride plan_stride),
// for node caps whose plan exceeds the LDS of a workgroup.
template <bool kGlobal>
__global__ __launch_bounds__(64) void k_decima_policy(const Params* __restrict__ P, const uint8_t* __restrict__ obs,
                                                      const float* __restrict__ feats, const int32_t* __restrict__ ccap,
                                                      const uint32_t* __restrict__ emask,
                                                      const int32_t* __restrict__ depth, const dp_f32x4* __restrict__ Wt,
                                                      int node_cap, uint64_t seed, uint64_t counter,
                                                      const uint8_t* __restrict__ env_mask, DecimaPolicyOut o,
                                                      int32_t* overflow, uint8_t* plan, int64_t plan_stride) {
  const int eid = blockIdx.x;
  if (env_mask != nullptr && env_mask[eid] == 0) {
    if (WaveHip::lane() == 0) {
      o.stage_idx[eid] = -1;
      o.num_exec[eid] = 1;
      o.job_idx[eid] = -1;
      o.exec_idx[eid] = 0;
      o.lgprob[eid] = 0.0f;
    }
    return;
  }
  uint8_t* lds = kGlobal ? plan + (int64_t)eid * plan_stride : g_smem;
  if (!decima_policy_env<kGlobal>(P, obs, feats, ccap, emask, depth, DpWGlobal{Wt}, node_cap, seed, counter, eid, lds,
                                  o) &&
      WaveHip::lane() == 0 && overflow != nullptr)
    atomicAdd(overflow, 1);
}

// per-job arrival/completion times and state (JobRec/JobTimes in the hot block) -> [num_envs][job_cap]
__global__ __launch_bounds__(64) void k_job_times(const Params* __restrict__ P, const uint8_t* state,
                                                  double* ta, double* tc, int32_t* st) {
  const int eid = blockIdx.x, J = P->L.job_cap;
  const uint8_t* hot = state + kParamsReserve + (int64_t)eid * P->L.env_bytes;
  const JobRec* jr = reinterpret_cast<const JobRec*>(hot + P->O.jobs);
  const JobTimes* jt = reinterpret_cast<const JobTimes*>(hot + P->O.jtimes);
  for (int j = threadIdx.x; j < J; j += 64) {
    const int64_t o = (int64_t)eid * J + j;
    if (ta) ta[o] = jt[j].tarr;
    if (tc) tc[o] = jt[j].tdone;
    if (st) st[o] = jr[j].state;
  }
}

// Kernel variant for a layout: LDS-resident instantiations specialised on the benchmark shape (BASELINE configs[1]:
// 10 executors, 50 jobs): fully (stage cap too) when the packed dataset's cap is the synthetic set's 50 x 18, else
// on (executors, jobs) with the stage cap read at run time (any other TPC-H-format dataset, e.g. the real traces
// loaded from data/tpch); other shapes use the generic instantiations.
static bool bench_shape(const Params& p) { return p.L.num_executors == 10 && p.L.job_cap == 50; }
static bool decima_shape(const Params& p) { return p.L.num_executors == 50 && p.L.job_cap == 200; }
static bool large_shape(const Params& p) { return p.L.num_executors == 100 && p.L.job_cap == 200; }
// Diagnostic switch: SSIM_GENERIC=1 runs every HBM-resident layout on the generic (run-time shape) kernels.
static bool generic_forced() {
  static const int on = [] {
    const char* v = getenv("SSIM_GENERIC");
    return (v != nullptr && v[0] == '1') ? 1 : 0;
  }();
  return on != 0;
}
static KernelSet pick_kernels(const Params& p) {
  if (!p.O.lds_resident) {  // HBM-resident: the configs[2] / [3] shapes have (executors, jobs)-specialised kernels
    if (generic_forced()) return kernels_hbm();
    if (large_shape(p)) return kernels_hbm_n100();
    if (decima_shape(p)) return kernels_hbm_n50();
    if (bench_shape(p)) return kernels_hbm_n10();
    return kernels_hbm();
  }
  if (bench_shape(p)) return p.L.stage_cap == 900 ? kernels_bench900() : kernels_bench();
  return kernels_lds();
}
static DecimaRolloutSet pick_decima(const Params& p) {
  return p.O.lds_resident                          ? (decima_shape(p) && !generic_forced() ? decima_rollout_lds50()
                                                                                          : decima_rollout_lds())
         : !decima_shape(p) || generic_forced()   ? decima_rollout_hbm()
                                                  : decima_rollout_hbm50();
}
static StepFn pick_step(const Params& p) { return pick_kernels(p).step; }
static RolloutFn pick_rollout(const Params& p, bool warmup = false) {
  const KernelSet k = pick_kernels(p);
  return warmup ? k.rollout_warmup : k.rollout;
}

// ------------------------------------------------------------------------------------------ C ABI
struct ssim_handle {
  Params params;  // host copy (device copy at the start of the state arena)
  uint8_t* state;
  uint8_t* obs;
  uint8_t* reset;
  int ticket_slot;  // budget-launch decision counter in use next (k_rollout kFlagTicketSlot)
  uint64_t* prof_next = nullptr;  // -DSSIM_PROFILE builds: per-wave phase sums of the next Decima rollout launch
  uint8_t* policy_plan = nullptr;  // ssim_decima_policy's global plan when a node cap's plan exceeds the LDS
  int64_t policy_plan_bytes = 0;
  void* policy_packed = nullptr;   // ssim_decima_policy's packed weights (kDpPackedBytes)
};

static thread_local char g_err[512] = "";

static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return set_err(SSIM_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return SSIM_OK;
}

static int decima_pack(const float* params, void* packed, void* stream) {
  hipLaunchKernelGGL(k_decima_pack, dim3((4 * kDpPacked + 255) / 256), dim3(256), 0, (hipStream_t)stream, params,
                     static_cast<float*>(packed));
  return hip_check(hipGetLastError(), "k_decima_pack launch");
}

// A launch with more than 64 KB of dynamic LDS (layout.h kLdsBudgetBig) needs the kernel's opt-in attribute. It is
// per-device, per-function state: the raised limit is remembered per (device, kernel) so the attribute call is made
// once, not before every step launch. The cache is shared by every host thread that launches, so it is guarded by a
// mutex (an unguarded entry could pair one kernel with another thread's larger limit and skip a needed call).
static std::mutex g_lds_mu;
static int lds_opt_in(const void* fn, int64_t lds) {
  if (lds <= kLdsBudget) return SSIM_OK;
  struct Entry {
    int dev;
    const void* fn;
    int64_t lds;
  };
  static Entry cache[64];
  static int n_cache = 0;
  int dev = 0;
  int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
  if (rc != SSIM_OK) return rc;
  std::lock_guard<std::mutex> lk(g_lds_mu);
  for (int i = 0; i < n_cache; ++i)
    if (cache[i].dev == dev && cache[i].fn == fn && cache[i].lds >= lds) return SSIM_OK;
  rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                 "engine kernel LDS attribute");
  if (rc == SSIM_OK && n_cache < 64) cache[n_cache++] = Entry{dev, fn, lds};
  return rc;
}

// Compute units of the current device (the layout's LDS-residency threshold, layout.h compute_layout); a whole MI355X
// when there is no device (host-only use of ssim_layout_for).
static int64_t device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      n <= 0) {
    (void)hipGetLastError();  // (clear the sticky error of a host without a device)
    return kChipCus;
  }
  return n;
}

extern "C" int ssim_layout_for(const ssim_config* cfg, ssim_layout* out) {
  StateOffsets O;
  if (cfg == nullptr || out == nullptr || !compute_layout(*cfg, out, &O, device_cus()))
    return set_err(SSIM_E_ARG, "ssim_layout_for: invalid config");
  return SSIM_OK;
}

extern "C" int ssim_create(const ssim_config* cfg, const ssim_dataset* dataset, void* state_arena,
                           void* obs_arena, void* reset_arena, ssim_handle** out) {
  if (cfg == nullptr || dataset == nullptr || state_arena == nullptr || obs_arena == nullptr ||
      reset_arena == nullptr || out == nullptr)
    return set_err(SSIM_E_ARG, "ssim_create: null argument");
  ssim_handle* h = new ssim_handle();
  if (!compute_layout(*cfg, &h->params.L, &h->params.O, device_cus())) {
    delete h;
    return set_err(SSIM_E_ARG, "ssim_create: invalid config");
  }
  if (h->params.O.lds_bytes > (h->params.O.lds_resident ? kLdsBudgetBig : kLdsBudget)) {
    delete h;
    return set_err(SSIM_E_ARG, "ssim_create: per-env scratch %lld B exceeds the LDS budget",
                   (long long)h->params.O.lds_bytes);
  }
  if (dataset->num_template_stages >= 32768 || dataset->num_templates >= 32768) {
    delete h;
    return set_err(SSIM_E_ARG, "ssim_create: dataset too large for int16 stage/template ids");
  }
  h->params.D = *dataset;
  h->params.C = *cfg;
  fill_hot_params(&h->params);
  h->state = static_cast<uint8_t*>(state_arena);
  h->obs = static_cast<uint8_t*>(obs_arena);
  h->reset = static_cast<uint8_t*>(reset_arena);
  {  // executor-key table for the sampler, from the dataset's executor_intervals
    const int N = cfg->num_executors;
    double* iv = new double[2 * (N + 1)];
    int rc0 = hip_check(hipMemcpy(iv, dataset->intervals, sizeof(double) * 2 * (N + 1), hipMemcpyDeviceToHost),
                        "intervals download");
    if (rc0 == SSIM_OK && !fill_interval_table(&h->params, iv, N))
      rc0 = set_err(SSIM_E_ARG, "ssim_create: executor_intervals values are not EXEC_LEVELS integers");
    delete[] iv;
    if (rc0 != SSIM_OK) {
      delete h;
      return rc0;
    }
  }
  {  // the duration-descriptor cache (engine.h) packs offset << 8 | length: usable when every list fits
    const int64_t nd = (int64_t)dataset->num_template_stages * 3 * kNumLevels;
    int32_t* dl = new int32_t[nd > 0 ? nd : 1];
    int32_t* dof = new int32_t[nd > 0 ? nd : 1];
    int rc0 = nd <= 0 ? SSIM_OK : hip_check(hipMemcpy(dl, dataset->dur_len, sizeof(int32_t) * nd, hipMemcpyDeviceToHost),
                                            "dur_len download");
    if (rc0 == SSIM_OK && nd > 0)
      rc0 = hip_check(hipMemcpy(dof, dataset->dur_off, sizeof(int32_t) * nd, hipMemcpyDeviceToHost), "dur_off download");
    bool fits = rc0 == SSIM_OK;
    for (int64_t i = 0; fits && i < nd; ++i)
      if (dl[i] > 255 || (dl[i] > 0 && (dof[i] < 0 || dof[i] >= (1 << 24)))) fits = false;
    h->params.hp.dcache = fits ? 1 : 0;
    delete[] dl;
    delete[] dof;
    if (rc0 != SSIM_OK) {
      delete h;
      return rc0;
    }
  }
  int rc = hip_check(hipMemcpy(h->state, &h->params, sizeof(Params), hipMemcpyHostToDevice), "params upload");
  if (rc == SSIM_OK)  // both budget slots start zeroed (each budget launch then zeroes the other, TicketStop)
    rc = hip_check(hipMemset(h->state + kTicketOffset, 0, (size_t)(2 * kTicketSlotBytes)), "budget slots clear");
  if (rc == SSIM_OK) rc = hip_check(hipMemset(h->obs, 0, (size_t)h->params.L.obs_bytes), "obs clear");
  if (rc == SSIM_OK)
    rc = hip_check(hipMemset(h->state + kParamsReserve, 0, (size_t)(h->params.L.state_bytes - kParamsReserve)),
                   "state clear");
  if (rc != SSIM_OK) {
    delete h;
    return rc;
  }
  *out = h;
  return SSIM_OK;
}

extern "C" int ssim_destroy(ssim_handle* h) {
  if (h != nullptr && h->policy_plan != nullptr) (void)hipFree(h->policy_plan);
  if (h != nullptr && h->policy_packed != nullptr) (void)hipFree(h->policy_packed);
  delete h;
  return SSIM_OK;
}

static const Params* dparams(const ssim_handle* h) { return reinterpret_cast<const Params*>(h->state); }

extern "C" int ssim_reset(ssim_handle* h, void* stream) {
  if (h == nullptr) return set_err(SSIM_E_ARG, "ssim_reset: null handle");
  const ssim_layout& L = h->params.L;
  hipLaunchKernelGGL(k_reset, dim3(L.num_envs), dim3(64), (size_t)L.scratch_bytes, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, h->reset);
  return hip_check(hipGetLastError(), "k_reset launch");
}

extern "C" int ssim_step(ssim_handle* h, const int32_t* stage_idx, const int32_t* num_exec, void* stream) {
  if (h == nullptr || stage_idx == nullptr || num_exec == nullptr) return set_err(SSIM_E_ARG, "ssim_step: null");
  const ssim_layout& L = h->params.L;
  const StepFn fn = pick_step(h->params);
  const int rc = lds_opt_in((const void*)fn, h->params.O.lds_bytes);
  if (rc != SSIM_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(L.num_envs), dim3(64), (size_t)h->params.O.lds_bytes, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, stage_idx, num_exec);
  return hip_check(hipGetLastError(), "k_step launch");
}

extern "C" int ssim_policy(ssim_handle* h, int32_t kind, uint64_t seed, uint64_t counter, int32_t* stage_idx,
                           int32_t* num_exec, void* stream) {
  if (h == nullptr || stage_idx == nullptr || num_exec == nullptr) return set_err(SSIM_E_ARG, "ssim_policy: null");
  if (kind != SSIM_POLICY_FAIR && kind != SSIM_POLICY_FIFO && kind != SSIM_POLICY_RANDOM)
    return set_err(SSIM_E_ARG, "ssim_policy: unknown policy %d", kind);
  const ssim_layout& L = h->params.L;
  hipLaunchKernelGGL(k_policy, dim3(L.num_envs), dim3(64), 0, (hipStream_t)stream, dparams(h), h->obs, kind,
                     seed, counter, stage_idx, num_exec);
  return hip_check(hipGetLastError(), "k_policy launch");
}

static int rollout_launch(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps, int64_t budget,
                          int32_t flags, const double* time_limits, int32_t* action_log, void* stream,
                          const int32_t* env_steps = nullptr) {
  if (h == nullptr || num_steps < 0 || budget < 0) return set_err(SSIM_E_ARG, "ssim_rollout: bad argument");
  if (kind != SSIM_POLICY_FAIR && kind != SSIM_POLICY_FIFO && kind != SSIM_POLICY_RANDOM)
    return set_err(SSIM_E_ARG, "ssim_rollout: unknown policy %d", kind);
  if ((flags & ~(SSIM_ROLLOUT_AUTORESET | SSIM_ROLLOUT_PREEMPT | SSIM_ROLLOUT_WARMUP)) != 0)
    return set_err(SSIM_E_ARG, "ssim_rollout_ex: unknown flags 0x%x", flags);
  if ((flags & SSIM_ROLLOUT_PREEMPT) && budget <= 0)
    return set_err(SSIM_E_ARG, "ssim_rollout: SSIM_ROLLOUT_PREEMPT needs a decision budget (ssim_rollout_budget)");
  if ((flags & SSIM_ROLLOUT_AUTORESET) && !(h->params.C.job_arrival_gap > 0.0))
    return set_err(SSIM_E_ARG, "ssim_rollout_ex: auto-reset needs job_arrival_gap in the config");
  const ssim_layout& L = h->params.L;
  const KernelSet ks = pick_kernels(h->params);
  const RolloutFn fn = (flags & SSIM_ROLLOUT_WARMUP) ? ks.rollout_warmup : ks.rollout;
  const int64_t lds = h->params.O.lds_bytes;
  const int rc = lds_opt_in((const void*)fn, lds);
  if (rc != SSIM_OK) return rc;
  // the budget slot this launch claims from; flipped only once the launch is enqueued (a failed launch leaves the
  // slot it would have zeroed dirty, so the next launch must use the same one again)
  if (budget > 0 && h->ticket_slot) flags |= kFlagTicketSlot;
  hipLaunchKernelGGL(fn, dim3(L.num_envs), dim3(64),
                     (size_t)lds, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, kind, seed, num_steps, flags, time_limits, h->reset, action_log,
                     (uint64_t*)nullptr, budget, env_steps);
  const int rc2 = hip_check(hipGetLastError(), "k_rollout launch");
  if (rc2 == SSIM_OK && budget > 0) h->ticket_slot ^= 1;
  return rc2;
}

extern "C" int ssim_rollout_ex(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps, int32_t flags,
                               const double* time_limits, int32_t* action_log, void* stream) {
  return rollout_launch(h, kind, seed, num_steps, 0, flags, time_limits, action_log, stream);
}

extern "C" int ssim_rollout_budget(ssim_handle* h, int32_t kind, uint64_t seed, int32_t max_steps,
                                   int64_t total_decisions, int32_t flags, const double* time_limits,
                                   int32_t* action_log, void* stream) {
  if (total_decisions <= 0) return set_err(SSIM_E_ARG, "ssim_rollout_budget: total_decisions must be > 0");
  return rollout_launch(h, kind, seed, max_steps, total_decisions, flags, time_limits, action_log, stream);
}

extern "C" int ssim_rollout_steps(ssim_handle* h, int32_t kind, uint64_t seed, const int32_t* env_steps,
                                  int32_t max_steps, int32_t flags, const double* time_limits, int32_t* action_log,
                                  void* stream) {
  if (env_steps == nullptr) return set_err(SSIM_E_ARG, "ssim_rollout_steps: null env_steps");
  return rollout_launch(h, kind, seed, max_steps, 0, flags, time_limits, action_log, stream, env_steps);
}

extern "C" int ssim_rollout(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps, int32_t* action_log,
                            void* stream) {
  return ssim_rollout_ex(h, kind, seed, num_steps, 0, nullptr, action_log, stream);
}

extern "C" int ssim_reset_sampled(ssim_handle* h, const uint8_t* mode, const uint64_t* seeds, const double* time_limits,
                                  void* stream) {
  if (h == nullptr || mode == nullptr) return set_err(SSIM_E_ARG, "ssim_reset_sampled: null argument");
  if (!(h->params.C.job_arrival_gap > 0.0))
    return set_err(SSIM_E_ARG, "ssim_reset_sampled: the config has no job_arrival_gap");
  const ssim_layout& L = h->params.L;
  hipLaunchKernelGGL(k_reset_sampled, dim3(L.num_envs), dim3(64), (size_t)L.scratch_bytes, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, h->reset, mode, seeds, time_limits);
  return hip_check(hipGetLastError(), "k_reset_sampled launch");
}

#ifdef SSIM_PROFILE
// Diagnostic build only: same rollout, per-wave phase cycle sums -> prof_out[num_envs][kNumPhases].
extern "C" int ssim_rollout_profiled(ssim_handle* h, int32_t kind, uint64_t seed, int32_t num_steps,
                                     uint64_t* prof_out, void* stream) {
  const ssim_layout& L = h->params.L;
  const KernelSet ks = pick_kernels(h->params);
  const RolloutFn fn = ks.rollout;
  const int64_t lds = h->params.O.lds_bytes;
  const int rc = lds_opt_in((const void*)fn, lds);
  if (rc != SSIM_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(L.num_envs), dim3(64), (size_t)lds, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, kind, seed, num_steps, 0, (const double*)nullptr, h->reset,
                     (int32_t*)nullptr, prof_out, (int64_t)0, (const int32_t*)nullptr);
  return hip_check(hipGetLastError(), "k_rollout(profiled) launch");
}
// Diagnostic build only: the budget rollout (as bench.py) with per-wave phase sums and realtime stamps.
extern "C" int ssim_rollout_budget_profiled(ssim_handle* h, int32_t kind, uint64_t seed, int32_t max_steps,
                                            int64_t total_decisions, int32_t flags, uint64_t* prof_out,
                                            const double* time_limits, void* stream) {
  const ssim_layout& L = h->params.L;
  if (total_decisions <= 0) return set_err(SSIM_E_ARG, "ssim_rollout_budget_profiled: total_decisions must be > 0");
  const KernelSet ks = pick_kernels(h->params);
  const RolloutFn fn = ks.rollout;
  const int64_t lds = h->params.O.lds_bytes;
  const int rc = lds_opt_in((const void*)fn, lds);
  if (rc != SSIM_OK) return rc;
  if (h->ticket_slot) flags |= kFlagTicketSlot;
  hipLaunchKernelGGL(fn, dim3(L.num_envs), dim3(64), (size_t)lds, (hipStream_t)stream,
                     dparams(h), h->state, h->obs, kind, seed, max_steps, flags, time_limits, h->reset,
                     (int32_t*)nullptr, prof_out, total_decisions, (const int32_t*)nullptr);
  const int rc2 = hip_check(hipGetLastError(), "k_rollout(budget, profiled) launch");
  if (rc2 == SSIM_OK) h->ticket_slot ^= 1;
  return rc2;
}
#endif

#ifdef SSIM_PROFILE
// Diagnostic build only: the next ssim_decima_rollout launch on `h` writes its per-wave phase sums to prof_out.
extern "C" int ssim_decima_profile_next(ssim_handle* h, uint64_t* prof_out) {
  h->prof_next = prof_out;
  return SSIM_OK;
}
#endif

extern "C" int ssim_job_times(ssim_handle* h, double* t_arrival, double* t_completed, int32_t* state, void* stream) {
  if (h == nullptr) return set_err(SSIM_E_ARG, "ssim_job_times: null handle");
  hipLaunchKernelGGL(k_job_times, dim3(h->params.L.num_envs), dim3(64), 0, (hipStream_t)stream, dparams(h), h->state,
                     t_arrival, t_completed, state);
  return hip_check(hipGetLastError(), "k_job_times launch");
}

// The set KAT (tests/test_gpu_sets.py) through the engine instantiation a launch on this handle runs: variant
// SSIM_DEBUG_ENGINE the step / rollout kernels' (pick_kernels), SSIM_DEBUG_DECIMA the persistent Decima rollout's
// (pick_decima), SSIM_DEBUG_KAT_BAD the test-only known-bad page assembly (N = 100 / J = 200, HBM-resident layouts).
static const char* debug_variant(const ssim_handle* h, int32_t variant, SetTraceFn* fn) {
  if (variant == SSIM_DEBUG_ENGINE) {
    const KernelSet k = pick_kernels(h->params);
    *fn = k.set_trace;
    return k.name;
  }
  if (variant == SSIM_DEBUG_DECIMA) {
    const DecimaRolloutSet k = pick_decima(h->params);
    *fn = k.set_trace;
    return k.name;
  }
  if (variant == SSIM_DEBUG_KAT_BAD && large_shape(h->params) && !h->params.O.lds_resident) {
    *fn = set_trace_kat_bad();
    return "kat_bad_page";
  }
  *fn = nullptr;
  return nullptr;
}

extern "C" const char* ssim_debug_kernel_name(const ssim_handle* h, int32_t variant) {
  SetTraceFn fn;
  const char* n = h != nullptr ? debug_variant(h, variant, &fn) : nullptr;
  return n != nullptr ? n : "";
}

extern "C" int ssim_debug_set_trace_ex(ssim_handle* h, const int32_t* ops, int32_t n_ops, int32_t width,
                                       int32_t* orders, int32_t variant, void* stream) {
  if (h == nullptr || ops == nullptr || orders == nullptr || n_ops < 0 || width <= 0)
    return set_err(SSIM_E_ARG, "ssim_debug_set_trace: bad argument");
  if (h->params.L.num_executors > 127 || h->params.L.job_cap < 1)
    return set_err(SSIM_E_ARG, "ssim_debug_set_trace: needs 1..127 executors and a job cap >= 1");
  SetTraceFn fn = nullptr;
  if (debug_variant(h, variant, &fn) == nullptr)
    return set_err(SSIM_E_ARG, "ssim_debug_set_trace: variant %d does not apply to this layout", variant);
  const int64_t lds = h->params.O.lds_bytes;
  const int rc = lds_opt_in((const void*)fn, lds);
  if (rc != SSIM_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(1), dim3(64), (size_t)lds, (hipStream_t)stream, dparams(h), h->state, h->obs, ops, n_ops,
                     width, orders);
  return hip_check(hipGetLastError(), "k_set_trace launch");
}

extern "C" int ssim_debug_set_trace(ssim_handle* h, const int32_t* ops, int32_t n_ops, int32_t width, int32_t* orders,
                                    void* stream) {
  return ssim_debug_set_trace_ex(h, ops, n_ops, width, orders, SSIM_DEBUG_ENGINE, stream);
}

extern "C" int ssim_decima_features(ssim_handle* h, float num_tasks_scale, float work_scale, float* node_feats,
                                    int32_t* commit_cap, uint32_t* edge_mask, int32_t* depth, void* stream) {
  if (h == nullptr || node_feats == nullptr || commit_cap == nullptr || edge_mask == nullptr || depth == nullptr)
    return set_err(SSIM_E_ARG, "ssim_decima_features: null argument");
  const ssim_layout& L = h->params.L;
  if (h->params.C.max_stages > kDecimaMaxDepth)
    return set_err(SSIM_E_ARG, "ssim_decima_features: max_stages %d > %d (edge-mask word)", h->params.C.max_stages,
                   kDecimaMaxDepth);
  const int64_t lds = decima_scratch_bytes(L.stage_cap);
  if (lds > kLdsBudget) return set_err(SSIM_E_ARG, "ssim_decima_features: stage_cap %d too large", L.stage_cap);
  hipLaunchKernelGGL(k_decima, dim3(L.num_envs), dim3(64), (size_t)lds, (hipStream_t)stream, dparams(h), h->obs,
                     num_tasks_scale, work_scale, node_feats, commit_cap, edge_mask, depth);
  return hip_check(hipGetLastError(), "k_decima launch");
}

extern "C" int ssim_decima_policy(ssim_handle* h, const float* node_feats, const int32_t* commit_cap,
                                  const uint32_t* edge_mask, const int32_t* depth, const float* params,
                                  int32_t num_params, int32_t node_cap, uint64_t seed, uint64_t counter,
                                  const uint8_t* env_mask, int32_t* stage_idx, int32_t* num_exec, int32_t* job_idx,
                                  int32_t* exec_idx, float* lgprob, float* stage_scores, float* exec_scores,
                                  int32_t* overflow, void* stream) {
  if (h == nullptr || node_feats == nullptr || commit_cap == nullptr || edge_mask == nullptr || depth == nullptr ||
      params == nullptr || stage_idx == nullptr || num_exec == nullptr || job_idx == nullptr ||
      exec_idx == nullptr || lgprob == nullptr)
    return set_err(SSIM_E_ARG, "ssim_decima_policy: null argument");
  if (num_params != kDecimaParams)
    return set_err(SSIM_E_ARG, "ssim_decima_policy: %d parameters, the fused kernel implements the "
                   "decima_tpch.yaml architecture (%d)", num_params, kDecimaParams);
  const ssim_layout& L = h->params.L;
  if (L.num_executors > 64 * kDpExecChunks)
    return set_err(SSIM_E_ARG, "ssim_decima_policy: more than %d executors", 64 * kDpExecChunks);
  if (node_cap <= 0 || node_cap > L.stage_cap) node_cap = L.stage_cap;
  if (node_cap < (L.num_executors + kDpEmb - 1) / kDpEmb) node_cap = (L.num_executors + kDpEmb - 1) / kDpEmb;
  const int64_t lds = decima_policy_lds_bytes(node_cap, L.job_cap);
  DecimaPolicyOut o{stage_idx, num_exec, job_idx, exec_idx, lgprob, stage_scores, exec_scores};
  if (h->policy_packed == nullptr) {
    const int rc = hip_check(hipMalloc(&h->policy_packed, (size_t)kDpPackedBytes), "packed weights allocation");
    if (rc != SSIM_OK) return rc;
  }
  {
    const int rc = decima_pack(params, h->policy_packed, stream);
    if (rc != SSIM_OK) return rc;
  }
  const dp_f32x4* wpk = static_cast<const dp_f32x4*>(h->policy_packed);
  if (lds > kDecimaPolicyLdsMax) {  // the plan in a handle-owned global region (grown on demand)
    const int64_t stride = (lds + 255) & ~int64_t(255), need = stride * L.num_envs;
    if (need > h->policy_plan_bytes) {
      if (h->policy_plan != nullptr) {
        int rc = hip_check(hipStreamSynchronize((hipStream_t)stream), "policy plan resize sync");
        if (rc != SSIM_OK) return rc;
        (void)hipFree(h->policy_plan);
        h->policy_plan = nullptr;
        h->policy_plan_bytes = 0;
      }
      int rc = hip_check(hipMalloc(&h->policy_plan, (size_t)need), "policy plan allocation");
      if (rc != SSIM_OK) return rc;
      h->policy_plan_bytes = need;
    }
    hipLaunchKernelGGL(k_decima_policy<true>, dim3(L.num_envs), dim3(64), 0, (hipStream_t)stream, dparams(h), h->obs,
                       node_feats, commit_cap, edge_mask, depth, wpk, node_cap, seed, counter, env_mask, o, overflow,
                       h->policy_plan, stride);
    return hip_check(hipGetLastError(), "k_decima_policy(global plan) launch");
  }
  {
    const int rc = lds_opt_in((const void*)k_decima_policy<false>, lds);
    if (rc != SSIM_OK) return rc;
  }
  hipLaunchKernelGGL(k_decima_policy<false>, dim3(L.num_envs), dim3(64), (size_t)lds, (hipStream_t)stream,
                     dparams(h), h->obs, node_feats, commit_cap, edge_mask, depth, wpk, node_cap, seed, counter,
                     env_mask, o, overflow, (uint8_t*)nullptr, (int64_t)0);
  return hip_check(hipGetLastError(), "k_decima_policy launch");
}

// The persistent Decima rollout's LDS plan (decima_rollout.h): the policy's per-node rows for observations of up to
// `cap` nodes in the wave's LDS, after the engine's own LDS (`off` relative to the scratch block), within the env's
// share of its CU (StateOffsets::lds_share: the share compute_layout's residency decision assumed, so the plan never
// lowers the workgroups per CU the layout counted on).
struct DecimaLdsPlan {
  int32_t cap, off;
  int64_t lds;       // dynamic LDS of the launch
  int32_t help_off;  // the exec-score helpers' mailbox (units with helper waves), after the rest
};
static DecimaLdsPlan decima_lds_plan(const Params& P, const DecimaRolloutSet& ks) {
  const StateOffsets& O = P.O;
  const ssim_layout& L = P.L;
  DecimaLdsPlan pl{0, 0, O.lds_bytes, 0};
  const int64_t help = ks.waves > 1 ? dp_help_bytes(L.num_executors) : 0;
  const int64_t eng = O.lds_resident ? O.hot_bytes + O.scratch_bytes : O.scratch_hbm_bytes;  // (HBM: row map cold)
  // Engines without the duration-descriptor cache hold only per-operation temporaries in their LDS scratch (set
  // tables, key lists, the commitment plan, observe()'s stage -> row map), none live across a decision: the plan
  // overlays them. (Round 6: LDS-resident engines too — the PPO collect's J = 200 / N = 50 envs keep a 146 KB hot block
  // in a CU's 160 KB, and overlaying their 10.8 KB scratch takes the plan from ~8 to ~60 nodes, so nearly every
  // decision's policy runs from LDS instead of the global plan.)
#ifdef SSIM_PROFILE
  const bool overlay = false;  // (the profile sums live in the scratch)
#else
  const bool overlay = L.num_executors > kDurCacheMaxExecs;
#endif
  // (past the LDS copy of the executor records, sc_execs, when the HBM-resident engine keeps one for the launch)
  const int64_t off = overlay ? (!O.lds_resident && SSIM_DR_EX_LDS ? O.sc_keys_a : 0)
                              : align16(O.lds_resident ? O.scratch_bytes : O.scratch_hbm_bytes);
  const int64_t base = O.lds_resident ? O.hot_bytes : 0;  // (the plan offset is relative to the scratch block)
  const int64_t room = O.lds_share - base - off - help;
  int cap = 0;
  while (cap < L.stage_cap && decima_policy_lds_bytes(cap + 1, kDpLdsDags) <= room &&
         decima_scratch_bytes(cap + 1) <= room)
    ++cap;
  pl.cap = cap;
  pl.off = (int32_t)off;
  if (cap > 0) {
    const int64_t need = base + off + decima_policy_lds_bytes(cap, kDpLdsDags);
    pl.lds = need > align16(eng) ? need : align16(eng);
  }
  if (help > 0) {
    pl.help_off = (int32_t)align16(pl.lds);
    pl.lds = pl.help_off + help;
  }
  return pl;
}

extern "C" int64_t ssim_decima_rollout_lds_bytes(const ssim_handle* h) {
  if (h == nullptr) return set_err(SSIM_E_ARG, "ssim_decima_rollout_lds_bytes: null handle");
  return decima_lds_plan(h->params, pick_decima(h->params)).lds;
}

extern "C" int64_t ssim_decima_workspace_bytes(const ssim_handle* h) {
  if (h == nullptr) return set_err(SSIM_E_ARG, "ssim_decima_workspace_bytes: null handle");
  return decima_work(h->params.L).total;
}

extern "C" int ssim_decima_rollout(ssim_handle* h, const float* params, int32_t num_params, float num_tasks_scale,
                                   float work_scale, uint64_t seed, uint64_t counter, int32_t max_steps,
                                   int64_t total_decisions, int32_t flags, const double* time_limits, void* workspace,
                                   int64_t workspace_bytes, const ssim_decima_samples* samples, int32_t* action_log,
                                   void* stream) {
  if (h == nullptr || params == nullptr || workspace == nullptr || max_steps < 0 || total_decisions < 0)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: bad argument");
  if (num_params != kDecimaParams)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: %d parameters, the fused kernel implements the "
                   "decima_tpch.yaml architecture (%d)", num_params, kDecimaParams);
  if ((flags & ~(SSIM_ROLLOUT_AUTORESET | SSIM_ROLLOUT_PREEMPT | SSIM_ROLLOUT_WARMUP | SSIM_ROLLOUT_TEST_REJECT)) != 0)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: unknown flags 0x%x", flags);
  if ((flags & SSIM_ROLLOUT_PREEMPT) && total_decisions <= 0)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: SSIM_ROLLOUT_PREEMPT needs a decision budget");
  if ((flags & SSIM_ROLLOUT_AUTORESET) && !(h->params.C.job_arrival_gap > 0.0))
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: auto-reset needs job_arrival_gap in the config");
  const ssim_layout& L = h->params.L;
  if (h->params.C.max_stages > kDecimaMaxDepth)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: max_stages %d > %d (edge-mask word)", h->params.C.max_stages,
                   kDecimaMaxDepth);
  if (L.num_executors > 64 * kDpExecChunks)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: more than %d executors", 64 * kDpExecChunks);
  const DecimaWork wl = decima_work(L);
  if (workspace_bytes < wl.total)
    return set_err(SSIM_E_ARG, "ssim_decima_rollout: workspace of %lld B, needs %lld (ssim_decima_workspace_bytes)",
                   (long long)workspace_bytes, (long long)wl.total);
  DecimaRolloutArgs a{};
  a.weights = reinterpret_cast<const dp_f32x4*>(static_cast<uint8_t*>(workspace) + wl.packed);
  a.work = static_cast<uint8_t*>(workspace);
  {
    const int rc = decima_pack(params, static_cast<uint8_t*>(workspace) + wl.packed, stream);
    if (rc != SSIM_OK) return rc;
  }
  a.wl = wl;
  a.num_tasks_scale = num_tasks_scale;
  a.work_scale = work_scale;
  a.seed = seed;
  a.counter = counter;
  if (samples != nullptr) {
    const ssim_decima_samples& sm = *samples;
    if (sm.cursor == nullptr || sm.rec == nullptr || sm.nodes == nullptr || sm.edges == nullptr || sm.dags == nullptr ||
        sm.cap_samples <= 0 || sm.cap_nodes < 0 || sm.cap_edges < 0 || sm.cap_dags < 0)
      return set_err(SSIM_E_ARG, "ssim_decima_rollout: incomplete sample arena");
    a.smp = sm;
  }
  const DecimaRolloutSet ks = pick_decima(h->params);
  const DecimaRolloutFn fn = (flags & SSIM_ROLLOUT_WARMUP) ? ks.rollout_warmup : ks.rollout;
  const DecimaLdsPlan pl = decima_lds_plan(h->params, ks);
  a.plan_cap = pl.cap;
  a.plan_off = pl.off;
  a.help_off = pl.help_off;
  const int64_t lds = pl.lds;
  const int rc = lds_opt_in((const void*)fn, lds);
  if (rc != SSIM_OK) return rc;
  if (total_decisions > 0 && h->ticket_slot) flags |= kFlagTicketSlot;
  hipLaunchKernelGGL(fn, dim3(L.num_envs), dim3(64 * ks.waves), (size_t)lds, (hipStream_t)stream, dparams(h),
                     h->state, h->obs, a, max_steps, flags, time_limits, h->reset, action_log, total_decisions,
                     h->prof_next);
  h->prof_next = nullptr;
  const int rc2 = hip_check(hipGetLastError(), "k_decima_rollout launch");
  if (rc2 == SSIM_OK && total_decisions > 0) h->ticket_slot ^= 1;
  return rc2;
}

extern "C" const char* ssim_last_error(void) { return g_err; }

#ifndef SSIM_BUILD_ID
#define SSIM_BUILD_ID "unversioned"
#endif
extern "C" const char* ssim_build_id(void) { return SSIM_BUILD_ID; }
