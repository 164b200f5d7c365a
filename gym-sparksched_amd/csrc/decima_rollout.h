// decima_rollout.h — persistent Decima rollouts: featurisation, the GNN policy and env.step per env in ONE launch.
//
// The reference collects Decima rollouts one env per process (trainers/rollout_worker.py:135-157: per decision
// DecimaObsWrapper.observation, DecimaScheduler.schedule, env.step). The lockstep GPU collector batches that over
// envs but pays ~4 launches and a host sync per decision, and every decision waits for the slowest env of the batch.
// Here each env's wave runs its own loop (kernels.h rollout_body): the Decima features of its current observation
// (decima.h), the fused policy (decima_policy.h), optionally a copy of the observation / action / reward into a
// per-env sample arena (the PPO learner's rollout buffer), then the step. No env waits for another; a launch runs
// whole episodes (collection) or a shared decision budget (benchmark, SSIM_ROLLOUT_PREEMPT | AUTORESET).
//
// The features' scratch and the policy's activation plan live in the wave's LDS share (the HBM-resident kernels run
// 16 one-wave workgroups per CU: 10 KB each, overlaying the engine's per-operation scratch) for observations of up to
// ~30 nodes and 16 DAGs (~9 in 10 decisions at J = 200), else in a per-env region of global memory (the workspace,
// sized for the stage cap). The policy weights are packed per launch (k_decima_pack) into the operand order of the
// matrix cores (decima_policy.h), a coalesced 16-B load per lane per four MFMA steps.
// Sampling: counter-based Gumbel-max on (seed, env, counter + the env's decision index in its episode), plus the
// episode number << 32 with auto-reset — the lockstep collector's stream (RolloutCollector: counter = base + k at
// its k-th step), so both collectors draw the same actions for the same observations.
#pragma once
#include "kernels.h"
#include "decima.h"
#include "decima_policy.h"

// 1: the HBM-resident Decima rollout keeps the executor records in LDS for the launch (Sim ex_lds), after which the
// policy plan starts (sparksched.hip decima_lds_plan); 0 (default): in HBM, and the plan takes the wave's whole LDS share
// from the scratch's start. The larger plan keeps more observations off the global plan: measured 2.82e7 vs 2.77e7
// decisions/s, HBM writes 5.8 vs 8.0 KB per decision (profiles/r06/decima_ex_lds/).
#ifndef SSIM_DR_EX_LDS
#define SSIM_DR_EX_LDS 0
#endif

// Per-env global workspace: [features scratch (decima.h) | policy plan for stage_cap nodes (decima_policy.h)], then
// the feature outputs for all envs (the ssim_decima_features layout).
struct DecimaWork {
  int64_t feat_scratch, plan, stride;  // per-env block
  int64_t feats, ccap, emask, depth;  // absolute offsets of the [num_envs] feature arrays
  int64_t packed, total;              // the packed policy weights (kDpPackedBytes), then the end
};
inline DecimaWork decima_work(const ssim_layout& L) {
  DecimaWork w{};
  w.feat_scratch = 0;
  w.plan = align16(decima_scratch_bytes(L.stage_cap));
  w.stride = (w.plan + decima_policy_lds_bytes(L.stage_cap, L.job_cap) + 255) & ~int64_t(255);
  int64_t o = w.stride * L.num_envs;
  w.feats = o;
  o = align16(o + (int64_t)L.num_envs * L.stage_cap * kDecimaFeatures * 4);
  w.ccap = o;
  o = align16(o + (int64_t)L.num_envs * L.job_cap * 4);
  w.emask = o;
  o = align16(o + (int64_t)L.num_envs * L.edge_cap * 4);
  w.depth = o;
  o = align16(o + (int64_t)L.num_envs * 4);
  w.packed = (o + 255) & ~int64_t(255);
  w.total = w.packed + kDpPackedBytes;
  return w;
}

struct DecimaRolloutArgs {
  const dp_f32x4* weights;  // the packed policy weights (decima_policy.h DpPacked; k_decima_pack of the parameters)
  uint8_t* work;         // decima_work(L).total bytes
  DecimaWork wl;
  float num_tasks_scale, work_scale;
  uint64_t seed, counter;
  int32_t autoreset;
  int32_t test_reject;      // SSIM_ROLLOUT_TEST_REJECT (test hook): the launch's first decision asks for N + 1 executors
  // The LDS plan: an observation of at most plan_cap nodes runs the features' scratch and the policy's activations in
  // the wave's LDS, at byte plan_off of its scratch block (what the layout would give the row map and the rest of the
  // CU's share; the engine keeps its row map in the cold block). Larger ones use the env's global workspace.
  int32_t plan_cap, plan_off;
  int32_t help_off;  // the exec-score helpers' mailbox (decima_policy.h DpHelp): byte offset in the workgroup's LDS
  ssim_decima_samples smp;  // smp.rec == nullptr: no sample arena
};

// The Decima decision of one env's current observation: its features (decima.h) and the fused policy
// (decima_policy.h), with the features' scratch and the policy's plan in the wave's LDS at byte `plan_lds` when the
// observation has at most `plan_cap` nodes (0: in the env's global workspace: feat_scratch / plan). (Inlined: as a
// call, the calling convention saved every live register around it, 1.2 KB per lane of scratch.) kHelp: the exec
// scores on the workgroup's helper waves, through the mailbox at LDS byte `help_lds` (decima_policy.h dp_exec_tiles).
template <bool kHelp = false>
__device__ __forceinline__ DpAction decima_decide(
    const Params* P0, const uint8_t* obs0, const dp_f32x4* weights0, uint8_t* feat_scratch0, uint8_t* plan0,
    float* feats0, int32_t* ccap0, uint32_t* emask0, int32_t* depth0, float num_tasks_scale, float work_scale,
    uint64_t seed, uint64_t ctr, int eid, int plan_cap, uint32_t plan_lds, uint64_t* pprof, uint32_t help_lds = 0) {
  using W = WaveHip;
  const Params* P = (const Params*)(const SSIM_GLOBAL Params*)P0;
  const uint8_t* obs = (const uint8_t*)(const SSIM_GLOBAL uint8_t*)obs0;
  const dp_f32x4* weights = (const dp_f32x4*)(const SSIM_GLOBAL dp_f32x4*)weights0;
  float* feats = (float*)(SSIM_GLOBAL float*)feats0;
  int32_t* ccap = (int32_t*)(SSIM_GLOBAL int32_t*)ccap0;
  uint32_t* emask = (uint32_t*)(SSIM_GLOBAL uint32_t*)emask0;
  int32_t* depth = (int32_t*)(SSIM_GLOBAL int32_t*)depth0;
  const ssim_layout& L = P->L;
  const DecimaPolicyOut none{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  const DpWGlobal wts{weights};
  DpAction act;
  DpHelp* const help = kHelp ? reinterpret_cast<DpHelp*>(g_smem + help_lds) : nullptr;
#ifdef SSIM_PROFILE
  uint64_t tp = W::clock();
#endif
#ifdef SSIM_DR_GLOBAL_ONLY
  if (false) {  // (A/B builds: the global plan only)
#else
  if (plan_cap > 0) {  // the LDS plan (wave-local: cheap syncs, no global round trips per phase)
#endif
    uint8_t* pl = g_smem + plan_lds;
    DecimaView<W>{L, obs, eid}.template run<false>(num_tasks_scale, work_scale, pl, feats, ccap, emask, depth,
                                                   plan_cap);
#ifdef SSIM_PROFILE
    if (pprof != nullptr && W::lane() == 0) W::lds_add_u64(pprof - kPhDecParts + kPhDecFeat, W::clock() - tp);
#endif
    decima_policy_env<false, kHelp>(P, obs, feats, ccap, emask, depth, wts, plan_cap, seed, ctr, eid, pl, none, &act,
                                    pprof, kDpLdsDags, help);
  } else {  // the env's global workspace
    uint8_t* fs = (uint8_t*)(SSIM_GLOBAL uint8_t*)feat_scratch0;
    uint8_t* pg = (uint8_t*)(SSIM_GLOBAL uint8_t*)plan0;
    DecimaView<W>{L, obs, eid}.template run<true>(num_tasks_scale, work_scale, fs, feats, ccap, emask, depth);
#ifdef SSIM_PROFILE
    if (pprof != nullptr && W::lane() == 0) W::lds_add_u64(pprof - kPhDecParts + kPhDecFeat, W::clock() - tp);
#endif
    decima_policy_env<true, kHelp>(P, obs, feats, ccap, emask, depth, wts, L.stage_cap, seed, ctr, eid, pg, none, &act,
                                   pprof, 0, help);
  }
  return act;
}

template <bool kHelp = false>
struct DecimaPolicy {
  const Params* P;
  const uint8_t* obs;
  DecimaRolloutArgs a;

  // Whether act() goes on to choose an action (rollout_body asks before it claims a budgeted decision): not when the
  // collector's episode is over (terminated, truncated by its StochasticTimeLimit, or frozen) or when the sample arena
  // cannot hold the current observation (the region-full mark is set for the host, which grows the arena and launches
  // again).
  template <class S>
  __device__ __forceinline__ bool can_act(const S& s) const {
    using W = WaveHip;
    if (!a.autoreset && (s.h.terminated || s.frozen() || s.h.wall >= s.h.time_limit || s.h.num_jobs == 0))
      return false;
    const ssim_decima_samples& sm = a.smp;
    if (sm.rec == nullptr) return true;
    const int32_t* cnt = reinterpret_cast<const int32_t*>(obs + P->L.ob_counts) + (int64_t)s.eid * SSIM_NUM_COUNTS;
    int32_t* cur = sm.cursor + (int64_t)s.eid * 8;
    if (W::uni(cur[0]) + 1 > sm.cap_samples || W::uni(cur[1]) + W::uni(cnt[SSIM_OC_NUM_NODES]) > sm.cap_nodes ||
        W::uni(cur[2]) + W::uni(cnt[SSIM_OC_NUM_EDGES]) > sm.cap_edges ||
        W::uni(cur[3]) + W::uni(cnt[SSIM_OC_NUM_JOBS]) > sm.cap_dags) {
      W::sync();
      if (W::lane() == 0) {  // region full: the host grows the arena (to fit what is recorded here), launches again
        cur[4] = 1;
        cur[5] = W::uni(cnt[SSIM_OC_NUM_NODES]);
        cur[6] = W::uni(cnt[SSIM_OC_NUM_EDGES]);
        cur[7] = W::uni(cnt[SSIM_OC_NUM_JOBS]);
      }
      W::sync();
      return false;
    }
    return true;
  }
  template <class S>
  __device__ __forceinline__ bool act(S& s, int k, StepIn* out) const {
    using W = WaveHip;
    const ssim_layout& L = P->L;
    const int eid = s.eid;
    // (rollout_body calls can_act() first: an arena-full or finished env never gets here)
    const ssim_decima_samples& sm = a.smp;
    const int32_t* cnt = reinterpret_cast<const int32_t*>(obs + L.ob_counts) + (int64_t)eid * SSIM_NUM_COUNTS;
    const int n = W::uni(cnt[SSIM_OC_NUM_NODES]), ne = W::uni(cnt[SSIM_OC_NUM_EDGES]);
    const int nj = W::uni(cnt[SSIM_OC_NUM_JOBS]);
    int32_t* cur = sm.cursor + (int64_t)eid * 8;
    int cs = 0, cn = 0, ce = 0, cg = 0;
    if (sm.rec != nullptr) {
      cs = W::uni(cur[0]);
      cn = W::uni(cur[1]);
      ce = W::uni(cur[2]);
      cg = W::uni(cur[3]);
    }
#ifdef SSIM_PROFILE
    uint64_t tp = W::clock();
#endif
    SSIM_MARK("decima_act_begin");
    uint8_t* wk = a.work + (int64_t)eid * a.wl.stride;
    float* feats = reinterpret_cast<float*>(a.work + a.wl.feats);
    int32_t* ccap = reinterpret_cast<int32_t*>(a.work + a.wl.ccap);
    uint32_t* emask = reinterpret_cast<uint32_t*>(a.work + a.wl.emask);
    int32_t* depth = reinterpret_cast<int32_t*>(a.work + a.wl.depth);
    const uint64_t ctr = a.counter + (uint64_t)s.h.decisions + (a.autoreset ? (uint64_t)s.h.episode << 32 : 0ull);
#ifdef SSIM_PROFILE
    uint64_t* pprof = s.prof + kPhDecParts;
#else
    uint64_t* pprof = nullptr;
#endif
    const bool lds_plan = n <= a.plan_cap && nj <= kDpLdsDags;
    SSIM_MARK("decima_policy_begin");
    const DpAction act = decima_decide<kHelp>(P, obs, a.weights, wk + a.wl.feat_scratch, wk + a.wl.plan, feats, ccap, emask,
                                       depth, a.num_tasks_scale, a.work_scale, a.seed, ctr, eid,
                                       lds_plan ? a.plan_cap : 0,
                                       (uint32_t)(s.scr + a.plan_off - g_smem), pprof, (uint32_t)a.help_off);
    SSIM_MARK("decima_policy_end");
#ifdef SSIM_PROFILE
    s.prof_add(kPhDecPolicy, W::clock() - tp);
    tp = W::clock();
#endif
    out->stage_idx = act.stage_idx;
    out->num_exec = act.num_exec;
    if (a.test_reject && k == 0) out->num_exec = L.num_executors + 1;  // (test hook: an action the env refuses)
    if (sm.rec != nullptr) {  // the observation as the learner's DagBatch rows (schedulers/decima.py build_batch)
      const float* f = feats + (int64_t)eid * L.stage_cap * kDecimaFeatures;
      const float* nodes = reinterpret_cast<const float*>(obs + L.ob_nodes) + (int64_t)eid * L.stage_cap * 3;
      const int64_t* links = reinterpret_cast<const int64_t*>(obs + L.ob_edge_links) + (int64_t)eid * L.edge_cap * 2;
      const int32_t* ptr = reinterpret_cast<const int32_t*>(obs + L.ob_dag_ptr) + (int64_t)eid * (L.job_cap + 1);
      const int32_t* cc = ccap + (int64_t)eid * L.job_cap;
      const uint32_t* em = emask + (int64_t)eid * L.edge_cap;
      float* xn = sm.nodes + ((int64_t)eid * sm.cap_nodes + cn) * 6;
      for (int i = W::lane(); i < n; i += W::kWidth) {
#pragma unroll
        for (int c = 0; c < kDecimaFeatures; ++c) xn[(int64_t)i * 6 + c] = f[(int64_t)i * kDecimaFeatures + c];
        xn[(int64_t)i * 6 + 5] = nodes[3 * i + 2];
      }
      int32_t* ed = sm.edges + ((int64_t)eid * sm.cap_edges + ce) * 4;
      for (int e = W::lane(); e < ne; e += W::kWidth) {
        ed[4 * e + 0] = (int32_t)links[2 * e];
        ed[4 * e + 1] = (int32_t)links[2 * e + 1];
        ed[4 * e + 2] = (int32_t)em[e];
        ed[4 * e + 3] = 0;
      }
      int32_t* dg = sm.dags + ((int64_t)eid * sm.cap_dags + cg) * 2;
      for (int k = W::lane(); k < nj; k += W::kWidth) {
        dg[2 * k + 0] = ptr[k + 1] - ptr[k];
        dg[2 * k + 1] = cc[k];
      }
      const int dep = W::uni(depth[eid]);
      W::sync();
      if (W::lane() == 0) {
        ssim_decima_sample r;
        r.num_nodes = n;
        r.num_edges = ne;
        r.num_dags = nj;
        r.depth = dep;
        r.node_off = cn;
        r.edge_off = ce;
        r.dag_off = cg;
        r.stage_idx = act.stage_idx;
        r.job_idx = act.job_idx;
        r.exec_idx = act.exec_idx;
        r.num_exec = act.num_exec;
        r.lgprob = act.lgprob;
        r.wall_before = s.h.wall;
        r.reward = 0.0;
        sm.rec[(int64_t)eid * sm.cap_samples + cs] = r;
        cur[0] = cs + 1;
        cur[1] = cn + n;
        cur[2] = ce + ne;
        cur[3] = cg + nj;
      }
      W::sync();
    }
#ifdef SSIM_PROFILE
    s.prof_add(kPhDecRecord, W::clock() - tp);
#endif
    SSIM_MARK("decima_act_end");
    return true;
  }
  // the decision's reward (observe() wrote it to the obs arena) into its sample
  template <class S>
  __device__ __forceinline__ void done(S& s) const {
    using W = WaveHip;
    const ssim_decima_samples& sm = a.smp;
    if (sm.rec == nullptr) return;
    const int eid = s.eid;
    const int cs = W::uni(sm.cursor[(int64_t)eid * 8]);
    const double r = W::uni(reinterpret_cast<const double*>(obs + P->L.ob_reward)[eid]);
    W::sync();
    if (W::lane() == 0 && cs > 0) sm.rec[(int64_t)eid * sm.cap_samples + cs - 1].reward = r;
    W::sync();
  }
  // The env refused the action act() recorded (it is frozen with SSIM_ERR_INVARIANT, the collector raises): the
  // sample and its observation rows come off the arena, so no sample ever holds an action the env did not take.
  template <class S>
  __device__ __forceinline__ void rejected(S& s) const {
    using W = WaveHip;
    const ssim_decima_samples& sm = a.smp;
    if (sm.rec == nullptr) return;
    W::sync();
    if (W::lane() == 0) {
      int32_t* cur = sm.cursor + (int64_t)s.eid * 8;
      const int cs = cur[0];
      if (cs > 0) {
        const ssim_decima_sample& r = sm.rec[(int64_t)s.eid * sm.cap_samples + cs - 1];
        cur[1] -= r.num_nodes;
        cur[2] -= r.num_edges;
        cur[3] -= r.num_dags;
        cur[0] = cs - 1;
      }
    }
    W::sync();
  }
};

#ifndef SSIM_DECIMA_ROLLOUT_WAVES
#define SSIM_DECIMA_ROLLOUT_WAVES 4
#endif
// kN / kJ: executor count and job cap as compile-time constants (0 = read from the layout), as kernels.h. kHelp: the
// workgroup is kDpHelpWaves waves; wave 0 runs the env, the others its exec-score tiles (decima_policy.h), until wave 0
// publishes kDpHelpExit at the end of its rollout (every path out of rollout_body comes back here).
template <bool kRes, int kN, int kJ, bool kHelp>
__device__ __forceinline__ void decima_rollout_body(const Params* __restrict__ P, uint8_t* state, uint8_t* obs,
                                                    DecimaRolloutArgs a, int num_steps, int flags,
                                                    const double* __restrict__ limits, uint8_t* reset,
                                                    int32_t* action_log, int64_t budget, uint64_t* prof_out) {
  DpHelp* const help = reinterpret_cast<DpHelp*>(g_smem + a.help_off);
  if constexpr (kHelp) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (wv != 0) {
      const DpWGlobal wts{(const dp_f32x4*)(const SSIM_GLOBAL dp_f32x4*)a.weights};
      dp_help_loop(wts, help, kN > 0 ? kN : P->L.num_executors, wv);
      return;
    }
  }
  a.autoreset = (flags & SSIM_ROLLOUT_AUTORESET) != 0;
  a.test_reject = (flags & SSIM_ROLLOUT_TEST_REJECT) != 0;
  const DecimaPolicy<kHelp> pol{P, obs, a};
  rollout_body<kRes, kN, kJ, 0, DecimaPolicy<kHelp>>(P, state, obs, pol, num_steps, flags, limits, reset, action_log,
                                                     prof_out, budget, nullptr, !kRes, SSIM_DR_EX_LDS != 0);
  if constexpr (kHelp) {
    if (WaveHip::lane() == 0) help->cmd = kDpHelpExit;
    __syncthreads();  // the helpers' barrier A: they read the exit and end
  }
}
#define SSIM_DR_WAVES(kRes) ((kRes) ? 1 : SSIM_DECIMA_ROLLOUT_WAVES)
#define SSIM_DR_THREADS(kHelp) ((kHelp) ? 64 * kDpHelpWaves : 64)
template <bool kRes, int kN = 0, int kJ = 0, bool kHelp = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, SSIM_DR_THREADS(kHelp)), amdgpu_waves_per_eu(SSIM_DR_WAVES(kRes)))) void k_decima_rollout(
    const Params* __restrict__ P, uint8_t* state, uint8_t* obs, DecimaRolloutArgs a, int num_steps, int flags,
    const double* __restrict__ limits, uint8_t* reset, int32_t* action_log, int64_t budget, uint64_t* prof_out) {
  decima_rollout_body<kRes, kN, kJ, kHelp>(P, state, obs, a, num_steps, flags, limits, reset, action_log, budget,
                                           prof_out);
}
// launches that are not measured (SSIM_ROLLOUT_WARMUP), under their own symbol
template <bool kRes, int kN = 0, int kJ = 0, bool kHelp = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, SSIM_DR_THREADS(kHelp)), amdgpu_waves_per_eu(SSIM_DR_WAVES(kRes)))) void k_decima_rollout_warmup(
    const Params* __restrict__ P, uint8_t* state, uint8_t* obs, DecimaRolloutArgs a, int num_steps, int flags,
    const double* __restrict__ limits, uint8_t* reset, int32_t* action_log, int64_t budget, uint64_t* prof_out) {
  decima_rollout_body<kRes, kN, kJ, kHelp>(P, state, obs, a, num_steps, flags, limits, reset, action_log, budget,
                                           prof_out);
}

using DecimaRolloutFn = void (*)(const Params*, uint8_t*, uint8_t*, DecimaRolloutArgs, int, int, const double*,
                                 uint8_t*, int32_t*, int64_t, uint64_t*);
struct DecimaRolloutSet {
  DecimaRolloutFn rollout, rollout_warmup;
  SetTraceFn set_trace;  // the set KAT through this unit's engine instantiation (kernels.h k_set_trace)
  const char* name;      // the translation unit (ssim_debug_kernel_name)
  int waves = 1;         // waves per env's workgroup (kDpHelpWaves: the exec-score helpers)
};
DecimaRolloutSet decima_rollout_hbm();    // k_dr_hbm.hip
DecimaRolloutSet decima_rollout_hbm50();  // k_dr_hbm50.hip: 50 executors / 200 jobs
DecimaRolloutSet decima_rollout_lds();    // k_dr_lds.hip
DecimaRolloutSet decima_rollout_lds50();  // k_dr_lds50.hip: 50 executors / 200 jobs
