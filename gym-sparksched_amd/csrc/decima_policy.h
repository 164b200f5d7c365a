// decima_policy.h — fused Decima GNN policy (inference + action sampling), one wavefront per env.
//
// The rollout-time forward of schedulers/decima/scheduler.py:70-101 (DecimaScheduler.schedule: encoder,
// stage policy, exec policy, utils.sample) for the reference architecture of config/decima_tpch.yaml:66-78
// (embed 16; GNN MLPs 5|16|21 -> 32 -> 16 -> 16 with LeakyReLU(0.2); policy MLPs 53|36 -> 64 -> 64 -> 1
// with Tanh), reading the obs arena and the ssim_decima_features outputs directly. The batched PyTorch
// module (spark_sched_sim/schedulers/decima.py) is the same math in ~150 small launches per decision; this
// kernel is one launch, with every node's activations in LDS and the weights read through the scalar cache
// (uniform addresses), each lane evaluating one node's (or edge's, DAG's, exec action's) MLP.
//
// Semantics per env (matching DecimaScheduler.schedule):
//   h_init = mlp_prep(x); without message-passing levels h = h_init (_forward_no_mp), else leaves
//   (no child edges) start at mlp_update(h_init) and levels depth-2 .. 0 run: for the level's edges
//   (parent p, child c) agg[p] += mlp_msg(h[c]) (old h), then h[p] = h_init[p] + mlp_update(agg[p]);
//   h_dag[g] = sum over the DAG's nodes of mlp_dag([x, h]); h_glob = sum over DAGs of mlp_glob(h_dag);
//   stage scores over schedulable nodes from [x, h, h_dag, h_glob], exec scores for k < commit cap of the
//   chosen node's DAG from [x_dag[:3], h_dag, h_glob, k/N]; each choice is a categorical draw from the
//   softmax (Gumbel-max with a counter-based device RNG), lgprob = log p(stage) + log p(exec).
// fp32 throughout (the reference's dtype); sums run in a different order than torch's, so scores agree
// within float rounding (tests/test_decima_policy.py compares with the PyTorch module).
#pragma once
#include <stdint.h>

#include "decima.h"
#include "policy.h"
#include "wave_hip.h"

namespace ssim {

constexpr int kDpEmb = 16;
constexpr int kDpExecChunks = 4;  // exec actions per env: N <= 64 * kDpExecChunks (escore reuses agg rows)
template <int IN, int H1, int H2, int OUT>
struct Mlp3 {  // torch nn.Linear layout: weight [out][in] row-major, then bias, per layer
  static constexpr int kParams = H1 * IN + H1 + H2 * H1 + H2 + OUT * H2 + OUT;
};
using MlpPrep = Mlp3<kDecimaFeatures, 32, 16, kDpEmb>;
using MlpMsg = Mlp3<kDpEmb, 32, 16, kDpEmb>;
using MlpDag = Mlp3<kDecimaFeatures + kDpEmb, 32, 16, kDpEmb>;
using MlpStage = Mlp3<kDecimaFeatures + 3 * kDpEmb, 64, 64, 1>;
using MlpExec = Mlp3<3 + 2 * kDpEmb + 1, 64, 64, 1>;
// parameter offsets in DecimaScheduler.parameters() order
constexpr int kOffPrep = 0;
constexpr int kOffMsg = kOffPrep + MlpPrep::kParams;
constexpr int kOffUpd = kOffMsg + MlpMsg::kParams;
constexpr int kOffDag = kOffUpd + MlpMsg::kParams;
constexpr int kOffGlob = kOffDag + MlpDag::kParams;
constexpr int kOffStage = kOffGlob + MlpMsg::kParams;
constexpr int kOffExec = kOffStage + MlpStage::kParams;
constexpr int kDecimaParams = kOffExec + MlpExec::kParams;  // 20802

constexpr int64_t kDecimaPolicyLdsMax = 160 * 1024;  // gfx950 LDS per workgroup (opt-in above 64 KB)

// LDS plan per env: h_init, h, agg [cap][16] f32, score f32 [cap], node->DAG i16 [cap], flags u8 [cap]
// (bit0 has-child, bit1 level dst), h_dag [J][16] f32, glob [16] f32.
struct DpLds {
  int64_t hi, hh, agg, score, ndag, flag, hdag, glob, total;
};
__host__ __device__ inline DpLds dp_lds(int64_t cap, int64_t job_cap) {
  DpLds o{};
  int64_t b = 0;
  o.hi = b;
  b += cap * kDpEmb * 4;
  o.hh = b;
  b += cap * kDpEmb * 4;
  o.agg = b;
  b += cap * kDpEmb * 4;
  o.score = b;
  b += cap * 4;
  o.ndag = b;
  b = align16(b + cap * 2);
  o.flag = b;
  b = align16(b + cap);
  o.hdag = b;  // one row per active job: a job with no active stage is complete, so #jobs <= #nodes <= cap
  b += (job_cap < cap ? job_cap : cap) * kDpEmb * 4;
  o.glob = b;
  b += kDpEmb * 4;
  o.total = align16(b);
  return o;
}
inline int64_t decima_policy_lds_bytes(int64_t node_cap, int64_t job_cap) { return dp_lds(node_cap, job_cap).total; }

__device__ __forceinline__ float dp_leaky(float v) { return v >= 0.0f ? v : 0.2f * v; }

// One lane's 3-layer MLP (act between layers, none after the last), weights via uniform addresses.
// Packed layout per MLP (ssim_decima_policy): the FIRST layer's weight transposed ([IN][H1]) so the input loop
// runs outermost over contiguous rows (each input is consumed once, only the H1 accumulators stay live);
// layers 2 and 3 fused (each hidden-2 unit is activated and folded into the outputs at once, no H2 array).
// Every sum runs in the same order as before (bias first, then ascending inputs), so the scores are
// bit-identical to the unfused form.
template <int IN, int H1, int H2, int OUT, bool kTanh>
__device__ __forceinline__ void dp_mlp(const float* __restrict__ p, const float* in, float* out) {
  const float* W0t = p;  // [IN][H1]
  const float* b0 = W0t + H1 * IN;
  const float* W1 = b0 + H1;  // [H2][H1]
  const float* b1 = W1 + H2 * H1;
  const float* W2 = b1 + H2;  // [OUT][H2]
  const float* b2 = W2 + OUT * H2;
  float a[H1];
#pragma unroll
  for (int j = 0; j < H1; ++j) a[j] = b0[j];
#pragma unroll 1
  for (int i = 0; i < IN; ++i) {
    const float v = in[i];
#pragma unroll
    for (int j = 0; j < H1; ++j) a[j] = __builtin_fmaf(W0t[i * H1 + j], v, a[j]);
  }
#pragma unroll
  for (int j = 0; j < H1; ++j) a[j] = kTanh ? tanhf(a[j]) : dp_leaky(a[j]);
  float o[OUT];
#pragma unroll
  for (int k = 0; k < OUT; ++k) o[k] = b2[k];
#pragma unroll 1
  for (int j = 0; j < H2; ++j) {  // not unrolled: one weight row (H1 floats) in SGPRs at a time
    float acc = b1[j];
#pragma unroll
    for (int i = 0; i < H1; ++i) acc = __builtin_fmaf(W1[j * H1 + i], a[i], acc);
    const float c = kTanh ? tanhf(acc) : dp_leaky(acc);
#pragma unroll
    for (int k = 0; k < OUT; ++k) o[k] = __builtin_fmaf(W2[k * H2 + j], c, o[k]);
  }
#pragma unroll
  for (int k = 0; k < OUT; ++k) out[k] = o[k];
}

// Gumbel(0,1) noise from a counter-based stream (splitmix64 of seed, env, counter, item).
__device__ __forceinline__ float dp_gumbel(uint64_t key, uint64_t item) {
  const uint64_t r = splitmix64(key ^ splitmix64(item + 0x632BE59BD9B4E019ULL));
  const double u = ((double)(r >> 11) + 0.5) * (1.0 / 9007199254740992.0);  // (0, 1)
  return (float)(-log(-log(u)));
}

struct DecimaPolicyOut {
  int32_t* stage_idx;  // [B] index among the env's schedulable stages (-1: none / skipped)
  int32_t* num_exec;   // [B] 1 + exec action (DecimaActWrapper.action)
  int32_t* job_idx;    // [B] active-job (DAG) index of the chosen stage
  int32_t* exec_idx;   // [B] exec action k
  float* lgprob;       // [B]
  float* stage_scores; // optional [B][stage_cap] (schedulable rows; others unspecified)
  float* exec_scores;  // optional [B][N] (k < cap)
};

// The chosen action in registers (wave-uniform), besides the DecimaPolicyOut arrays.
struct DpAction {
  int32_t stage_idx, num_exec, job_idx, exec_idx;
  float lgprob;
};

// Accumulation into the plan's agg / h_dag / glob rows. LDS plan: ds_add_f32. Global plan (kGlobal): the hardware
// f32 atomic in L2 (the plan is coarse-grained device memory), not the compare-and-swap loop atomicAdd would emit.
template <bool kGlobal>
__device__ __forceinline__ void dp_acc(float* p, float v) {
  if constexpr (kGlobal)
    WaveHip::fadd(p, v);  // global_atomic_add_f32, workgroup scope (the plan is the wave's own)
  else
    atomicAdd(p, v);
}
// A read of an accumulated (atomically updated) plan word: past the L1 on the global plan (wave_hip.h lds_load).
template <bool kGlobal>
__device__ __forceinline__ float dp_ld(const float* p) {
  if constexpr (kGlobal)
    return WaveHip::ld_rel(p);
  else
    return *p;
}

// Returns false if the env has more nodes than the plan holds (the caller reports it). `lds`: the plan, in LDS
// (k_decima_policy) or, with kGlobal, a per-env region of global memory (the persistent Decima rollout, whose
// 16 waves per CU leave no LDS for a J=200 plan); the atomic accumulation phases then end with an agent-scope
// fence (decima.h scratch_sync). `act` (optional) receives the action.
template <bool kGlobal = false>
__device__ __forceinline__ bool decima_policy_env(const Params* __restrict__ P, const uint8_t* __restrict__ obs,
                                         const float* __restrict__ feats, const int32_t* __restrict__ ccap,
                                         const uint32_t* __restrict__ emask, const int32_t* __restrict__ depth,
                                         const float* __restrict__ Wt, int node_cap, uint64_t seed,
                                         uint64_t counter, int eid, uint8_t* lds, const DecimaPolicyOut& o,
                                         DpAction* act = nullptr) {
  using W = WaveHip;
  const ssim_layout& L = P->L;
  const int S = L.stage_cap, J = L.job_cap, E = L.edge_cap, N = L.num_executors;
  const int32_t* cnt = reinterpret_cast<const int32_t*>(obs + L.ob_counts) + (int64_t)eid * SSIM_NUM_COUNTS;
  const int n = W::uni(cnt[SSIM_OC_NUM_NODES]), ne = W::uni(cnt[SSIM_OC_NUM_EDGES]);
  const int nj = W::uni(cnt[SSIM_OC_NUM_JOBS]);
  const int lane = W::lane();
  auto out_none = [&]() {
    if (act != nullptr) *act = DpAction{-1, 1, -1, 0, 0.0f};
    if (lane == 0 && o.stage_idx != nullptr) {
      o.stage_idx[eid] = -1;
      o.num_exec[eid] = 1;
      o.job_idx[eid] = -1;
      o.exec_idx[eid] = 0;
      o.lgprob[eid] = 0.0f;
    }
  };
  if (n <= 0 || nj <= 0) {
    out_none();
    return true;
  }
  if (n > node_cap) {
    out_none();
    return false;
  }
  const float* x = feats + (int64_t)eid * S * kDecimaFeatures;
  const float* nodes = reinterpret_cast<const float*>(obs + L.ob_nodes) + (int64_t)eid * S * 3;
  const int64_t* links = reinterpret_cast<const int64_t*>(obs + L.ob_edge_links) + (int64_t)eid * E * 2;
  const int32_t* ptr = reinterpret_cast<const int32_t*>(obs + L.ob_dag_ptr) + (int64_t)eid * (J + 1);
  const int32_t* cc = ccap + (int64_t)eid * J;
  const uint32_t* em = emask + (int64_t)eid * E;
  const int levels = W::uni(depth[eid]) > 1 ? W::uni(depth[eid]) - 1 : 0;

  const DpLds lo = dp_lds(node_cap, J);
  float* hi = reinterpret_cast<float*>(lds + lo.hi);
  float* hh = reinterpret_cast<float*>(lds + lo.hh);
  float* agg = reinterpret_cast<float*>(lds + lo.agg);
  float* score = reinterpret_cast<float*>(lds + lo.score);
  int16_t* ndag = reinterpret_cast<int16_t*>(lds + lo.ndag);
  uint8_t* flag = lds + lo.flag;
  float* hdag = reinterpret_cast<float*>(lds + lo.hdag);
  float* glob = reinterpret_cast<float*>(lds + lo.glob);

  // node -> DAG, flags
  for (int k = lane; k < nj; k += 64)
    for (int i = ptr[k]; i < ptr[k + 1]; ++i) ndag[i] = (int16_t)k;
  for (int i = lane; i < n; i += 64) flag[i] = 0;
  for (int k = lane; k < nj * kDpEmb; k += 64) hdag[k] = 0.0f;
  if (lane < kDpEmb) glob[lane] = 0.0f;
  scratch_sync<W, kGlobal>();
  for (int e = lane; e < ne; e += 64) flag[(int)links[2 * e]] = 1;  // parent has a child
  scratch_sync<W, kGlobal>();
  // h_init = mlp_prep(x); h = h_init (no levels) or mlp_update(h_init) for leaves
  for (int i = lane; i < n; i += 64) {
    float xi[kDecimaFeatures], v[kDpEmb], u[kDpEmb];
#pragma unroll
    for (int f = 0; f < kDecimaFeatures; ++f) xi[f] = x[i * kDecimaFeatures + f];
    dp_mlp<kDecimaFeatures, 32, 16, kDpEmb, false>(Wt + kOffPrep, xi, v);
#pragma unroll
    for (int f = 0; f < kDpEmb; ++f) hi[i * kDpEmb + f] = v[f];
    if (levels > 0) {
      if (!(flag[i] & 1)) {
        dp_mlp<kDpEmb, 32, 16, kDpEmb, false>(Wt + kOffUpd, v, u);
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) hh[i * kDpEmb + f] = u[f];
      } else {
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) hh[i * kDpEmb + f] = 0.0f;
      }
    } else {
#pragma unroll
      for (int f = 0; f < kDpEmb; ++f) hh[i * kDpEmb + f] = v[f];
    }
  }
  scratch_sync<W, kGlobal>();
  // message passing, deepest level first (reverse flow: children -> parents)
  for (int lvl = levels - 1; lvl >= 0; --lvl) {
    for (int e = lane; e < ne; e += 64) {  // zero agg and mark dst for the level's parents
      if ((em[e] >> lvl) & 1u) {
        const int p = (int)links[2 * e];
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) agg[p * kDpEmb + f] = 0.0f;
        flag[p] |= 2;
      }
    }
    scratch_sync<W, kGlobal>();
    for (int e = lane; e < ne; e += 64) {  // agg[p] += mlp_msg(h[c]) with the level's old h
      if ((em[e] >> lvl) & 1u) {
        const int p = (int)links[2 * e], c = (int)links[2 * e + 1];
        float hc[kDpEmb], m[kDpEmb];
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) hc[f] = hh[c * kDpEmb + f];
        dp_mlp<kDpEmb, 32, 16, kDpEmb, false>(Wt + kOffMsg, hc, m);
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) dp_acc<kGlobal>(agg + p * kDpEmb + f, m[f]);
      }
    }
    scratch_sync<W, kGlobal>();
    for (int i = lane; i < n; i += 64) {  // h[p] = h_init[p] + mlp_update(agg[p])
      if (flag[i] & 2) {
        float a[kDpEmb], u[kDpEmb];
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) a[f] = dp_ld<kGlobal>(agg + i * kDpEmb + f);
        dp_mlp<kDpEmb, 32, 16, kDpEmb, false>(Wt + kOffUpd, a, u);
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) hh[i * kDpEmb + f] = hi[i * kDpEmb + f] + u[f];
        flag[i] &= 1;
      }
    }
    scratch_sync<W, kGlobal>();
  }
  // DAG and global summaries
  for (int i = lane; i < n; i += 64) {
    float in[kDecimaFeatures + kDpEmb], v[kDpEmb];
#pragma unroll
    for (int f = 0; f < kDecimaFeatures; ++f) in[f] = x[i * kDecimaFeatures + f];
#pragma unroll
    for (int f = 0; f < kDpEmb; ++f) in[kDecimaFeatures + f] = hh[i * kDpEmb + f];
    dp_mlp<kDecimaFeatures + kDpEmb, 32, 16, kDpEmb, false>(Wt + kOffDag, in, v);
    const int g = ndag[i];
#pragma unroll
    for (int f = 0; f < kDpEmb; ++f) dp_acc<kGlobal>(hdag + g * kDpEmb + f, v[f]);
  }
  scratch_sync<W, kGlobal>();
  for (int g = lane; g < nj; g += 64) {
    float in[kDpEmb], v[kDpEmb];
#pragma unroll
    for (int f = 0; f < kDpEmb; ++f) in[f] = dp_ld<kGlobal>(hdag + g * kDpEmb + f);
    dp_mlp<kDpEmb, 32, 16, kDpEmb, false>(Wt + kOffGlob, in, v);
#pragma unroll
    for (int f = 0; f < kDpEmb; ++f) dp_acc<kGlobal>(glob + f, v[f]);
  }
  scratch_sync<W, kGlobal>();
  float gl[kDpEmb];
#pragma unroll
  for (int f = 0; f < kDpEmb; ++f) gl[f] = dp_ld<kGlobal>(glob + f);
  // stage scores over schedulable nodes, then a categorical draw (max-shifted softmax, Gumbel-max)
  const uint64_t key = splitmix64(seed ^ splitmix64((uint64_t)eid * 0x9E3779B97F4A7C15ULL + counter));
  float mx = -__builtin_inff(), best = -__builtin_inff();
  int pick = -1;
  for (int i = lane; i < n; i += 64) {
    if (nodes[3 * i + 2] != 0.0f) {
      float in[kDecimaFeatures + 3 * kDpEmb], s;
      const int g = ndag[i];
#pragma unroll
      for (int f = 0; f < kDecimaFeatures; ++f) in[f] = x[i * kDecimaFeatures + f];
#pragma unroll
      for (int f = 0; f < kDpEmb; ++f) {
        in[kDecimaFeatures + f] = hh[i * kDpEmb + f];
        in[kDecimaFeatures + kDpEmb + f] = dp_ld<kGlobal>(hdag + g * kDpEmb + f);
        in[kDecimaFeatures + 2 * kDpEmb + f] = gl[f];
      }
      dp_mlp<kDecimaFeatures + 3 * kDpEmb, 64, 64, 1, true>(Wt + kOffStage, in, &s);
      score[i] = s;
      if (o.stage_scores) o.stage_scores[(int64_t)eid * S + i] = s;
      mx = s > mx ? s : mx;
      const float gs = s + dp_gumbel(key, (uint64_t)i);
      if (gs > best) {
        best = gs;
        pick = i;
      }
    }
  }
  mx = W::max_f(mx);
  // winning lane of the Gumbel race (ties: lowest node)
  const float bmax = W::max_f(best);
  const uint64_t win = W::ballot(pick >= 0 && best == bmax);
  if (win == 0) {
    out_none();
    return true;
  }
  int node = 0x7FFFFFFF;
  for (uint64_t m = win; m; m &= m - 1) {
    const int cand = W::bcast_i(pick, W::ffs(m));
    node = cand < node ? cand : node;
  }
  scratch_sync<W, kGlobal>();
  float z = 0.0f;
  int rank = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {  // wave-uniform trip count: ballots need every lane
    const int i = i0 + lane;
    const bool sch = i < n && nodes[3 * i + 2] != 0.0f;
    if (sch) z += expf(score[i] - mx);
    rank += W::popc(W::ballot(sch && i < node));
  }
  z = W::sum_f(z);
  const float lp_stage = score[node] - mx - logf(z);
  // exec scores for k < commit cap of the chosen DAG
  const int g = ndag[node];
  const int cap = min(max(W::uni(cc[g]), 0), N);
  float in[3 + 2 * kDpEmb + 1];
  const int p0 = ptr[g];
#pragma unroll
  for (int f = 0; f < 3; ++f) in[f] = x[p0 * kDecimaFeatures + f];
#pragma unroll
  for (int f = 0; f < kDpEmb; ++f) {
    in[3 + f] = dp_ld<kGlobal>(hdag + g * kDpEmb + f);
    in[3 + kDpEmb + f] = gl[f];
  }
  float emx = -__builtin_inff(), ebest = -__builtin_inff(), es_k = 0.0f;
  int epick = -1;
  float* escore = agg;  // [N] (agg is free after message passing)
  for (int k = lane; k < cap; k += 64) {  // exec action k/N per lane
    float s;
    in[3 + 2 * kDpEmb] = (float)k / (float)N;
    dp_mlp<3 + 2 * kDpEmb + 1, 64, 64, 1, true>(Wt + kOffExec, in, &s);
    escore[k] = s;
    if (o.exec_scores) o.exec_scores[(int64_t)eid * N + k] = s;
    emx = s > emx ? s : emx;
    const float gs = s + dp_gumbel(key ^ 0xE7037ED1A0B428DBULL, (uint64_t)k);
    if (gs > ebest) {
      ebest = gs;
      epick = k;
      es_k = s;
    }
  }
  emx = W::max_f(emx);
  scratch_sync<W, kGlobal>();
  float ez = 0.0f;
  for (int k = lane; k < cap; k += 64) ez += expf(escore[k] - emx);
  ez = W::sum_f(ez);
  const float eb = W::max_f(ebest);
  const uint64_t ew = W::ballot(epick >= 0 && ebest == eb);
  int kx = 0;
  float sk = 0.0f;
  if (ew) {
    const int l = W::ffs(ew);
    kx = W::bcast_i(epick, l);
    sk = __builtin_bit_cast(float, W::bcast_i(__builtin_bit_cast(int, es_k), l));
  }
  const float lp_exec = ew ? sk - emx - logf(ez) : 0.0f;
  if (act != nullptr) *act = DpAction{rank, kx + 1, g, kx, lp_stage + lp_exec};
  if (lane == 0 && o.stage_idx != nullptr) {
    o.stage_idx[eid] = rank;
    o.num_exec[eid] = kx + 1;
    o.job_idx[eid] = g;
    o.exec_idx[eid] = kx;
    o.lgprob[eid] = lp_stage + lp_exec;
  }
  return true;
}

}  // namespace ssim
