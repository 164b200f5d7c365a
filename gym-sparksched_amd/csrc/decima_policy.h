// decima_policy.h — fused Decima GNN policy (inference + action sampling), one wavefront per env.
//
// The rollout-time forward of schedulers/decima/scheduler.py:70-101 (DecimaScheduler.schedule: encoder,
// stage policy, exec policy, utils.sample) for the reference architecture of config/decima_tpch.yaml:66-78
// (embed 16; GNN MLPs 5|16|21 -> 32 -> 16 -> 16 with LeakyReLU(0.2); policy MLPs 53|36 -> 64 -> 64 -> 1
// with Tanh), reading the obs arena and the ssim_decima_features outputs directly. The batched PyTorch
// module (spark_sched_sim/schedulers/decima.py) is the same math in ~150 small launches per decision; this
// kernel is one launch, with every node's activations in the plan (LDS, or a global region) and the MLPs on the
// matrix cores over tiles of 32 nodes / DAGs / exec actions (dp_mlp16, dp_mlp1).
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
constexpr int kDpLdsDags = 16;  // DAG rows of the persistent rollout's LDS plan (observations with more take the global)

// Plan per env: h_init, h, agg, msg [cap][16] f32, score f32 [cap], node->DAG i16 [cap], flags u8 [cap] (bit0
// has-child), level marks u8 [cap] (bit0 child of a level edge, bit1 parent of one), compacted node lists i16 [cap]
// (the level's children, the level's parents, the schedulable nodes), h_dag [J][16] f32, glob [16] f32.
struct DpLds {
  int64_t hi, hh, agg, msg, score, ndag, flag, mark, clist, plist, slist, hdag, glob, total;
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
  o.msg = b;
  b += cap * kDpEmb * 4;
  o.score = b;
  b += cap * 4;
  o.ndag = b;
  b = align16(b + cap * 2);
  o.flag = b;
  b = align16(b + cap);
  o.mark = b;
  b = align16(b + cap);
  o.clist = b;
  b = align16(b + cap * 2);
  o.plist = b;
  b = align16(b + cap * 2);
  o.slist = b;
  b = align16(b + cap * 2);
  o.hdag = b;  // one row per active job: a job with no active stage is complete, so #jobs <= #nodes <= cap
  b += (job_cap < cap ? job_cap : cap) * kDpEmb * 4;
  o.glob = b;
  b += kDpEmb * 4;
  o.total = align16(b);
  return o;
}
inline int64_t decima_policy_lds_bytes(int64_t node_cap, int64_t job_cap) { return dp_lds(node_cap, job_cap).total; }

__device__ __forceinline__ float dp_leaky(float v) { return v >= 0.0f ? v : 0.2f * v; }

// MLPs on the matrix cores, one tile of 16 rows (nodes, DAGs or exec actions) per call: every layer is a transposed
// product Y^T[units x 16 rows] = W[units x in] . X^T[in x 16 rows] + b on v_mfma_f32_16x16x4_f32 (f32 in, f32
// accumulate: a k-ordered fmaf chain per output, no reduced precision). Lane l works on row l & 15; lane quarter
// q = l >> 4 supplies input k = 4s + q of step s. The accumulator of a 16-unit tile holds, in register r of lane l,
// unit 4q + r of row l & 15, and a hidden layer takes the previous layer's accumulators as its B operand (step r of
// tile t' reads unit 16t' + 4q + r: the input order is permuted to match), so layers chain in registers. 16-row tiles
// fit the observations of the Decima workloads (~16 nodes per decision at J=200); a per-lane MLP (one row per lane,
// weights as scalar operands) left most lanes idle there and waited on a scalar load per weight row.
//
// The weights (A operands) come from a PACKED copy of the parameters in the order the matrix cores consume them
// (DpPacked below; k_decima_pack builds it from the module's parameters() at each launch): per output tile and group
// of four steps, each lane's four A values are one aligned 16-B word, and the 64 lanes' words are contiguous. A group
// of four MFMA steps per output tile is then ONE 16-B load per lane (ds_read_b128 from the LDS copy of the persistent
// rollout, a coalesced 1-KB global_load_dwordx4 otherwise) at a compile-time offset from one lane-offset register,
// instead of a 4-B gather per step through a 64-bit pointer per tile from 16 different weight rows.
typedef float dp_f32x4 __attribute__((ext_vector_type(4)));

// Packed layout of one MLP (units of 16 B): W0 [T1][G0][64 lanes] (lane l, word j of group g, tile t: W0[16t + (l &
// 15)][16g + 4j + (l >> 4)], zero past IN), b0, W1 [T2][T1][64] (word r of group t': W1[16t + (l & 15)][16t' + 4(l >>
// 4) + r]), b1, then W2 as W1 for 16 outputs, or natural for one output (the score MLPs' last layer runs on the VALU),
// and b2.
template <int IN, int H1, int H2, int OUT>
struct Mlp3P {
  static constexpr int G0 = (IN + 15) / 16, T1 = H1 / 16, T2 = H2 / 16;
  static constexpr int kW0 = 0;
  static constexpr int kB0 = kW0 + T1 * G0 * 64;
  static constexpr int kW1 = kB0 + H1 / 4;
  static constexpr int kB1 = kW1 + T2 * T1 * 64;
  static constexpr int kW2 = kB1 + H2 / 4;
  static constexpr int kB2 = kW2 + (OUT == 16 ? T2 * 64 : H2 / 4);
  static constexpr int kSize = kB2 + (OUT + 3) / 4;
  // Natural (nn.Linear, parameters() order) index of packed float f, -1 for a zero pad.
  __host__ __device__ static int src(int f) {
    const int oB0 = H1 * IN, oW1 = oB0 + H1, oB1 = oW1 + H2 * H1, oW2 = oB1 + H2, oB2 = oW2 + OUT * H2;
    if (f < 4 * kB0) {
      const int j = f & 3, l = (f >> 2) & 63, tg = f >> 8, t = tg / G0, g = tg % G0;
      const int k = 16 * g + 4 * j + (l >> 4);
      return k < IN ? (16 * t + (l & 15)) * IN + k : -1;
    }
    if (f < 4 * kW1) return oB0 + (f - 4 * kB0);
    if (f < 4 * kB1) {
      const int u = f - 4 * kW1, r = u & 3, l = (u >> 2) & 63, tt = u >> 8, t = tt / T1, tp = tt % T1;
      return oW1 + (16 * t + (l & 15)) * H1 + 16 * tp + 4 * (l >> 4) + r;
    }
    if (f < 4 * kW2) return oB1 + (f - 4 * kB1);
    if (f < 4 * kB2) {
      const int u = f - 4 * kW2;
      if (OUT != 16) return oW2 + u;
      const int r = u & 3, l = (u >> 2) & 63, tp = u >> 8;
      return oW2 + (l & 15) * H2 + 16 * tp + 4 * (l >> 4) + r;
    }
    const int u = f - 4 * kB2;
    return u < OUT ? oB2 + u : -1;
  }
};
using PPrep = Mlp3P<kDecimaFeatures, 32, 16, kDpEmb>;
using PMsg = Mlp3P<kDpEmb, 32, 16, kDpEmb>;
using PDag = Mlp3P<kDecimaFeatures + kDpEmb, 32, 16, kDpEmb>;
using PStage = Mlp3P<kDecimaFeatures + 3 * kDpEmb, 64, 64, 1>;
using PExec = Mlp3P<3 + 2 * kDpEmb + 1, 64, 64, 1>;
// packed MLP bases (16-B units), in parameters() order
constexpr int kPPrep = 0;
constexpr int kPMsg = kPPrep + PPrep::kSize;
constexpr int kPUpd = kPMsg + PMsg::kSize;
constexpr int kPDag = kPUpd + PMsg::kSize;
constexpr int kPGlob = kPDag + PDag::kSize;
constexpr int kPStage = kPGlob + PMsg::kSize;
constexpr int kPExec = kPStage + PStage::kSize;
constexpr int kDpPacked = kPExec + PExec::kSize;           // 16-B units
constexpr int64_t kDpPackedBytes = 16 * (int64_t)kDpPacked;  // ~92 KB
// Natural index of packed float f of the whole policy (k_decima_pack), -1 = zero
__host__ __device__ inline int dp_pack_src(int f) {
  if (f < 4 * kPMsg) return kOffPrep + PPrep::src(f - 4 * kPPrep);
  int r;
  if (f < 4 * kPUpd) return (r = PMsg::src(f - 4 * kPMsg)) < 0 ? -1 : kOffMsg + r;
  if (f < 4 * kPDag) return (r = PMsg::src(f - 4 * kPUpd)) < 0 ? -1 : kOffUpd + r;
  if (f < 4 * kPGlob) return (r = PDag::src(f - 4 * kPDag)) < 0 ? -1 : kOffDag + r;
  if (f < 4 * kPStage) return (r = PMsg::src(f - 4 * kPGlob)) < 0 ? -1 : kOffGlob + r;
  if (f < 4 * kPExec) return (r = PStage::src(f - 4 * kPStage)) < 0 ? -1 : kOffStage + r;
  return (r = PExec::src(f - 4 * kPExec)) < 0 ? -1 : kOffExec + r;
}

// Weight sources: the packed copy in global memory, or its LDS copy (the persistent rollout's workgroups stage it).
// grp(o): this lane's 16-B word of the group at o (16-B units); vec(o): the word at o (bias / last-layer vectors).
// `lane`: this lane's index, made opaque per MLP call (dp_opaque): the per-lane word offsets (lane + a compile-time
// offset, one per tile and group) and the lane-quarter conditions derived from it are then computed inside each call.
// From a plain __lane_id() the compiler hoisted all of them to the kernel entry, where hundreds of such values were
// live at once and went to scratch memory (the persistent rollout reloaded them from there in every MLP).
struct DpWGlobal {
  const dp_f32x4* p;
  int lane = (int)__lane_id();
  __device__ __forceinline__ dp_f32x4 grp(int o) const { return p[o + lane]; }
  __device__ __forceinline__ dp_f32x4 vec(int o) const { return p[o]; }
};
typedef __attribute__((address_space(3))) const dp_f32x4 dp_lds_f32x4;
struct DpWLds {
  dp_lds_f32x4* p;
  int lane = (int)__lane_id();
  __device__ __forceinline__ dp_f32x4 grp(int o) const { return p[o + lane]; }
  __device__ __forceinline__ dp_f32x4 vec(int o) const { return p[o]; }
};
// The weight pointer made opaque at each MLP call: every load derived from it is then loop-variant, so the compiler
// does not hoist those of every MLP of the policy out of the tile loops to the function entry (where they were all
// live at once: hundreds of VGPRs).
__device__ __forceinline__ int64_t dp_zero() {  // an opaque 0 (offsets keep a pointer's address space; casts do not)
  int64_t z = 0;
  asm volatile("" : "+s"(z));
  return z;
}
__device__ __forceinline__ int dp_lane_opq() {  // __lane_id() behind an empty asm (not hoisted out of the caller)
  int l = (int)__lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ DpWGlobal dp_opaque(DpWGlobal w) {
  w.p += dp_zero();
  w.lane = dp_lane_opq();
  return w;
}
__device__ __forceinline__ DpWLds dp_opaque(DpWLds w) {
  w.lane = dp_lane_opq();
  return w;
}
// A row-source pointer made opaque at each tile: the per-lane addresses of a tile's inputs (one per MFMA step) then
// depend on the tile and are not hoisted out of the tile loops, where they were all live at once (64-bit addresses and
// exec masks per step: the policy spilled to scratch memory even as a standalone kernel).
template <class T>
__device__ __forceinline__ T* dp_opq(T* p) {
  return p + dp_zero();
}

// tanh from the hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32): 1 - 2 / (1 + e^(2|x|)), sign restored; below
// |x| = 2^-12 tanh(x) = x to f32 precision (the subtraction would cancel there). Absolute error ~1e-7 against the
// correctly rounded tanh: the score MLPs' two Tanh layers then stay within the 1e-5 the policy tests allow against the
// PyTorch module, at ~8 instructions instead of the ~40 of the library tanhf (the dominant VALU cost of a score tile).
__device__ __forceinline__ float dp_tanh(float x) {
  const float a = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(a * 2.8853900817779268f);  // e^(2a) = 2^(2a log2 e)
  const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
  return __builtin_copysignf(a < 0.000244140625f ? a : t, x);
}
template <bool kTanh>
__device__ __forceinline__ float dp_act(float v) {
  return kTanh ? dp_tanh(v) : dp_leaky(v);
}

// first layer: inputs xin(k), k < IN, of this lane's row (natural k order); packed W0 at ow, b0 at ob. One group of
// four steps per iteration: a 16-B A word per output tile, then the steps (scheduling barrier between groups: a
// group's loads are issued together and not hoisted past the group before, which bounds the registers in flight).
template <int IN, int H, class WS, class XF>
__device__ __forceinline__ void dp_layer_in(const WS& w, int ow, int ob, XF xin, dp_f32x4 (&y)[H / 16]) {
  static_assert(H % 16 == 0, "layer widths: multiples of 16");
  constexpr int T = H / 16, STEPS = (IN + 3) / 4, G = (IN + 15) / 16;
  const int q = w.lane >> 4;
#pragma unroll
  for (int t = 0; t < T; ++t) y[t] = w.vec(ob + 4 * t + q);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    dp_f32x4 wa[T];
#pragma unroll
    for (int t = 0; t < T; ++t) wa[t] = w.grp(ow + (t * G + g) * 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int st = 4 * g + j;
      if (st < STEPS) {
        const bool kin = 4 * st + 3 < IN || 4 * st + q < IN;
        const float xv = kin ? xin(4 * st + q) : 0.0f;
#pragma unroll
        for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][j], xv, y[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// hidden / output layer from the previous layer's accumulators x (HP units, activated here); packed W at ow, b at ob
template <int HP, int H, bool kTanh, class WS>
__device__ __forceinline__ void dp_layer_h(const WS& w, int ow, int ob, const dp_f32x4 (&x)[HP / 16],
                                           dp_f32x4 (&y)[H / 16]) {
  static_assert(H % 16 == 0 && HP % 16 == 0, "layer widths: multiples of 16");
  constexpr int T = H / 16, TP = HP / 16;
  const int q = w.lane >> 4;
#pragma unroll
  for (int t = 0; t < T; ++t) y[t] = w.vec(ob + 4 * t + q);
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    dp_f32x4 wa[T];
#pragma unroll
    for (int t = 0; t < T; ++t) wa[t] = w.grp(ow + (t * TP + tp) * 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float xv = dp_act<kTanh>(x[tp][r]);
#pragma unroll
      for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][r], xv, y[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// SSIM_DP_PIPELINE (set by the one-wave-per-SIMD translation units, k_dr_lds*.hip): the same layers with every weight
// and input load issued one group ahead of the steps that use it, and each MLP's biases, first weight group of every
// layer and last-layer vector loaded at its start, so one MLP waits for one round of loads instead of one per group
// (~8 for a score MLP: at one wave per SIMD nothing else hides them). The same operands in the same order: the results
// are those of the plain layers bit for bit. (~100 more registers in flight: the 4-wave units, at 128, keep the plain
// form.)
#ifndef SSIM_DP_PIPELINE
#define SSIM_DP_PIPELINE 0
#endif
#if SSIM_DP_PIPELINE
// first layer with its group 0 weights in wa and its biases in y already
template <int IN, int H, class WS, class XF>
__device__ __forceinline__ void dp_layer_in_p(const WS& w, int ow, XF xin, dp_f32x4 (&wa)[H / 16],
                                              dp_f32x4 (&y)[H / 16]) {
  constexpr int T = H / 16, STEPS = (IN + 3) / 4, G = (IN + 15) / 16;
  const int q = w.lane >> 4;
  auto in = [&](int st) { return st < STEPS && (4 * st + 3 < IN || 4 * st + q < IN) ? xin(4 * st + q) : 0.0f; };
  float xa[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) xa[j] = in(j);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    dp_f32x4 wn[T];
    float xn[4];
    if (g + 1 < G) {
#pragma unroll
      for (int t = 0; t < T; ++t) wn[t] = w.grp(ow + (t * G + g + 1) * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) xn[j] = in(4 * (g + 1) + j);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (4 * g + j < STEPS) {
#pragma unroll
        for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][j], xa[j], y[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (g + 1 < G) {
#pragma unroll
      for (int t = 0; t < T; ++t) wa[t] = wn[t];
#pragma unroll
      for (int j = 0; j < 4; ++j) xa[j] = xn[j];
    }
  }
}
// hidden / output layer with its group 0 weights in wa and its biases in y already
template <int HP, int H, bool kTanh, class WS>
__device__ __forceinline__ void dp_layer_h_p(const WS& w, int ow, const dp_f32x4 (&x)[HP / 16],
                                             dp_f32x4 (&wa)[H / 16], dp_f32x4 (&y)[H / 16]) {
  constexpr int T = H / 16, TP = HP / 16;
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    dp_f32x4 wn[T];
    if (tp + 1 < TP) {
#pragma unroll
      for (int t = 0; t < T; ++t) wn[t] = w.grp(ow + (t * TP + tp + 1) * 64);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float xv = dp_act<kTanh>(x[tp][r]);
#pragma unroll
      for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][r], xv, y[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (tp + 1 < TP) {
#pragma unroll
      for (int t = 0; t < T; ++t) wa[t] = wn[t];
    }
  }
}
#endif
// 3-layer MLP with 16 outputs (the GNN MLPs, LeakyReLU(0.2) between layers) at packed base `pb`: y register r of lane
// l = output 4 (l >> 4) + r of row l & 15
template <int IN, int H1, int H2, class WS, class XF>
__device__ __forceinline__ void dp_mlp16(const WS& w0, int pb, XF xin, dp_f32x4 (&y)[1]) {
  using PL = Mlp3P<IN, H1, H2, kDpEmb>;
  const WS w = dp_opaque(w0);
  dp_f32x4 a1[H1 / 16], a2[H2 / 16];
#if SSIM_DP_PIPELINE
  constexpr int T1 = H1 / 16, T2 = H2 / 16;
  const int q = w.lane >> 4;
  dp_f32x4 w0g[T1], w1g[T2], w2g[1];
#pragma unroll
  for (int t = 0; t < T1; ++t) {
    a1[t] = w.vec(pb + PL::kB0 + 4 * t + q);
    w0g[t] = w.grp(pb + PL::kW0 + t * PL::G0 * 64);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    a2[t] = w.vec(pb + PL::kB1 + 4 * t + q);
    w1g[t] = w.grp(pb + PL::kW1 + t * T1 * 64);
  }
  y[0] = w.vec(pb + PL::kB2 + q);
  w2g[0] = w.grp(pb + PL::kW2);
  dp_layer_in_p<IN, H1>(w, pb + PL::kW0, xin, w0g, a1);
  dp_layer_h_p<H1, H2, false>(w, pb + PL::kW1, a1, w1g, a2);
  dp_layer_h_p<H2, kDpEmb, false>(w, pb + PL::kW2, a2, w2g, y);
#else
  dp_layer_in<IN, H1>(w, pb + PL::kW0, pb + PL::kB0, xin, a1);
  dp_layer_h<H1, H2, false>(w, pb + PL::kW1, pb + PL::kB1, a1, a2);
  dp_layer_h<H2, kDpEmb, false>(w, pb + PL::kW2, pb + PL::kB2, a2, y);
#endif
}
// 3-layer MLP with one output (the policy score MLPs, Tanh between layers): the score of row l & 15, in every quarter
template <int IN, int H1, int H2, class WS, class XF>
__device__ __forceinline__ float dp_mlp1(const WS& w0, int pb, XF xin) {
  using PL = Mlp3P<IN, H1, H2, 1>;
  const WS w = dp_opaque(w0);
  dp_f32x4 a1[H1 / 16], a2[H2 / 16];
  const int q = w.lane >> 4;
#if SSIM_DP_PIPELINE
  constexpr int T1 = H1 / 16, T2 = H2 / 16;
  dp_f32x4 w0g[T1], w1g[T2], w2v[T2];
#pragma unroll
  for (int t = 0; t < T1; ++t) {
    a1[t] = w.vec(pb + PL::kB0 + 4 * t + q);
    w0g[t] = w.grp(pb + PL::kW0 + t * PL::G0 * 64);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    a2[t] = w.vec(pb + PL::kB1 + 4 * t + q);
    w1g[t] = w.grp(pb + PL::kW1 + t * T1 * 64);
    w2v[t] = w.vec(pb + PL::kW2 + 4 * t + q);
  }
  float part = q == 0 ? w.vec(pb + PL::kB2)[0] : 0.0f;
  dp_layer_in_p<IN, H1>(w, pb + PL::kW0, xin, w0g, a1);
  dp_layer_h_p<H1, H2, true>(w, pb + PL::kW1, a1, w1g, a2);
#pragma unroll
  for (int t = 0; t < T2; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) part = __builtin_fmaf(w2v[t][r], dp_tanh(a2[t][r]), part);
  }
#else
  dp_layer_in<IN, H1>(w, pb + PL::kW0, pb + PL::kB0, xin, a1);
  dp_layer_h<H1, H2, true>(w, pb + PL::kW1, pb + PL::kB1, a1, a2);
  float part = q == 0 ? w.vec(pb + PL::kB2)[0] : 0.0f;  // the last layer (H2 -> 1) on the VALU: this quarter's units,
#pragma unroll                                          // then all four
  for (int t = 0; t < H2 / 16; ++t) {
    const dp_f32x4 w2 = w.vec(pb + PL::kW2 + 4 * t + q);
#pragma unroll
    for (int r = 0; r < 4; ++r) part = __builtin_fmaf(w2[r], dp_tanh(a2[t][r]), part);
  }
#endif
  part += WaveHip::shfl_xor_f(part, 16);
  return part + WaveHip::shfl_xor_f(part, 32);
}

// Gumbel(0,1) noise from a counter-based stream (splitmix64 of seed, env, counter, item).
__device__ __forceinline__ float dp_gumbel(uint64_t key, uint64_t item) {
  const uint64_t r = splitmix64(key ^ splitmix64(item + 0x632BE59BD9B4E019ULL));
  const double u = ((double)(r >> 11) + 0.5) * (1.0 / 9007199254740992.0);  // (0, 1)
  return (float)(-log(-log(u)));
}

// Exec-score helpers (the one-env-per-CU persistent rollout, k_dr_lds50): the env's workgroup has kDpHelpWaves waves,
// wave 0 runs the env and the others score exec-action tiles. The exec MLP (36 -> 64 -> 64 -> 1) is a ~10k-cycle chain
// per 16-row tile on one SIMD. Two ways to take it off wave 0's chain, through the LDS mailbox below (the tiles' shared
// inputs out, the scores back; two workgroup barriers per decision order it: published -> A -> tiles -> B -> read):
// * speculative: when the schedulable nodes' DAGs (at most kDpSpecCand) need at most kDpHelpWaves - 1 tiles in all,
//   the helpers score every candidate DAG's actions while wave 0 scores the stages, and wave 0 then reads the chosen
//   DAG's (barrier A before the stage tiles, B after them);
// * otherwise, after the stage draw, the chosen DAG's tiles over all the waves (tile j on wave j % kDpHelpWaves).
// The same MLP, inputs and Gumbel noise as the one-wave loop of decima_policy_env, so the same values bit for bit.
// The helpers' loop waits at barrier A and leaves on kDpHelpExit, which wave 0 publishes once its rollout ends
// (decima_rollout.h).
constexpr int kDpHelpWaves = 4;
constexpr int kDpSpecCand = 3;
enum : int32_t { kDpHelpWork = 1, kDpHelpExit = 2 };
struct DpHelp {
  int32_t cmd, ncand, first;  // kDpHelpWork / kDpHelpExit; candidate DAGs; the first wave taking tiles (1: helpers only)
  int32_t cap[kDpSpecCand];   // exec actions to score (k < cap) per candidate
  int32_t dag[kDpSpecCand];   // the candidates' DAGs
  int32_t pad;
  uint64_t key;               // the decision's Gumbel key
  float base[kDpSpecCand][36];  // exec-MLP inputs 0..34 of every row of the candidate (input 35 is the row's k / N)
};
// mailbox bytes for N executors: the header, then sc [kDpSpecCand][N] and the Gumbel-perturbed scores gs [..][N]
__host__ __device__ inline int64_t dp_help_bytes(int64_t n_exec) {
  return align16((int64_t)sizeof(DpHelp) + 8 * kDpSpecCand * n_exec);
}
__device__ __forceinline__ float* dp_help_sc(DpHelp* hb, int N, int c) { return reinterpret_cast<float*>(hb + 1) + c * N; }
__device__ __forceinline__ float* dp_help_gs(DpHelp* hb, int N, int c) {
  return reinterpret_cast<float*>(hb + 1) + (kDpSpecCand + c) * N;
}

// The mailbox's tiles assigned to wave w: tile j (candidates in order, then rows) runs on wave first + j % (waves -
// first); action k of candidate c: its score into sc[c][k], its Gumbel-perturbed score into gs[c][k].
template <class WS>
__device__ __forceinline__ void dp_exec_tiles(const WS& Wt, DpHelp* hb, int N, int w) {
  using W = WaveHip;
  const int nc = W::uni(hb->ncand), first = W::uni(hb->first);
  const uint64_t key = W::uni(hb->key);
  const int lane = W::lane(), rl = lane & 15, hl = lane >> 4;
  int j = 0;
  for (int c = 0; c < nc; ++c) {
    const int cap = W::uni(hb->cap[c]);
    for (int t0 = 0; t0 < cap; t0 += 16, ++j) {
      if (first + j % (kDpHelpWaves - first) != w) continue;
      const int k = t0 + rl;
      const float* bq = dp_opq(hb->base[c]);
      const float sc = dp_mlp1<3 + 2 * kDpEmb + 1, 64, 64>(Wt, kPExec, [&](int f) {
        return f < 3 + 2 * kDpEmb ? bq[f] : (float)k / (float)N;
      });
      if (k < cap && hl == 0) {
        dp_help_sc(hb, N, c)[k] = sc;
        dp_help_gs(hb, N, c)[k] = sc + dp_gumbel(key ^ 0xE7037ED1A0B428DBULL, (uint64_t)k);
      }
    }
  }
}
// The helper waves' loop (waves 1 .. kDpHelpWaves - 1 of a helped workgroup)
template <class WS>
__device__ __forceinline__ void dp_help_loop(const WS& Wt, DpHelp* hb, int N, int w) {
  for (;;) {
    __syncthreads();  // A: a decision's inputs published, or the exit
    if (WaveHip::uni(hb->cmd) != kDpHelpWork) return;
    dp_exec_tiles(Wt, hb, N, w);
    __syncthreads();  // B: scores written
  }
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
// fence (decima.h scratch_sync). `act` (optional) receives the action. kHelp: the exec scores run on the workgroup's
// helper waves through the LDS mailbox `help` (dp_exec_tiles).
template <bool kGlobal = false, bool kHelp = false, class WS>
__device__ __forceinline__ bool decima_policy_env(const Params* __restrict__ P, const uint8_t* __restrict__ obs,
                                         const float* __restrict__ feats, const int32_t* __restrict__ ccap,
                                         const uint32_t* __restrict__ emask, const int32_t* __restrict__ depth,
                                         const WS& Wt, int node_cap, uint64_t seed,
                                         uint64_t counter, int eid, uint8_t* lds, const DecimaPolicyOut& o,
                                         DpAction* act = nullptr, uint64_t* prof = nullptr,
                                         int dag_cap = 0, DpHelp* help = nullptr) {
  using W = WaveHip;
  // diagnostic -DSSIM_PROFILE builds: shader cycles per part and the observation's sizes into prof[0..9] (LDS, lane 0)
#ifdef SSIM_PROFILE
  uint64_t tq = W::clock();
  auto lap = [&](int slot) {
    const uint64_t t = W::clock();
    if (prof != nullptr && W::lane() == 0) W::lds_add_u64(prof + slot, t - tq);
    tq = t;
  };
  auto count = [&](int slot, uint64_t v) {
    if (prof != nullptr && W::lane() == 0) W::lds_add_u64(prof + slot, v);
  };
#else
  (void)prof;
  auto lap = [](int) {};
  auto count = [](int, uint64_t) {};
#endif
  // -DSSIM_PROFILE_FINE (with SSIM_PROFILE): slots 5..8 time the score sections' parts instead of counting sizes
#ifdef SSIM_PROFILE_FINE
  auto lapf = [&](int slot) { lap(slot); };
  auto countf = [](int, uint64_t) {};
#else
  auto lapf = [](int) {};
  auto countf = [&](int slot, uint64_t v) { count(slot, v); };
#endif
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

  const DpLds lo = dp_lds(node_cap, dag_cap > 0 ? dag_cap : J);  // (dag_cap: the caller guarantees nj <= dag_cap)
  float* hi = reinterpret_cast<float*>(lds + lo.hi);
  float* hh = reinterpret_cast<float*>(lds + lo.hh);
  float* agg = reinterpret_cast<float*>(lds + lo.agg);
  float* msg = reinterpret_cast<float*>(lds + lo.msg);
  float* score = reinterpret_cast<float*>(lds + lo.score);
  int16_t* ndag = reinterpret_cast<int16_t*>(lds + lo.ndag);
  uint8_t* flag = lds + lo.flag;
  uint8_t* mark = lds + lo.mark;
  int16_t* clist = reinterpret_cast<int16_t*>(lds + lo.clist);
  int16_t* plist = reinterpret_cast<int16_t*>(lds + lo.plist);
  int16_t* slist = reinterpret_cast<int16_t*>(lds + lo.slist);
  float* hdag = reinterpret_cast<float*>(lds + lo.hdag);
  float* glob = reinterpret_cast<float*>(lds + lo.glob);

  // node -> DAG, flags
  for (int k = lane; k < nj; k += 64)
    for (int i = ptr[k]; i < ptr[k + 1]; ++i) ndag[i] = (int16_t)k;
  for (int i = lane; i < n; i += 64) {
    flag[i] = 0;
    mark[i] = 0;
  }
  for (int k = lane; k < nj * kDpEmb; k += 64) hdag[k] = 0.0f;
  if (lane < kDpEmb) glob[lane] = 0.0f;
  scratch_sync<W, kGlobal>();
  for (int e = lane; e < ne; e += 64) flag[(int)links[2 * e]] = 1;  // parent has a child
  scratch_sync<W, kGlobal>();
  lap(0);  // setup
  countf(5, (uint64_t)n);
  countf(6, (uint64_t)ne);
  countf(7, (uint64_t)levels);
  // h_init = mlp_prep(x); h = h_init (no levels) or mlp_update(h_init) for leaves. Tiles of 16 nodes (every lane runs
  // the matrix-core MLPs: the tile loops are wave-uniform); lane l stores outputs 4 (l >> 4) + r, r < 4, of node
  // t0 + (l & 15).
  const int hl = lane >> 4, rl = lane & 15;  // (matrix-core tiles: row, quarter)
  for (int t0 = 0; t0 < n; t0 += 16) {
    const int i = t0 + rl;
    const bool ok = i < n;
    dp_f32x4 v[1];
    const float* xq = dp_opq(x);
    dp_mlp16<kDecimaFeatures, 32, 16>(Wt, kPPrep, [&](int k) { return ok ? xq[i * kDecimaFeatures + k] : 0.0f; }, v);
    if (ok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) hi[i * kDpEmb + 4 * hl + r] = v[0][r];
    }
    if (levels > 0) {
      scratch_sync<W, kGlobal>();
      dp_f32x4 u[1];
      const float* hq = dp_opq(hi);
      dp_mlp16<kDpEmb, 32, 16>(Wt, kPUpd, [&](int k) { return ok ? hq[i * kDpEmb + k] : 0.0f; }, u);
      if (ok) {
        const bool leaf = !(flag[i] & 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) hh[i * kDpEmb + 4 * hl + r] = leaf ? u[0][r] : 0.0f;
      }
    } else if (ok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) hh[i * kDpEmb + 4 * hl + r] = v[0][r];
    }
  }
  scratch_sync<W, kGlobal>();
  lap(1);  // prep
  // message passing, deepest level first (reverse flow: children -> parents). Per level the MLPs run over compacted
  // node lists (the level's children, then its parents): a lane-parallel pass over all edges or nodes would evaluate
  // an MLP for every 64-row chunk holding ANY level row, i.e. nearly every chunk at every level. Each child's message
  // is computed once (mlp_msg of its old h, as the reference's msg = mlp_msg(h) before the gather) and summed into
  // every parent it reaches in the level.
  for (int lvl = levels - 1; lvl >= 0; --lvl) {
    for (int e = lane; e < ne; e += 64) {  // mark the level's children and parents, zero the parents' agg
      if ((em[e] >> lvl) & 1u) {
        const int p = (int)links[2 * e], c = (int)links[2 * e + 1];
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) agg[p * kDpEmb + f] = 0.0f;
        mark[c] |= 1;  // (a node is only ever marked by lanes setting the same bit in one store: child and parent
      }                //  marks go in separate passes below)
    }
    scratch_sync<W, kGlobal>();
    for (int e = lane; e < ne; e += 64)
      if ((em[e] >> lvl) & 1u) mark[(int)links[2 * e]] |= 2;
    scratch_sync<W, kGlobal>();
    int nc = 0, np = 0;  // compact (children, parents) in node order; clear the marks
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      const int m = i < n ? mark[i] : 0;
      const uint64_t bc = W::ballot(m & 1), bp = W::ballot(m & 2);
      if (m & 1) clist[nc + W::rank(bc)] = (int16_t)i;
      if (m & 2) plist[np + W::rank(bp)] = (int16_t)i;
      if (m) mark[i] = 0;
      nc += W::popc(bc);
      np += W::popc(bp);
    }
    scratch_sync<W, kGlobal>();
    for (int t0 = 0; t0 < nc; t0 += 16) {  // msg[c] = mlp_msg(h[c]) with the level's old h
      const bool ok = t0 + rl < nc;
      const int c = ok ? clist[t0 + rl] : 0;
      dp_f32x4 m[1];
      const float* hq = dp_opq(hh);
      dp_mlp16<kDpEmb, 32, 16>(Wt, kPMsg, [&](int k) { return ok ? hq[c * kDpEmb + k] : 0.0f; }, m);
      if (ok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) msg[c * kDpEmb + 4 * hl + r] = m[0][r];
      }
    }
    scratch_sync<W, kGlobal>();
    for (int e = lane; e < ne; e += 64) {  // agg[p] += msg[c] over the level's edges
      if ((em[e] >> lvl) & 1u) {
        const int p = (int)links[2 * e], c = (int)links[2 * e + 1];
#pragma unroll
        for (int f = 0; f < kDpEmb; ++f) dp_acc<kGlobal>(agg + p * kDpEmb + f, msg[c * kDpEmb + f]);
      }
    }
    scratch_sync<W, kGlobal>();
    for (int t0 = 0; t0 < np; t0 += 16) {  // h[p] = h_init[p] + mlp_update(agg[p])
      const bool ok = t0 + rl < np;
      const int i = ok ? plist[t0 + rl] : 0;
      dp_f32x4 u[1];
      const float* aq = dp_opq(agg);
      dp_mlp16<kDpEmb, 32, 16>(Wt, kPUpd, [&](int k) { return ok ? dp_ld<kGlobal>(aq + i * kDpEmb + k) : 0.0f; },
                               u);
      if (ok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * hl + r;
          hh[i * kDpEmb + f] = hi[i * kDpEmb + f] + u[0][r];
        }
      }
    }
    scratch_sync<W, kGlobal>();
  }
  lap(2);  // message passing
  // DAG and global summaries
  for (int t0 = 0; t0 < n; t0 += 16) {
    const int i = t0 + rl;
    const bool ok = i < n;
    dp_f32x4 v[1];
    const float* xq = dp_opq(x);
    const float* hq = dp_opq(hh);
    dp_mlp16<kDecimaFeatures + kDpEmb, 32, 16>(Wt, kPDag, [&](int k) {
      return !ok ? 0.0f : k < kDecimaFeatures ? xq[i * kDecimaFeatures + k] : hq[i * kDpEmb + k - kDecimaFeatures];
    }, v);
    if (ok) {
      const int g = ndag[i];
#pragma unroll
      for (int r = 0; r < 4; ++r) dp_acc<kGlobal>(hdag + g * kDpEmb + 4 * hl + r, v[0][r]);
    }
  }
  scratch_sync<W, kGlobal>();
  for (int t0 = 0; t0 < nj; t0 += 16) {
    const int g = t0 + rl;
    const bool ok = g < nj;
    dp_f32x4 v[1];
    const float* dq = dp_opq(hdag);
    dp_mlp16<kDpEmb, 32, 16>(Wt, kPGlob, [&](int k) { return ok ? dp_ld<kGlobal>(dq + g * kDpEmb + k) : 0.0f; },
                             v);
    if (ok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) dp_acc<kGlobal>(glob + 4 * hl + r, v[0][r]);
    }
  }
  scratch_sync<W, kGlobal>();
  // stage scores over schedulable nodes, then a categorical draw (max-shifted softmax, Gumbel-max)
  const uint64_t key = splitmix64(seed ^ splitmix64((uint64_t)eid * 0x9E3779B97F4A7C15ULL + counter));
  lap(3);  // DAG / global summaries
  int nsch = 0;  // the schedulable nodes, compacted in node order
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const bool sch = i < n && nodes[3 * i + 2] != 0.0f;
    const uint64_t b = W::ballot(sch);
    if (sch) slist[nsch + W::rank(b)] = (int16_t)i;
    nsch += W::popc(b);
  }
  scratch_sync<W, kGlobal>();
  // exec-MLP inputs of DAG gc into mailbox slot c (kHelp)
  auto publish = [&](int c, int gc, int capc, int pc) {
    if (lane < 3 + 2 * kDpEmb)
      help->base[c][lane] = lane < 3            ? x[pc * kDecimaFeatures + lane]
                            : lane < 3 + kDpEmb ? dp_ld<kGlobal>(hdag + gc * kDpEmb + lane - 3)
                                                : dp_ld<kGlobal>(glob + lane - 3 - kDpEmb);
    if (lane == 0) {
      help->cap[c] = capc;
      help->dag[c] = gc;
    }
  };
  bool spec = false;  // the candidates' exec scores on the helpers, during the stage tiles
  if constexpr (kHelp) {
    if (nsch <= 64) {
      const int gl = lane < nsch ? ndag[slist[lane]] : -1;
      const int cl = lane < nsch ? cc[gl] : 0, pl = lane < nsch ? ptr[gl] : 0;  // (one round trip for all)
      int cg[kDpSpecCand], cc_[kDpSpecCand], cp[kDpSpecCand], nc = 0, tiles = 0;
      for (int s = 0; s < nsch; ++s) {  // distinct DAGs in schedulable-node order
        const int gs = W::bcast_i(gl, s);
        bool seen = false;
#pragma unroll
        for (int c = 0; c < kDpSpecCand; ++c) seen |= c < nc && cg[c] == gs;
        if (seen) continue;
        if (nc == kDpSpecCand) {
          nc = kDpSpecCand + 1;
          break;
        }
        cg[nc] = gs;
        cc_[nc] = min(max(W::bcast_i(cl, s), 0), N);
        cp[nc] = W::bcast_i(pl, s);
        tiles += (cc_[nc] + 15) / 16;
        ++nc;
      }
      spec = nc <= kDpSpecCand && tiles > 0 && tiles < kDpHelpWaves;
      if (spec) {
#pragma unroll
        for (int c = 0; c < kDpSpecCand; ++c)
          if (c < nc) publish(c, cg[c], cc_[c], cp[c]);
        if (lane == 0) {
          help->ncand = nc;
          help->first = 1;
          help->key = key;
          help->cmd = kDpHelpWork;
        }
        __syncthreads();  // A
      }
    }
  }
  lapf(5);  // (fine: stage compaction)
  float mx = -__builtin_inff(), best = -__builtin_inff();
  int pick = -1;
  for (int t0 = 0; t0 < nsch; t0 += 16) {  // score = mlp_stage([x, h, h_dag, h_glob]) per schedulable node
    const bool ok = t0 + rl < nsch;
    const int i = ok ? slist[t0 + rl] : 0;
    const int g = ndag[i];
    const float* xq = dp_opq(x);
    const float* hq = dp_opq(hh);
    const float* dq = dp_opq(hdag);
    const float* gq = dp_opq(glob);
    const float sc = dp_mlp1<kDecimaFeatures + 3 * kDpEmb, 64, 64>(Wt, kPStage, [&](int k) {
      return !ok                                   ? 0.0f
             : k < kDecimaFeatures                 ? xq[i * kDecimaFeatures + k]
             : k < kDecimaFeatures + kDpEmb        ? hq[i * kDpEmb + k - kDecimaFeatures]
             : k < kDecimaFeatures + 2 * kDpEmb    ? dp_ld<kGlobal>(dq + g * kDpEmb + k - kDecimaFeatures - kDpEmb)
                                                   : dp_ld<kGlobal>(gq + k - kDecimaFeatures - 2 * kDpEmb);
    });
    if (ok && hl == 0) {  // (every quarter holds the score; quarter 0 owns the row)
      score[i] = sc;
      if (o.stage_scores) o.stage_scores[(int64_t)eid * S + i] = sc;
      mx = sc > mx ? sc : mx;
      const float gs = sc + dp_gumbel(key, (uint64_t)i);
      if (gs > best) {
        best = gs;
        pick = i;
      }
    }
  }
  if constexpr (kHelp) {
    if (spec) __syncthreads();  // B (before any return: the helpers meet it)
  }
  lapf(6);  // (fine: stage tiles)
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
  lap(4);  // stage scores + draw
  countf(8, (uint64_t)nsch);
  // exec scores for k < commit cap of the chosen DAG
  const int g = ndag[node];
  const int cap = min(max(W::uni(cc[g]), 0), N);
  const int p0 = ptr[g];
  lapf(7);  // (fine: exec prologue)
  float emx = -__builtin_inff(), ebest = -__builtin_inff(), es_k = 0.0f;
  int epick = -1;
  float* escore = agg;  // [N] (agg is free after message passing)
  if constexpr (kHelp) {  // the tiles over the workgroup's waves (dp_exec_tiles), then the same reduction
    int c = 0;
    if (spec) {  // already scored: the chosen DAG's slot
      const int nc = W::uni(help->ncand);
      for (int c2 = 1; c2 < nc; ++c2)
        if (W::uni(help->dag[c2]) == g) c = c2;
    }
    if (!spec) {
      publish(0, g, cap, p0);
      if (lane == 0) {
        help->ncand = 1;
        help->first = 0;
        help->key = key;
        help->cmd = kDpHelpWork;
      }
      const bool many = cap > 16;  // one tile: no helpers needed
      if (many) __syncthreads();  // A
      else W::sync();
      dp_exec_tiles(Wt, help, N, 0);
      if (many) __syncthreads();  // B
      else W::sync();
    }
    escore = dp_help_sc(help, N, c);
    const float* egs = dp_help_gs(help, N, c);
    for (int t0 = 0; t0 < cap; t0 += 16) {
      const int k = t0 + rl;
      if (k < cap && hl == 0) {
        const float sc = escore[k], gs = egs[k];
        if (o.exec_scores) o.exec_scores[(int64_t)eid * N + k] = sc;
        emx = sc > emx ? sc : emx;
        if (gs > ebest) {
          ebest = gs;
          epick = k;
          es_k = sc;
        }
      }
    }
  }
  for (int t0 = 0; !kHelp && t0 < cap; t0 += 16) {  // score of exec action k / N, k < cap, from [x_dag[:3], h_dag, h_glob, k/N]
    const int k = t0 + rl;
    const bool ok = k < cap;
    const float* xq = dp_opq(x);
    const float* dq = dp_opq(hdag);
    const float* gq = dp_opq(glob);
    const float sc = dp_mlp1<3 + 2 * kDpEmb + 1, 64, 64>(Wt, kPExec, [&](int f) {
      return f < 3             ? xq[p0 * kDecimaFeatures + f]
             : f < 3 + kDpEmb  ? dp_ld<kGlobal>(dq + g * kDpEmb + f - 3)
             : f < 3 + 2 * kDpEmb ? dp_ld<kGlobal>(gq + f - 3 - kDpEmb)
                                  : (float)k / (float)N;
    });
    if (ok && hl == 0) {
      escore[k] = sc;
      if (o.exec_scores) o.exec_scores[(int64_t)eid * N + k] = sc;
      emx = sc > emx ? sc : emx;
      const float gs = sc + dp_gumbel(key ^ 0xE7037ED1A0B428DBULL, (uint64_t)k);
      if (gs > ebest) {
        ebest = gs;
        epick = k;
        es_k = sc;
      }
    }
  }
  lapf(8);  // (fine: exec tiles)
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
  lap(9);  // exec scores + draw
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
