// decima.h — Decima observation featurisation on device, one wavefront per env.
//
// Restates schedulers/decima/env_wrapper.py:69-143 (DecimaObsWrapper.observation / _build_node_features)
// and schedulers/decima/utils.py:238-267 (make_dag_layer_edge_masks) over the obs arena the step kernel
// wrote (spark_sched_sim.py:345-406 layout), so a GPU policy consumes it without a host round trip.
//
// Outputs per env (caller-owned, row-major):
//   node_feats f32 [stage_cap][5]  rows < num_nodes: commit_cap/N, +-1 source-job flag, supply/N,
//                                  remaining/num_tasks_scale, remaining*recent_duration/work_scale
//                                  (the reference's dtypes: f64 quotients rounded to f32 for columns 0 and 2,
//                                  f32 arithmetic for 3 and 4)
//   commit_cap i32 [job_cap]       exec_mask[j, :commit_cap[j]] = True (env_wrapper.py:74-82, 92-94)
//   edge_mask  u32 [edge_cap]      bit l set <=> edge e is in message-passing mask l (l < depth-1)
//   depth      i32                 number of topological generations of the active DAG batch
// The reference's bool [depth-1, num_edges] masks are the bit planes of edge_mask: with level(v) the
// topological generation of node v and M(v) = (1 << level(v)) | OR over parents p of (1 << level(p)),
// node v is in generation l or a successor of it iff bit l of M(v) is set (utils.py:256-262), so the
// edge (u, v) mask word is M(u) & M(v). Generations are longest-path depths, found by relaxation.
#pragma once
#include <stdint.h>

#include "engine.h"

namespace ssim {

constexpr int kDecimaFeatures = 5;   // env_wrapper.py:9
constexpr int kDecimaMaxDepth = 32;  // edge_mask bits; DAG depth <= max_stages (checked at the ABI)

// LDS scratch per env: level i32[S], parent-level bits u32[S], job of node i16[S] (S: the node capacity)
inline int64_t decima_scratch_bytes(int64_t stage_cap) { return align16(10 * stage_cap); }

// Cross-lane ordering of the scratch updates. LDS scratch (k_decima): the wave's own ds operations are in order, a
// wave barrier suffices. Global scratch (kGlobal, the persistent Decima rollout: per-env scratch in HBM, too big for
// the LDS share of 16 waves per CU): a workgroup-scope fence waits for the wave's stores and atomics; the atomics are
// performed in L2, so every read of an atomically updated word is a W::lds_load (sc0: past the CU's L1).
template <class W, bool kGlobal>
__device__ __forceinline__ void scratch_sync() {
  if constexpr (kGlobal)
    W::gsync();
  else
    W::sync();
}

template <class W>
struct DecimaView {
  const ssim_layout& L;
  const uint8_t* obs;
  int eid;

  // scratch: decima_scratch_bytes(scap) bytes laid out for scap nodes (>= the observation's; default the stage cap)
  template <bool kGlobal = false>
  __device__ __forceinline__ void run(float num_tasks_scale, float work_scale, uint8_t* scratch, float* feats,
                                      int32_t* ccap, uint32_t* emask, int32_t* depth_out, int scap = 0) const {
    const int S = L.stage_cap, J = L.job_cap, E = L.edge_cap, N = L.num_executors;
    const int SC = scap > 0 ? scap : S;
    const int32_t* cnt = reinterpret_cast<const int32_t*>(obs + L.ob_counts) + (int64_t)eid * SSIM_NUM_COUNTS;
    const int n = W::uni(cnt[SSIM_OC_NUM_NODES]), ne = W::uni(cnt[SSIM_OC_NUM_EDGES]);
    const int nj = W::uni(cnt[SSIM_OC_NUM_JOBS]), comm = W::uni(cnt[SSIM_OC_COMMITTABLE]);
    const int src = W::uni(cnt[SSIM_OC_SOURCE_JOB_IDX]);
    const float* nodes = reinterpret_cast<const float*>(obs + L.ob_nodes) + (int64_t)eid * S * 3;
    const int64_t* links = reinterpret_cast<const int64_t*>(obs + L.ob_edge_links) + (int64_t)eid * E * 2;
    const int32_t* ptr = reinterpret_cast<const int32_t*>(obs + L.ob_dag_ptr) + (int64_t)eid * (J + 1);
    const int32_t* sup = reinterpret_cast<const int32_t*>(obs + L.ob_supplies) + (int64_t)eid * J;
    int32_t* lev = reinterpret_cast<int32_t*>(scratch);
    uint32_t* plm = reinterpret_cast<uint32_t*>(scratch + 4 * (int64_t)SC);
    int16_t* job_of = reinterpret_cast<int16_t*>(scratch + 8 * (int64_t)SC);
    float* f = feats + (int64_t)eid * S * kDecimaFeatures;
    int32_t* cc = ccap + (int64_t)eid * J;
    uint32_t* em = emask + (int64_t)eid * E;

    // commit caps (env_wrapper.py:72-82) and node -> active-job row
    for (int k = W::lane(); k < nj; k += W::kWidth) {
      const int gap = N - sup[k] > 0 ? N - sup[k] : 0;
      cc[k] = k == src ? comm : (gap < comm ? gap : comm);
      for (int i = ptr[k]; i < ptr[k + 1]; ++i) job_of[i] = (int16_t)k;
    }
    for (int i = W::lane(); i < n; i += W::kWidth) {
      lev[i] = 0;
      plm[i] = 0u;
    }
    scratch_sync<W, kGlobal>();
    // node features (env_wrapper.py:110-143)
    for (int i = W::lane(); i < n; i += W::kWidth) {
      const int k = job_of[i];
      const int s = sup[k];
      const int gap = N - s > 0 ? N - s : 0;
      const int cap = k == src ? comm : (gap < comm ? gap : comm);
      const float rem = nodes[3 * i + 0], rec = nodes[3 * i + 1];
      float* r = f + (int64_t)i * kDecimaFeatures;
      r[0] = (float)((double)cap / (double)N);
      r[1] = k == src ? 1.0f : -1.0f;
      r[2] = (float)((double)s / (double)N);
      r[3] = W::fdiv(rem, num_tasks_scale);
      r[4] = W::fdiv(W::fmul(rem, rec), work_scale);
    }
    // topological generations = longest-path depth from the sources (nx.topological_generations)
    for (int pass = 0; pass <= n; ++pass) {
      bool changed = false;
      for (int e = W::lane(); e < ne; e += W::kWidth) {
        const int a = (int)links[2 * e], b = (int)links[2 * e + 1];
        const int want = W::lds_load(lev + a) + 1;
        if (W::lds_load(lev + b) < want) {
          W::amax(lev + b, want);
          changed = true;
        }
      }
      scratch_sync<W, kGlobal>();
      if (!W::ballot(changed)) break;
    }
    int dmax = -1;
    for (int i = W::lane(); i < n; i += W::kWidth) {
      const int l = W::lds_load(lev + i);
      dmax = l > dmax ? l : dmax;
    }
    const int depth = W::max_i(dmax) + 1;  // 0 generations for an empty batch
    for (int e = W::lane(); e < ne; e += W::kWidth) {
      const int a = (int)links[2 * e], b = (int)links[2 * e + 1];
      W::aor(plm + b, 1u << (W::lds_load(lev + a) & 31));
    }
    scratch_sync<W, kGlobal>();
    const int* plmi = reinterpret_cast<const int*>(plm);
    for (int e = W::lane(); e < ne; e += W::kWidth) {
      const int a = (int)links[2 * e], b = (int)links[2 * e + 1];
      const uint32_t ma = (1u << (W::lds_load(lev + a) & 31)) | (uint32_t)W::lds_load(plmi + a);
      const uint32_t mb = (1u << (W::lds_load(lev + b) & 31)) | (uint32_t)W::lds_load(plmi + b);
      em[e] = ma & mb;
    }
    if (W::lane() == 0) depth_out[eid] = depth > kDecimaMaxDepth ? -1 : depth;
    scratch_sync<W, kGlobal>();
  }
};

}  // namespace ssim
