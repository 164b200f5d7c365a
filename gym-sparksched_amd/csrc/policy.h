// policy.h — on-device action drivers that read the observation arena, one wavefront per env.
//
//   FAIR / FIFO : RoundRobinScheduler.schedule (schedulers/heuristics/round_robin.py:14-49) with
//                 find_stage / preprocess_obs (schedulers/heuristics/utils.py:5-37): prefer the source
//                 job with all committable executors, else the first job (arrival order) under the cap.
//   RANDOM      : uniform choice among jobs that have a schedulable stage (the distribution produced by
//                 random_scheduler.py:16-32's rejection loop), find_stage, num_exec ~ U{1..committable};
//                 the stream is a counter-based splitmix64 of (seed, env, counter), so a run is exactly
//                 reproducible; parity tests record these actions and replay them on the CPU oracle.
#pragma once
#include <stdint.h>

#include "engine.h"

namespace ssim {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// uniform integer in [0, n) from 32 random bits (n >= 1)
__device__ __forceinline__ int uniform_below(uint64_t bits, int n) {
  return (int)(((bits & 0xFFFFFFFFULL) * (uint64_t)n) >> 32);
}

// The decision rule of the device policies over a per-active-job view (nj active jobs, index k in arrival
// order): pick(k) = find_stage of job k (-1 = none), supply(k) = its exec supply; comm = committable
// executors, src = source_job_idx. Shared by the obs-arena view (k_policy) and the fused rollout, which
// passes the picks its observation pass computed (Sim::observe) so both give the same action.
template <class W, class Pick, class Supply>
__device__ __forceinline__ StepIn policy_act(int kind, uint64_t seed, uint64_t counter, int eid, int N, int nj,
                                             int comm, int src, Pick pick, Supply supply) {
  StepIn a;
  a.stage_idx = -1;
  a.num_exec = comm > 0 ? comm : 1;
  if (kind == SSIM_POLICY_FAIR || kind == SSIM_POLICY_FIFO) {
    const int cap = kind == SSIM_POLICY_FAIR ? (N + (nj > 1 ? nj : 1) - 1) / (nj > 1 ? nj : 1) : N;
    if (src < nj) {
      const int s = W::uni(pick(src));
      if (s >= 0) {
        a.stage_idx = s;
        return a;
      }
    }
    for (int k0 = 0; k0 < nj; k0 += W::kWidth) {
      const int k = k0 + W::lane();
      const bool ok = k < nj && k != src && supply(k) < cap;
      const int s = ok ? pick(k) : -1;
      const uint64_t m = W::ballot(s >= 0);
      if (m) {
        const int l = W::ffs(m);
        a.stage_idx = W::bcast_i(s, l);
        const int room = cap - W::bcast_i(ok ? supply(k) : 0, l);
        a.num_exec = comm < room ? comm : room;
        return a;
      }
    }
    return a;
  }
  // RANDOM
  const uint64_t key = splitmix64(seed ^ splitmix64((uint64_t)eid * 0xD1B54A32D192ED03ULL + counter));
  if (nj <= W::kWidth) {  // one chunk: each lane keeps its job's pick
    const int k = W::lane();
    const int s = k < nj ? pick(k) : -1;
    const uint64_t m = W::ballot(s >= 0);
    const int valid = W::popc(m);
    if (valid > 0) {
      const int r = uniform_below(splitmix64(key ^ 0x1ULL), valid);
      const int l = W::ffs(W::ballot(s >= 0 && W::rank(m) == r));
      a.stage_idx = W::bcast_i(s, l);
    }
  } else {
    int valid = 0;
    for (int k0 = 0; k0 < nj; k0 += W::kWidth) {
      const int k = k0 + W::lane();
      valid += W::popc(W::ballot(k < nj && pick(k) >= 0));
    }
    if (valid > 0) {
      int r = uniform_below(splitmix64(key ^ 0x1ULL), valid);
      for (int k0 = 0; k0 < nj; k0 += W::kWidth) {
        const int k = k0 + W::lane();
        const int s = k < nj ? pick(k) : -1;
        const uint64_t m = W::ballot(s >= 0);
        const int cnt = W::popc(m);
        if (r < cnt) {
          const int l = W::ffs(W::ballot(s >= 0 && W::rank(m) == r));
          a.stage_idx = W::bcast_i(s, l);
          break;
        }
        r -= cnt;
      }
    }
  }
  a.num_exec = comm > 0 ? 1 + uniform_below(splitmix64(key ^ 0x2ULL), comm) : 1;
  return a;
}

template <class W>
struct PolicyView {
  const ssim_layout& L;
  const uint8_t* obs;
  int eid;

  __device__ __forceinline__ const int32_t* counts() const {
    return reinterpret_cast<const int32_t*>(obs + L.ob_counts) + (int64_t)eid * SSIM_NUM_COUNTS;
  }
  __device__ __forceinline__ const int32_t* ptr() const {
    return reinterpret_cast<const int32_t*>(obs + L.ob_dag_ptr) + (int64_t)eid * (L.job_cap + 1);
  }
  __device__ __forceinline__ const int32_t* sup() const {
    return reinterpret_cast<const int32_t*>(obs + L.ob_supplies) + (int64_t)eid * L.job_cap;
  }
  __device__ __forceinline__ const int32_t* srank() const {
    return reinterpret_cast<const int32_t*>(obs + L.ob_sched_rank) + (int64_t)eid * L.stage_cap;
  }
  __device__ __forceinline__ const uint8_t* front() const { return obs + L.ob_frontier + (int64_t)eid * L.stage_cap; }

  // find_stage (utils.py:17-37) for active job index k; -1 if none
  __device__ __forceinline__ int find_stage(int k) const {
    const int32_t* p = ptr();
    const int32_t* r = srank();
    const uint8_t* f = front();
    int fallback = -1;
    for (int node = p[k]; node < p[k + 1]; ++node) {
      const int i = r[node];
      if (i < 0) continue;
      if (f[node]) return i;
      if (fallback < 0) fallback = i;
    }
    return fallback;
  }

  __device__ __forceinline__ StepIn act(int kind, uint64_t seed, uint64_t counter) const {
    const int32_t* c = counts();
    const int32_t* su = sup();
    return policy_act<W>(kind, seed, counter, eid, L.num_executors, c[SSIM_OC_NUM_JOBS], c[SSIM_OC_COMMITTABLE],
                         c[SSIM_OC_SOURCE_JOB_IDX], [&](int k) { return find_stage(k); },
                         [&](int k) { return su[k]; });
  }
};

// The fused rollout's policy input: the header (loaded) and the picks of the env's last observation
// (Sim::observe), read from the hot block instead of the obs arena the same wave just wrote.
template <class SimT>
__device__ __forceinline__ StepIn sim_policy(SimT& s, int kind, uint64_t seed) {
  using W = typename SimT::WT;
  const int16_t* aj = s.template H<int16_t>(s.O.active_jobs);
  const uint64_t counter = (uint64_t)s.h.decisions + ((uint64_t)s.h.episode << 32);
  return policy_act<W>(
      kind, seed, counter, s.eid, s.NE, s.h.n_active_jobs, s.committable(), s.h.src_idx,
      [&](int k) {
        const int key = s.job(aj[k]).pick;
        return key == 0x7FFFFFFF ? -1 : (key & 0xFFFF);
      },
      [&](int k) { return (int)s.job(aj[k]).supply; });
}

}  // namespace ssim
