// rollout.h — the decision loop of the fused rollouts (kernels.h rollout_body), independent of the wave policy W so
// the test-only host build (tests/hostsim) runs the same loop.
#pragma once
#include "engine.h"
#include "policy.h"

namespace ssim {

// A budget-free stop (the host build's rollouts; on device the shared budget is kernels.h TicketStop): never claims,
// never preempts.
struct NoBudget : NoStop {
  uint8_t* base = nullptr;
  bool on = false;
  __device__ __forceinline__ int64_t claim(int64_t, int64_t&) const { return 0; }
  __device__ __forceinline__ void give_back(int64_t) const {}
};

// The action driver of a fused rollout: `act` chooses the next action of the env (false: the env takes no more
// decisions in this launch, e.g. the Decima collector's episode ended or its sample arena is full), `done` runs after
// a decision this launch started has completed (its observation written), `rejected` when the env refused the action
// act() chose (the env is then frozen with SSIM_ERR_INVARIANT).
struct HeuristicPolicy {  // fair / FIFO / random (policy.h)
  int kind;
  uint64_t seed;
  // whether act() would choose an action (checked before a budget claim, so a claim is never spent on an env whose
  // policy then declines)
  template <class S>
  __device__ __forceinline__ bool can_act(const S&) const {
    return true;
  }
  template <class S>
  __device__ __forceinline__ bool act(S& s, int /*k*/, StepIn* a) const {
    *a = sim_policy(s, kind, seed);
    return true;
  }
  template <class S>
  __device__ __forceinline__ void done(S&) const {}
  template <class S>
  __device__ __forceinline__ void rejected(S&) const {}
};

// The state of one wave's rollout within a launch.
struct RolloutCursor {
  int k;             // decisions this launch started
  int64_t granted;   // budget decisions claimed and not yet started
  int64_t last;      // the budget counter at the wave's previous claim
};
// The decision loop of a fused rollout on engine `s` (any residency). `reset_env(s)` resets a finished episode in
// place.
template <class SimT, class Pol, class StopT, class ResetFn>
__device__ __forceinline__ void rollout_loop(SimT& s, const Pol& pol, const StopT& stop, RolloutCursor& c, int B,
                                            int eid, int num_steps, bool autoreset, int32_t* action_log,
                                            const ResetFn& reset_env) {
  using W = typename SimT::WT;
  // One loop both starts steps and completes a step a previous launch preempted (pending), so the simulation /
  // observation code (finish_step) is inlined once per engine.
  for (;;) {
#ifdef SSIM_PROFILE
    const uint64_t t0 = W::clock();
#endif
    s.load_header();
    // episode over (terminated, or truncated by the time limit): reset(seed=None) in place, before anything else
    // (one call site for the whole loop). A preemptible budget launch resets only when it holds a claimed
    // decision for the new episode: an episode that ends as the budget runs out is reset at the start of the
    // env's next launch, so no wave spends the end of a launch on a reset.
    if (autoreset && s.h.num_jobs > 0 && !s.frozen() && (s.h.terminated || s.h.wall >= s.h.time_limit) &&
        !s.pending()) {  // (a step preempted past the time limit completes first)
      if (stop.on && c.granted == 0 && (c.granted = stop.claim(B, c.last)) == 0) break;
#ifdef SSIM_PROFILE
      const uint64_t tr = W::clock();
#endif
      reset_env(s);
#ifdef SSIM_PROFILE
      s.prof_add(kPhReset, W::clock() - tr);
      s.prof_add(kCtReset, 1);
#endif
      continue;
    }
    double st0 = 0.0;
    bool simulate;
    if (s.pending()) {  // completes first, whatever this launch's mode; not one of its num_steps
      st0 = s.take_pending();
      simulate = true;
    } else {
      if (c.k >= num_steps) break;
      if (!pol.can_act(s)) break;
      if (stop.base != nullptr) {
        if (!autoreset && (s.h.terminated || s.frozen())) break;
        if (c.granted == 0 && (c.granted = stop.claim(B, c.last)) == 0) break;
        --c.granted;
      }
      StepIn a;
      if (!pol.act(s, c.k, &a)) break;  // (never after can_act: a claimed decision is always taken)
#ifdef SSIM_PROFILE
      s.prof_add(kPhPolicy, W::clock() - t0);
#endif
      if (action_log != nullptr && W::lane() == 0) {
        action_log[((int64_t)c.k * B + eid) * 2 + 0] = a.stage_idx;
        action_log[((int64_t)c.k * B + eid) * 2 + 1] = a.num_exec;
      }
      ++c.k;
      W::sync();
      simulate = s.step_begin(a, &st0);
      if (!simulate && s.rejected) {  // a device policy chose an invalid action: freeze the env (the host sees it)
        pol.rejected(s);  // (a recording policy drops what it recorded for the refused action)
        s.fail(SSIM_ERR_INVARIANT);
        s.store_header();
        s.write_err_only(0u);
        break;
      }
      if (!simulate) pol.done(s);
    }
    if (simulate) {
      if (!s.finish_step(st0, stop)) break;  // stopped mid-simulation: pending until the next launch
      pol.done(s);
    }
#ifdef SSIM_PROFILE
    {
      const uint64_t dc = W::clock() - t0;
      int b = 63 - __builtin_clzll(dc | 1ull) - 10;
      b = b < 0 ? 0 : b > 15 ? 15 : b;
      s.prof_add(kHist0 + b, 1);
      s.prof_add(kPhIter, dc);
    }
#endif
  }
}

}  // namespace ssim
