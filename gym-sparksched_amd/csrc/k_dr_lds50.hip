// k_dr_lds50.hip — persistent Decima rollout (decima_rollout.h): hot block LDS-resident, specialised on the
// config/decima_tpch.yaml env (50 executors / 200 jobs): the 16 envs of a PPO iteration (configs[4]), one env per CU,
// whose other SIMDs run the env's exec-score tiles (kDpHelpWaves waves per workgroup, decima_policy.h dp_exec_tiles).
#define SSIM_DP_PIPELINE 1  // (one wave per SIMD: decima_policy.h dp_layer_in_p)
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_lds50() {
  return {k_decima_rollout<true, 50, 200, true>, k_decima_rollout_warmup<true, 50, 200, true>,
          k_set_trace<WaveHip, true, 50, 200, 0, kTagDrLds50>, "dr_lds50", kDpHelpWaves};
}
