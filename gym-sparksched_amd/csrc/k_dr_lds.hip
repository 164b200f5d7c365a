// k_dr_lds.hip — persistent Decima rollout (decima_rollout.h): hot block LDS-resident (small batches, e.g. the 16 envs
// of a decima_tpch.yaml PPO iteration, one env per CU with the opt-in 160 KB of LDS).
#define SSIM_DP_PIPELINE 1  // (one wave per SIMD: decima_policy.h dp_layer_in_p)
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_lds() { return {k_decima_rollout<true>, k_decima_rollout_warmup<true>, k_set_trace<WaveHip, true, 0, 0, 0, kTagDrLds>,
          "dr_lds"}; }
