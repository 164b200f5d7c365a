// k_dr_hbm.hip — persistent Decima rollout (decima_rollout.h): hot block in HBM, any shape (configs[2]: 4096 envs,
// J = 200 / N = 50). Register event slots for up to 128 executors, as k_hbm.hip.
#define SSIM_EV_PAGES_GENERIC 2
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_hbm() { return {k_decima_rollout<false>, k_decima_rollout_warmup<false>, k_set_trace<WaveHip, false, 0, 0, 0, kTagDrHbm>,
          "dr_hbm"}; }
