// k_dr_hbm.hip — persistent Decima rollout (decima_rollout.h): hot block in HBM, any shape (configs[2]: 4096 envs,
// J = 200 / N = 50). Register event slots for up to 128 executors, as k_hbm.hip.
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#define SSIM_EV_PAGES_GENERIC 2
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_hbm() { return {k_decima_rollout<false>, k_decima_rollout_warmup<false>, k_set_trace<WaveHip, false, 0, 0, 0, kTagDrHbm>,
          "dr_hbm"}; }
