// k_dr_hbm50.hip — persistent Decima rollout (decima_rollout.h): hot block in HBM, specialised on the
// config/decima_tpch.yaml env (50 executors / 200 jobs; configs[2]'s 4096 envs). One page of register event slots.
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_hbm50() {
  return {k_decima_rollout<false, 50, 200>, k_decima_rollout_warmup<false, 50, 200>,
          k_set_trace<WaveHip, false, 50, 200, 0, kTagDrHbm50>, "dr_hbm50"};
}
