// k_dr_win50.hip — persistent Decima rollout (decima_rollout.h) of the config/decima_tpch.yaml env (50 executors /
// 200 jobs; configs[2]'s 4096 envs) on the WINDOWED engine (kernels.h rollout_body): each env from an LDS copy of its
// live window, the HBM-resident engine for envs whose window outgrows the rings.
#include "decima_rollout.h"

DecimaRolloutSet decima_rollout_win50() {
  return {k_decima_rollout<true, 50, 200, kWinStages, kWinJobs>, k_decima_rollout_warmup<true, 50, 200, kWinStages,
                                                                                        kWinJobs>,
          k_set_trace<WaveHip, false, 50, 200, 0, kTagDrWin50>, "dr_win50", kWinJobs, kWinStages};
}
