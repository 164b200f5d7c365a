// k_hbm_n50.hip — step / rollout kernels: hot block in HBM, specialised on 50 executors / 200 jobs (the
// config/decima_tpch.yaml env of configs[2] and configs[4]; the stage cap is read at run time).
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#include "kernels.h"

KernelSet kernels_hbm_n50() { return kernel_set<false, 50, 200, 0, kTagHbmN50>("hbm_n50"); }
