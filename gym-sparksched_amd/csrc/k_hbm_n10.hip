// k_hbm_n10.hip — step / rollout kernels: hot block in HBM, specialised on 10 executors / 50 jobs (BASELINE
// configs[1]'s env at batch sizes past what the LDS-resident kernel holds at once, layout.h kLdsRoundsMax; the stage
// cap is read at run time).
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#include "kernels.h"

KernelSet kernels_hbm_n10() { return kernel_set<false, 10, 50, 0, kTagHbmN10>("hbm_n10"); }
