// k_hbm.hip — step / rollout kernels: hot block in HBM, any shape.
// register event slots for up to 128 executors (the configs[3] shard's 100): engine.h kEvPages
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#define SSIM_EV_PAGES_GENERIC 2
#include "kernels.h"

KernelSet kernels_hbm() { return kernel_set<false, 0, 0, 0, kTagHbm>("hbm"); }
