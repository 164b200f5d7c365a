// k_hbm.hip — step / rollout kernels: hot block in HBM, any shape.
// register event slots for up to 128 executors (the configs[3] shard's 100): engine.h kEvPages
#define SSIM_EV_PAGES_GENERIC 2
#include "kernels.h"

KernelSet kernels_hbm() { return kernel_set<false, 0, 0, 0, kTagHbm>("hbm"); }
