// k_hbm_n10.hip — step / rollout kernels: hot block in HBM, specialised on 10 executors / 50 jobs (BASELINE
// configs[1]'s env at batch sizes past what the LDS-resident kernel holds at once, layout.h kLdsRoundsMax; the stage
// cap is read at run time).
#include "kernels.h"

KernelSet kernels_hbm_n10() { return kernel_set<false, 10, 50, 0, kTagHbmN10>("hbm_n10"); }
