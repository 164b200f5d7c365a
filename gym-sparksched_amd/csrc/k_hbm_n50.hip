// k_hbm_n50.hip — step / rollout kernels: hot block in HBM, specialised on 50 executors / 200 jobs (the
// config/decima_tpch.yaml env of configs[2] and configs[4]; the stage cap is read at run time).
#include "kernels.h"

KernelSet kernels_hbm_n50() { return kernel_set<false, 50, 200, 0, kTagHbmN50>("hbm_n50"); }
