// k_hbm.hip — step / rollout kernels: hot block in HBM, any shape.
#include "kernels.h"

KernelSet kernels_hbm() { return kernel_set<false, 0, 0, 0>(); }
