// k_lds.hip — step / rollout kernels: LDS-resident, any shape.
#include "kernels.h"

KernelSet kernels_lds() { return kernel_set<true, 0, 0, 0, kTagLds>("lds"); }
