// k_bench900.hip — step / rollout kernels: LDS-resident, 10 executors / 50 jobs / stage cap 900 (the synthetic TPC-H set).
#include "kernels.h"

KernelSet kernels_bench900() { return kernel_set<true, 10, 50, 900, kTagBench900>("bench900"); }
