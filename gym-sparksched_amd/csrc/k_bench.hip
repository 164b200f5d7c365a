// k_bench.hip — step / rollout kernels: LDS-resident, 10 executors / 50 jobs, stage cap read at run time.
#include "kernels.h"

KernelSet kernels_bench() { return kernel_set<true, 10, 50, 0, kTagBench>("bench"); }
