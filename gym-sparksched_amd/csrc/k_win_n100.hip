// k_win_n100.hip — the configs[3] shard's shape (100 executors / 200 jobs) with WINDOWED rollouts: each env runs
// from an LDS copy of its live window (rings of kWinStages stages / kWinJobs jobs, engine.h), ~18 KB instead of the
// ~150 KB hot block, so 2 envs share a SIMD; envs whose window outgrows the rings continue HBM-resident in the same
// wave. Steps (k_step) stay HBM-resident.
#include "kernels.h"

KernelSet kernels_win_n100() { return kernel_set_windowed<100, 200, 0, kWinStages, kWinJobs, kTagWinN100>("win_n100"); }
