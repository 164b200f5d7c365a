// k_win_n50.hip — the config/decima_tpch.yaml env shape (50 executors / 200 jobs) with windowed rollouts
// (k_win_n100.hip); steps stay HBM-resident.
#include "kernels.h"

KernelSet kernels_win_n50() { return kernel_set_windowed<50, 200, 0, kWinStages, kWinJobs, kTagWinN50>("win_n50"); }
