// k_hbm_n100.hip — step / rollout kernels: hot block in HBM, specialised on 100 executors / 200 jobs (the configs[3]
// shard's shape; the stage cap is read at run time). Compile-time N and J fold the executor / job / commitment
// section offsets and loop bounds into immediates, which takes SGPR pressure (and spills) off the 4-wave kernel.
#include "kernels.h"

KernelSet kernels_hbm_n100() { return kernel_set<false, 100, 200, 0, kTagHbmN100>("hbm_n100"); }

// the set KAT's known-bad variant (tests/test_gpu_sets.py): the same instantiation on the test-only wave type that
// reproduces the ROCm 7.2 page-assembly miscompile (engine.h KatBadPage); it must FAIL the KAT
SetTraceFn set_trace_kat_bad() { return k_set_trace<WaveHipKatBadPage, false, 100, 200, 0, kTagKatBad>; }
