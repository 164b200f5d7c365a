// k_hbm_n100.hip — step / rollout kernels: hot block in HBM, specialised on 100 executors / 200 jobs (the configs[3]
// shard's shape; the stage cap is read at run time). Compile-time N and J fold the executor / job / commitment
// section offsets and loop bounds into immediates, which takes SGPR pressure (and spills) off the 4-wave kernel.
// 4-wave HBM-resident kernels (128 VGPRs): the lane index opaque at every use (wave_hip.h), so per-lane addresses are
// not hoisted to the kernel entry and spilled (configs[2] rollout 1012 -> 128 B/lane of scratch, configs[3] 248 -> 32).
#define SSIM_OPAQUE_LANE 1
#include "kernels.h"

KernelSet kernels_hbm_n100() { return kernel_set<false, 100, 200, 0, kTagHbmN100>("hbm_n100"); }

// the set KAT's known-bad variant (tests/test_gpu_sets.py): the same instantiation on the test-only wave type that
// reproduces the ROCm 7.2 page-assembly miscompile (engine.h KatBadPage); it must FAIL the KAT
SetTraceFn set_trace_kat_bad() { return k_set_trace<WaveHipKatBadPage, false, 100, 200, 0, kTagKatBad>; }
