#!/bin/bash
# Round-6 final measurement pass of the tree's build: GPU suite + smoke, the bench lines (with CPU baselines), rocprofv3
# kernel summaries and PMC passes (waves, fetch, write) per workload. Each step has its own time limit; a fault-like
# exit stops the script (gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${FINAL_STEPS:-all}
want() { [ "$S" = all ] || case " $S " in *" $1 "*) return 0;; esac; [ "$S" = all ]; }
if want tests; then bash scripts/gpu_check.sh smoke pytest || exit $?; fi
if want bench; then
  bash scripts/gpu_check.sh bench || exit $?
  bash scripts/gpu_check.sh bench_large bench_decima bench_ppo || exit $?
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_cpu.log 2>&1 || exit $?
fi
if want prof; then
  bash scripts/gpu_check.sh prof prof_driver || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_large" -o run --output-format csv -- python3 bench.py --workload large --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_large.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_decima" -o run --output-format csv -- python3 bench.py --workload decima --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/prof_decima.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_ppo" -o run --output-format csv -- python3 bench.py --workload ppo --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ppo.log 2>&1 || exit $?
fi
if want pmc; then
  PMC_PASSES="waves fetch write" bash scripts/gpu_check.sh pmc pmc300 pmc_large pmc_decima || exit $?
fi
echo "=== r6_final done"
