#!/bin/bash
# GPU-box check runner: each step has its own time limit; a fault-like exit (timeout 124/137,
# abort 134, segfault 139, >128) stops the script before any further GPU work. Ordinary failures
# (exit 1, e.g. a failing test) are recorded and the next step runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
# heartbeat: a step that runs minutes without printing (a test fanning the oracle replay out over the CPUs) is not
# hung; each step still has its own time limit below
( while sleep 50; do date +%T >> "$OUT/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name: fault-like exit $rc"; exit $rc; fi
}
for s in "$@"; do
  case "$s" in
    smoke)   step smoke 300 python __graft_entry__.py ;;
    pytest)  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    pytestall) step pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread ;;
    pytestk) step pytest_k 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" ;;
    diag)    step diag_large 240 python -u scripts/diag_large.py 64,20,0 4096,10,0 4096,5,8000 ;;
    sets)    step pytest_sets 300 python -u -m pytest tests/test_gpu_sets.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
    bench_large_nocpu) step bench_large_nocpu 300 python bench.py --workload large --steps 100 --warmup 20 --no-cpu-baseline ;;
    bench_decima_nocpu) step bench_decima_nocpu 300 python bench.py --workload decima --steps 40 --warmup 5 --no-cpu-baseline ;;
    bench_driver) step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench)   step bench 400 python bench.py ;;
    bench_nocpu) step bench_nocpu 300 python bench.py --no-cpu-baseline ;;
    bench_step) step bench_step 300 python bench.py --no-cpu-baseline --mode step ;;
    bench_decima) step bench_decima 400 python bench.py --workload decima --steps 40 --warmup 5 ;;
    bench_ppo) step bench_ppo 900 python bench.py --workload ppo --steps 2 --warmup 1 ;;
    prof_decima) step prof_decima 600 python scripts/profile_decima.py ;;
    bench_large) step bench_large 400 python bench.py --workload large --steps 100 --warmup 20 ;;
    bench_cap850) step bench_cap850 300 python bench.py --no-cpu-baseline --dataset-seed 1 ;;
    learner) step learner 600 python scripts/profile_learner.py ;;
    prof)    step prof 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    phase)   step phase 600 python scripts/phase_profile.py ;;
    sweep)   step sweep 900 bash scripts/steps_sweep.sh ;;
    env_sweep) step env_sweep 1000 bash scripts/env_sweep.sh ;;
    ab)      step ab 900 bash scripts/ab_tpch.sh ;;
    ab_hbm)  step ab_hbm 1200 bash scripts/ab_hbm.sh ;;
    cpubase) step cpubase 900 python scripts/cpu_baselines.py ;;
    abargs)  step abargs 900 bash scripts/ab_args.sh ;;
    overhead) step overhead 300 python scripts/launch_overhead.py ;;
    overhead_ab) for lib in gym-sparksched_amd/build/ab/*.so; do n=$(basename "$lib" .so); echo "--- $n"; SSIM_LIB="$PWD/$lib" step "overhead_$n" 300 python scripts/launch_overhead.py; done ;;
    launch)  step launch 600 python scripts/launch_profile.py ;;
    prof_driver) step prof_driver 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_driver" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 ;;
    ab20np)  step ab20np 900 env AB_TAG=s20np AB_ARGS="--steps 20 --warmup 5 --no-preempt" bash scripts/ab_tpch.sh ;;
    ab20)    step ab20 900 env AB_TAG=s20 AB_ARGS="--steps 20 --warmup 5" bash scripts/ab_tpch.sh ;;
    pmc)     step pmc 900 bash scripts/pmc_profile.sh ;;
    pmc300)  step pmc300 900 env PMC_TAG=k300 PMC_ARGS="--steps 300 --warmup 50" bash scripts/pmc_profile.sh ;;
    pmc_large) step pmc_large 900 env PMC_TAG=large PMC_ARGS="--workload large --steps 100 --warmup 20" bash scripts/pmc_profile.sh ;;
    pmc_decima) step pmc_decima 900 env PMC_TAG=decima PMC_ARGS="--workload decima --steps 40 --warmup 5" bash scripts/pmc_profile.sh ;;
    ab20x)   step ab20x 1200 env AB_TAG=s20 AB_ARGS="--steps 20 --warmup 5" AB_REPS=3 bash scripts/ab_tpch.sh ;;
    prof_step) step prof_step 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_step" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --steps 100 ;;
    hostsim_rate) step hostsim_rate 300 python scripts/hostsim_rate.py 20 ;;
    pmc_latency) step pmc_latency 600 env PMC_TAG=latency PMC_PASSES=latency bash scripts/pmc_profile.sh ;;
    pmc_decima_persist) step pmc_decima_persist 900 env PMC_TAG=decima_persistent PMC_ARGS="--workload decima --steps 40 --warmup 5" bash scripts/pmc_profile.sh ;;
    prof_decima_persist) step prof_decima_persist 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_decima_persist" -o run --output-format csv -- python3 bench.py --workload decima --steps 40 --warmup 5 --no-cpu-baseline ;;
    phase_decima) step phase_decima 600 python scripts/phase_profile_decima.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
