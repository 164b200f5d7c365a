#!/bin/bash
# A/B of alternative builds (gym-sparksched_amd/build/${AB_OUT:-ab}/*.so) on the PPO iteration (configs[4]): collect and
# learn seconds per iteration, alternating AB_REPS times; each run has its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 "${AB_REPS:-2}"); do
  for lib in gym-sparksched_amd/build/${AB_OUT:-ab}/*.so; do
    n=$(basename "$lib" .so)
    SSIM_LIB="$PWD/$lib" timeout -k 10 400 python bench.py --workload ppo --steps 2 --warmup 1 --no-cpu-baseline > "gpurun_out/ab/${n}_ppo_$rep.log" 2>&1
    rc=$?
    echo "$n rep$rep rc=$rc $(grep '^{' gpurun_out/ab/${n}_ppo_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['phase_seconds_rank0'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab/${n}_ppo_$rep.log"; exit $rc; fi
  done
done
