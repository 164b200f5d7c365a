#!/bin/bash
# configs[3]'s env (J=200, N=100, time limits) on the HBM-resident specialised kernel at several env counts per GPU
# (bench.py --workload large, 100-step budget launches). Writes gpurun_out/env_sweep_large/. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/env_sweep_large
mkdir -p "$OUT"
for B in ${SWEEP_ENVS:-1024 2048 4096 8192}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --workload large --envs "$B" --steps 100 --warmup 20 > "$OUT/bench_$B.log" 2>&1 || exit $?
  echo "envs=$B $(grep -o '"value": [0-9.e+]*' "$OUT/bench_$B.log")"
done
