#!/bin/bash
# Decima rollout variants (gym-sparksched_amd/build/ab/*.so): rate + HBM fetch / write per decision (separate PMC
# passes). Each run has its own time limit; stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab_decima_pmc
mkdir -p "$OUT"
ARGS="--workload decima --steps 40 --warmup 5 --no-cpu-baseline"
for lib in gym-sparksched_amd/build/${AB_OUT:-ab}/*.so; do
  n=$(basename "$lib" .so)
  SSIM_LIB="$PWD/$lib" timeout -k 10 300 python bench.py $ARGS > "$OUT/${n}_bench.log" 2>&1
  rc=$?; echo "$n bench rc=$rc $(grep -o '"value": [0-9.]*' $OUT/${n}_bench.log)"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${n}_bench.log"; exit $rc; fi
  for pas in FETCH_SIZE WRITE_SIZE; do
    SSIM_LIB="$PWD/$lib" timeout -s KILL 300 rocprofv3 --pmc $pas -d "$PWD/$OUT/${n}_$pas" -o run --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/${n}_$pas.log" 2>&1
    rc=$?; echo "$n $pas rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${n}_$pas.log"; exit $rc; fi
  done
done
echo "=== ab_decima_pmc done"
