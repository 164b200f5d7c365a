#!/bin/bash
# A/B of library variants (gym-sparksched_amd/build/ab/<name>.so via SSIM_LIB) against the in-tree library on one
# bench command, alternating, AB_REPS rounds: AB_ARGS="--workload decima --steps 40 --warmup 5" bash scripts/ab_lib.sh
set -u
O=gpurun_out/ab_lib; mkdir -p $O
ARGS=${AB_ARGS:-"--no-cpu-baseline"}
for i in $(seq 1 ${AB_REPS:-2}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > $O/main_$i.log 2>&1 || exit $?
  for lib in gym-sparksched_amd/build/ab/*.so; do
    n=$(basename $lib .so)
    SSIM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > $O/${n}_$i.log 2>&1 || exit $?
  done
done
for f in $O/*.log; do echo "$f $(grep -o '"value": [0-9.e+]*' $f)"; done
