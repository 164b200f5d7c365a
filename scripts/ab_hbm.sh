#!/bin/bash
# A/B of alternative builds (gym-sparksched_amd/build/ab/*.so) on the HBM-resident workloads; each run has
# its own time limit and the script stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for lib in gym-sparksched_amd/build/ab/*.so; do
  n=$(basename "$lib" .so)
  for w in "large --steps 100 --warmup 100" "decima --steps 20 --warmup 5"; do
    set -- $w
    SSIM_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > "gpurun_out/ab/${n}_$1.log" 2>&1
    rc=$?
    echo "$n $1 rc=$rc $(tail -1 gpurun_out/ab/${n}_$1.log | cut -c1-120)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
