#!/bin/bash
# A/B of alternative builds (gym-sparksched_amd/build/ab/*.so) on the default bench, alternating twice;
# each run has its own time limit and the script stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 "${AB_REPS:-2}"); do
  for lib in gym-sparksched_amd/build/${AB_OUT:-ab}/*.so; do
    n=$(basename "$lib" .so)
    SSIM_LIB="$PWD/$lib" timeout -k 10 200 python bench.py --no-cpu-baseline ${AB_ARGS:-} > "gpurun_out/ab/${n}_tpch_${AB_TAG:-d}_$rep.log" 2>&1
    rc=$?
    echo "$n rep$rep rc=$rc $(tail -1 gpurun_out/ab/${n}_tpch_${AB_TAG:-d}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d[\"value\"]/1e6,3), \"M\", round(d[\"roofline\"][\"kernel_ms_per_launch\"],4), \"ms\")" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
