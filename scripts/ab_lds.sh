#!/bin/bash
# A/B of the rollout launch's LDS floor (SSIM_LDS_FLOOR_KB): padding the dynamic LDS request caps how many
# env waves one CU hosts, so the 1024-env default spreads over all CUs. Each run has its own time limit and
# the script stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_lds
for kb in "$@"; do
  SSIM_LDS_FLOOR_KB=$kb timeout -k 10 200 python bench.py --no-cpu-baseline > "gpurun_out/ab_lds/kb${kb}.log" 2>&1
  rc=$?
  echo "kb=$kb rc=$rc $(tail -1 gpurun_out/ab_lds/kb${kb}.log | cut -c1-110)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
