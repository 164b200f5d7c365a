#!/bin/bash
# A/B: the round-3 library (ab_r3/, staged by hand, not tracked) vs the current one on the default bench, then the
# configs[1] env on the HBM-resident kernels vs the LDS-resident one at several env counts. gpurun_out/ab1/.
set -u
O=gpurun_out/ab1; mkdir -p $O
if [ -d ab_r3 ]; then
  for i in 1 2; do
    timeout -k 10 120 python ab_r3/bench.py --no-cpu-baseline > $O/r3_$i.log 2>&1 || exit $?
    timeout -k 10 120 python bench.py --no-cpu-baseline > $O/cur_$i.log 2>&1 || exit $?
  done
fi
for B in ${AB_ENVS:-2048 3072 4096 8192}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --force-hbm --envs $B > $O/hbm_$B.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline --envs $B > $O/lds_$B.log 2>&1 || exit $?
done
