#!/bin/bash
# A/B of Decima rollout variant libraries (gym-sparksched_amd/build/ab_dr/*.so, scripts/build_ab.py with
# AB_OUT=ab_dr): configs[2] bench line per variant, alternating, AB_REPS rounds.
cd "$(dirname "$0")/.."
O=gpurun_out/ab_decima
mkdir -p $O
for r in $(seq 1 ${AB_REPS:-1}); do
  for L in gym-sparksched_amd/build/ab_dr/*.so; do
    n=$(basename $L .so)
    SSIM_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --workload decima --steps 40 --warmup 5 > $O/${n}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/${n}_$r.log').read().strip().splitlines()[-1]); print('$n', $r, round(d['value']/1e6,3), 'M/s', d['roofline']['kernel_ms_per_launch'])"
  done
done
