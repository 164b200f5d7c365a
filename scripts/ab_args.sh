#!/bin/bash
# A/B of bench argument sets on the in-tree library, alternating (AB_SETS: ';'-separated arg strings), REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_args
IFS=';' read -ra SETS <<< "${AB_SETS:---steps 20 --warmup 5;--steps 20 --warmup 5 --no-preempt}"
for rep in $(seq 1 "${REPS:-2}"); do
  i=0
  for a in "${SETS[@]}"; do
    i=$((i + 1))
    timeout -k 10 200 python bench.py --no-cpu-baseline $a > "gpurun_out/ab_args/set${i}_$rep.log" 2>&1
    rc=$?
    echo "set$i [$a] rep$rep rc=$rc $(tail -1 gpurun_out/ab_args/set${i}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), 'M', round(d['roofline']['kernel_ms_per_launch'],4), 'ms')" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
