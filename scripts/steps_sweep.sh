#!/bin/bash
# Kernel time per launch vs. steps per launch (fixed per-launch cost vs. per-step cost), budget and lockstep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/steps_sweep
mkdir -p "$OUT"
for mode in budget lockstep; do
  extra=""; [ "$mode" = lockstep ] && extra="--lockstep"
  for k in ${SWEEP_STEPS:-5 10 20 40 80 160}; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps "$k" --warmup 5 $extra > "$OUT/${mode}_$k.json" 2>/dev/null
    rc=$?
    if [ $rc -ne 0 ]; then echo "$mode $k rc=$rc"; exit $rc; fi
    python - "$OUT/${mode}_$k.json" "$mode" "$k" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[2]:9s} steps={sys.argv[3]:>4s} value={d['value']/1e6:7.2f}M kernel_ms={r['kernel_ms_per_launch']:.4f} "
      f"ev/dec={d['events_per_decision']:.2f} eps={d['episodes_finished']}")
PY
  done
done
