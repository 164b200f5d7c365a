#!/bin/bash
# configs[1] (50 TPC-H jobs / 10 executors, random valid actions) at several env counts per GPU: bench.py's default
# timed sequence (300 steps, 50 warm-up) and one PMC pass of the wave counters (SQ_WAVE_CYCLES, SQ_WAIT_ANY, ...) of
# the same command per count. Writes gpurun_out/env_sweep/. Stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/env_sweep
mkdir -p "$OUT"
export TMPDIR=/tmp
for B in ${SWEEP_ENVS:-1024 4096 16384}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --envs "$B" --steps 300 --warmup 50 > "$OUT/bench_$B.log" 2>&1
  rc=$?; echo "bench envs=$B rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$B.log"; exit $rc; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d "$PWD/$OUT/pmc_$B" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --envs "$B" --steps 300 --warmup 50 > "$OUT/pmc_$B.log" 2>&1
  rc=$?; echo "pmc envs=$B rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pmc_$B.log"; exit $rc; }
done
python - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
rows = []
for b in sorted(int(os.path.basename(p)[6:-4]) for p in glob.glob(os.path.join(out, "bench_*.log"))):
    line = [l for l in open(os.path.join(out, f"bench_{b}.log")) if l.startswith("{")][-1]
    d = json.loads(line)
    csvp = glob.glob(os.path.join(out, f"pmc_{b}", "**", "*counter_collection.csv"), recursive=True)
    pmc = {}
    if csvp:
        recs = [r for r in csv.DictReader(open(csvp[0])) if "k_rollout" in r["Kernel_Name"] and "warmup" not in r["Kernel_Name"]]
        last = max(int(r["Dispatch_Id"]) for r in recs)
        for r in recs:
            if int(r["Dispatch_Id"]) == last:
                pmc[r["Counter_Name"]] = pmc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cyc = pmc.get("SQ_WAVE_CYCLES", 0.0)
    rows.append({"envs": b, "decisions_per_s": d["value"], "kernel_ms_per_launch": d["roofline"]["kernel_ms_per_launch"],
                 "wait_any_frac": pmc.get("SQ_WAIT_ANY", 0.0) / cyc if cyc else None,
                 "active_inst_frac": pmc.get("SQ_ACTIVE_INST_ANY", 0.0) / cyc if cyc else None,
                 "waves": pmc.get("SQ_WAVES")})
    print(json.dumps(rows[-1]))
json.dump(rows, open(os.path.join(out, "env_sweep.json"), "w"), indent=1)
PY
