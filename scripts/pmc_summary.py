#!/usr/bin/env python
"""Summarise scripts/pmc_profile.sh output (gpurun_out/pmc/) into a JSON of per-kernel PMC figures.

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from separate passes,
are reported by rocprofv3 in KB (x1024), and FETCH_SIZE is doubled on gfx950 (it tallies 128-B read
requests at 64 B). Figures are taken from the timed (last) dispatch of each kernel and normalised by the
decisions that dispatch made (the bench JSON line in the same pass's log), so bench.py can scale them to
any launch length.

usage: python scripts/pmc_summary.py [gpurun_out/pmc] [out.json]
"""

import csv
import json
import os
import sys


def last_dispatch(path, prefix):
    def base(n):  # "void k_rollout<true, 10, 50>(ssim::Params const*, ...)" -> "k_rollout"
        return n.split("(")[0].split("<")[0].split()[-1]

    rows = [r for r in csv.DictReader(open(path)) if base(r["Kernel_Name"]) == prefix]
    if not rows:
        return None, {}
    last = max(int(r["Dispatch_Id"]) for r in rows)
    vals = {}
    name = None
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    return name, vals


def bench_line(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    res = {"source": "rocprofv3 --pmc, one pass per counter group (scripts/pmc_profile.sh)", "kernels": {}}
    for kern in ("k_rollout", "k_step", "k_decima_rollout"):
        entry = {}
        for pas in ("waves", "icache", "fetch", "write"):
            csvp = os.path.join(root, pas, "run_counter_collection.csv")
            if not os.path.exists(csvp):
                continue
            name, vals = last_dispatch(csvp, kern)
            if not vals:
                continue
            b = bench_line(os.path.join(root, pas + ".log"))
            steps = b["steps"] if b else None
            dec = None
            if b:
                # the timed dispatch is one rollout launch (all steps) or one step launch
                cfg = b["config"]
                spl = cfg.get("steps_per_launch", b["steps"] if cfg["mode"] == "rollout" else 1)
                dec = b["decisions"] * spl / b["steps"]  # launches are equal-length (bench --chunk)
            entry["kernel_name"] = name
            if b and b.get("build_id"):  # every pass must have run the same library build
                if entry.setdefault("build_id", b["build_id"]) != b["build_id"]:
                    raise SystemExit(f"pass {pas} ran build {b['build_id']}, earlier passes {entry['build_id']}")
            entry.setdefault("decisions_per_dispatch", dec)
            entry.setdefault("config", b["config"] if b else None)
            entry.setdefault("steps", steps)
            entry[pas] = vals
        if not entry:
            continue
        dec = entry.get("decisions_per_dispatch")
        if dec and "fetch" in entry and "write" in entry:
            fetch = entry["fetch"]["FETCH_SIZE"] * 1024.0 * 2.0
            write = entry["write"]["WRITE_SIZE"] * 1024.0
            entry["hbm_fetch_bytes_per_decision"] = fetch / dec
            entry["hbm_write_bytes_per_decision"] = write / dec
            entry["hbm_bytes_per_decision"] = (fetch + write) / dec
        if dec and "waves" in entry:
            w = entry["waves"]
            entry["per_decision"] = {k: v / dec for k, v in w.items()}
            cyc = w.get("SQ_WAVE_CYCLES", 0.0)
            if cyc:
                entry["wave_cycle_split"] = {k: w[k] / cyc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                     "SQ_ACTIVE_INST_ANY") if k in w}
                # the bound that binds for one wave per SIMD: the fraction of the wave's life it
                # spends issuing instructions (SQ_* wave counters count quad-cycles; ratios are unit-free)
                pd = entry["per_decision"]
                entry["issue"] = {
                    "bound": "issue/latency: one wave per SIMD, one serial event chain per env",
                    "frac": w["SQ_ACTIVE_INST_ANY"] / cyc, "wait_frac": w.get("SQ_WAIT_ANY", 0.0) / cyc,
                    "wave_cycles_per_decision": 4.0 * pd["SQ_WAVE_CYCLES"],
                    "instructions_per_decision": {k.replace("SQ_INSTS_", "").lower(): pd[k] for k in pd
                                                  if k.startswith("SQ_INSTS_")},
                    "simds": 1024}
        res["kernels"][kern] = entry
    txt = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
