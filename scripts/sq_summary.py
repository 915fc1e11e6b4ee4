"""Summarise rocprofv3 SQ counter passes (scripts/pmc_sq.sh output) for one
kernel into profiles/<name>/sq_summary.json and profiles/sq_<config>.json.

Counters are wave-instruction counts and quad-cycle counts summed over the
dispatch (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*
count quad-cycles).  Derived:
  valu_issue_util  = SQ_INSTS_VALU x 2 cycles / (kernel ns x 2.4 GHz x 1024 SIMDs)
                     (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles)
  wait_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (parked at s_waitcnt / barrier)
  active_valu_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  salu_per_valu    = SQ_INSTS_SALU / SQ_INSTS_VALU
  sq_busy_frac     = SQ_BUSY_CYCLES / (kernel ns x 2.4 GHz x 32 SQs)  (cycles, summed over the 32 SEs)
Usage: python scripts/sq_summary.py <pmc dir> <profile name> <config key> <kernel substring> <kernel avg ns>
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK_GHZ = 2.4
SIMDS = 1024
SQ_INSTANCES = 32  # one SQ per shader engine (MI355X_MICROARCH.md: 32 SEs); SQ_BUSY_CYCLES sums them


def main(src, name, config, kernel, avg_ns):
    vals = {}
    for f in sorted(glob.glob(os.path.join(src, "g*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id", "0"), 0.0)
            per[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
        for c, d in per.items():
            vals[c] = sum(d.values()) / len(d)
    out = {"kernel_substring": kernel, "kernel_avg_ns": avg_ns, "per_launch": vals}
    g = vals.get
    if g("SQ_INSTS_VALU") and avg_ns:
        out["valu_issue_util"] = round(g("SQ_INSTS_VALU") * 2 / (avg_ns * CLOCK_GHZ * SIMDS), 4)
    if g("SQ_WAVE_CYCLES"):
        if g("SQ_WAIT_ANY") is not None:
            out["wait_frac"] = round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 4)
        if g("SQ_ACTIVE_INST_VALU") is not None:
            out["active_valu_frac"] = round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 4)
        if g("SQ_WAIT_INST_ANY") is not None:
            out["issue_stall_frac"] = round(g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), 4)
    if g("SQ_INSTS_SALU") and g("SQ_INSTS_VALU"):
        out["salu_per_valu"] = round(g("SQ_INSTS_SALU") / g("SQ_INSTS_VALU"), 3)
    if g("SQ_BUSY_CYCLES") and avg_ns:
        out["sq_busy_frac"] = round(g("SQ_BUSY_CYCLES") / (avg_ns * CLOCK_GHZ * SQ_INSTANCES), 4)
    out["note"] = ("rocprofv3 --pmc, one pass per counter group (scripts/pmc_sq.sh); SQ_* summed over the "
                   "dispatch; quad-cycle units for *_CYCLES / WAIT / ACTIVE; valu_issue_util assumes 2 cycles "
                   "per wave64 VALU instruction at %.1f GHz on %d SIMDs" % (CLOCK_GHZ, SIMDS))
    dst = os.path.join(ROOT, "profiles", name)
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "sq_summary.json"), "w"), indent=1)
    out["source"] = "profiles/" + name
    json.dump(out, open(os.path.join(ROOT, "profiles", "sq_%s.json" % config), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2], a[3], float(a[4]))
