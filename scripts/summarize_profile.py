"""Copy a rocprofv3 run (scripts/profile.sh output) into profiles/<name>/.

Writes kernel_stats.csv (the --kernel-trace --stats summary), pmc_summary.json
(FETCH_SIZE / WRITE_SIZE per dispatch of the POA kernel) and, for the bench
config, profiles/traffic_poa_<config>.json which bench.py reports as
roofline.traffic.  HBM bytes per launch = 2 x FETCH_SIZE (gfx950 tallies a
128 B read request as 64 B; MI355X_MICROARCH.md, HBM/rocprofv3 section)
+ WRITE_SIZE, both in KB.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, name, config="B", windows=1024, kernel="poa_window_kernel", steps=None):
    dst = os.path.join(ROOT, "profiles", name)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))))
    poa = [r for r in stats if kernel in r["Name"]]
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = csv.DictReader(open(os.path.join(src, "pmc_" + c, "pmc_counter_collection.csv")))
        vals[c] = [float(r["Counter_Value"]) for r in rows
                   if kernel in r["Kernel_Name"] and r["Counter_Name"] == c]
    fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    hbm = int((2 * fetch + write) * 1024)
    summ = {"kernel": poa[0]["Name"] if poa else None,
            "avg_duration_ns": float(poa[0]["AverageNs"]) if poa else None,
            "counters_kb_per_launch": vals,
            "hbm_bytes_per_launch": hbm,
            "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, KB per dispatch; "
                    "hbm bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024"}
    if config == "E":
        # config E streams many launches of varying size: bytes per window,
        # summed over every dispatch of the profiled run
        fsum = sum(vals["FETCH_SIZE"])
        wsum = sum(vals["WRITE_SIZE"])
        tot = int((2 * fsum + wsum) * 1024)
        summ["hbm_bytes_all_dispatches"] = tot
        summ["windows"] = windows
        summ["hbm_bytes_per_window"] = tot / windows
    json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    if config == "E":
        json.dump({"config": config, "windows": windows, "hbm_bytes_per_window": tot / windows,
                   "source": "profiles/" + name}, open(os.path.join(ROOT, "profiles", "traffic_poa_E.json"), "w"),
                  indent=1)
    elif kernel.startswith("poa_window_kernel"):
        json.dump({"config": config, "windows": windows, "hbm_bytes_per_launch": hbm, "source": "profiles/" + name},
                  open(os.path.join(ROOT, "profiles", "traffic_poa_%s.json" % config), "w"), indent=1)
    else:
        t = {"config": config, "pairs": windows, "hbm_bytes_per_launch": hbm, "source": "profiles/" + name}
        if steps:
            # align_all() of a large batch runs several launches per step
            # (pipeline stages on two streams): bytes per step = every
            # dispatch of the profiled run / the steps it ran (warmup included)
            t["dispatches_per_step"] = len(vals["FETCH_SIZE"]) / steps
            t["hbm_bytes_per_step"] = int((2 * sum(vals["FETCH_SIZE"]) + sum(vals["WRITE_SIZE"])) * 1024 / steps)
            t["kernel_ns_sum_per_step"] = (float(poa[0]["TotalDurationNs"]) / steps) if poa else None
            summ.update({k: t[k] for k in ("dispatches_per_step", "hbm_bytes_per_step", "kernel_ns_sum_per_step")})
            json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
        json.dump(t, open(os.path.join(ROOT, "profiles", "traffic_aligner_%s.json" % config), "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2] if len(a) > 2 else "B", int(a[3]) if len(a) > 3 else 1024,
         a[4] if len(a) > 4 else "poa_window_kernel", int(a[5]) if len(a) > 5 else None)
