#!/usr/bin/env python3
"""Summarise a profiles/run_profiles.sh output directory into a small committed JSON:
per kernel, calls / average duration (kernel trace) and per-dispatch FETCH_SIZE / WRITE_SIZE
(rocprofv3 reports KB; gfx950 FETCH_SIZE under-reads wide streaming reads by 2x, see
MI355X_MICROARCH.md §HBM — both the raw value and the x2-corrected bytes are kept)."""
import csv
import json
import os
import sys


def short(name):
    name = name.replace("bre::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:80]


def main(d, out):
    res = {}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        res.setdefault(k, {})
        res[k]["calls"] = int(r["Calls"])
        res[k]["avg_ns"] = float(r["AverageNs"])
        res[k]["total_ns"] = float(r["TotalDurationNs"])
    # per-dispatch durations of the gather kernels, in launch order (the bench's iteration-0 launch is
    # the one its roofline times with HIP events)
    trace = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        for r in csv.DictReader(open(trace)):
            k = short(r["Kernel_Name"])
            if ("gather" in k or "k_photons" in k or "k_camera" in k) and k in res:
                ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
                res[k].setdefault("dispatch_ms", []).append(round(ms, 3))
    for v in res.values():  # the passes' medians (round 5: pipelined passes beside the gather)
        if v.get("dispatch_ms"):
            srt = sorted(v["dispatch_ms"])
            v["median_dispatch_ms"] = srt[len(srt) // 2]
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = {}
        for r in csv.DictReader(open(p)):
            agg.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
        for k, v in agg.items():
            res.setdefault(k, {})
            res[k][cname + "_KB_per_dispatch"] = sum(v) / len(v)
    for k, v in res.items():
        if "FETCH_SIZE_KB_per_dispatch" in v:
            v["hbm_read_bytes_corrected"] = v["FETCH_SIZE_KB_per_dispatch"] * 1024 * 2
        if "WRITE_SIZE_KB_per_dispatch" in v:
            v["hbm_write_bytes"] = v["WRITE_SIZE_KB_per_dispatch"] * 1024
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if "gather" in k}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
