#!/usr/bin/env python3
"""Summarise profiles/sq_passes.sh output: per gather kernel, the SQ counters summed over its
dispatches, plus derived issue figures.

gfx950 units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
per wave (summed over waves); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  A SIMD-32 issues one wave64
VALU instruction per 2 cycles, so the chip's VALU issue peak is 256 CU x 4 SIMD / 2 = 512 wave
instructions per clock; `valu_issue_frac` = SQ_INSTS_VALU / (512 x kernel clocks)."""
import csv
import json
import os
import sys

CUS, SIMDS = 256, 4


def short(name):
    name = name.replace("bre::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:80]


def load(d, sub):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    agg = {}
    if not os.path.exists(p):
        return agg
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        agg.setdefault(k, {})
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return agg


def main(d, out):
    res = {}
    for sub in ("sqa", "sqb"):
        for k, v in load(d, sub).items():
            if "gather" not in k and "reduce" not in k:
                continue
            res.setdefault(k, {})
            for c, x in v.items():
                res[k][c if c not in res[k] else c + "_" + sub] = x
    for k, v in res.items():
        clocks = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # per-XCD clock count of the dispatches
        if clocks > 0 and "SQ_INSTS_VALU" in v:
            v["valu_issue_frac"] = v["SQ_INSTS_VALU"] / (CUS * SIMDS / 2.0 * clocks)
            v["lds_inst_per_clock_per_cu"] = v.get("SQ_INSTS_LDS", 0.0) / (CUS * clocks)
        if v.get("SQ_WAVE_CYCLES"):
            wc = v["SQ_WAVE_CYCLES"]
            v["wait_any_frac"] = v.get("SQ_WAIT_ANY", 0.0) / wc
            v["wait_inst_any_frac"] = v.get("SQ_WAIT_INST_ANY", 0.0) / wc
            v["active_inst_any_frac"] = v.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
