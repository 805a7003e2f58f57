#!/bin/bash
# Round 4 run 34 (via gpurun): average resident waves of the tile kernel at N = 1 and for an emulated
# rank of 8 (C2, one timed iteration 0 and one iteration 8): SQ_WAVES / SQ_WAVE_CYCLES / SQ_BUSY_CYCLES /
# GRBM_GUI_ACTIVE in one PMC pass each -- is the rank's excess a launch tail (fewer resident waves)?
set -o pipefail
OUT=${1:-gpurun_out/r4/run34}
mkdir -p "$OUT"
export TMPDIR=/tmp
for x in "n1:" "r0of8:--emulate-shard 0/8"; do
  n=${x%%:*}; a=${x#*:}
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU \
      --kernel-trace --output-format csv -d "$OUT/$n" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-pmc --no-diag $a \
      > "$OUT/$n.log" 2>&1 || { echo "pmc $n failed"; tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for r in csv.DictReader(open(f)):
    if "k_gather_tile" not in r["Kernel_Name"]:
        continue
    d = r["Dispatch_Id"]
    acc[d][r["Counter_Name"]] += float(r["Counter_Value"])
    dur[d] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e6
for d in sorted(acc, key=int):
    v = acc[d]
    clk = v["GRBM_GUI_ACTIVE"] / 8.0
    print(sys.argv[1].split("/")[-1], "dispatch", d, "ms %.2f" % dur[d], "waves %.0f" % v["SQ_WAVES"],
          "avg resident waves/CU %.2f" % (v["SQ_WAVE_CYCLES"] / max(clk, 1) / 256.0),
          "busy frac %.3f" % (v["SQ_BUSY_CYCLES"] / max(clk, 1) / 32.0), "VALU/wave %.0f" % (v["SQ_INSTS_VALU"] / max(v["SQ_WAVES"], 1)))
PY
done
