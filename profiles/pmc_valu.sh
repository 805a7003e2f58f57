#!/bin/bash
# One SQ PMC pass over a short C2 bench run (instruction mix / utilisation of the gather kernels).
# usage: profiles/pmc_valu.sh OUTDIR [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
shift || true
ARGS=("$@")
if [ ${#ARGS[@]} -eq 0 ]; then ARGS=(--steps 1 --warmup 1 --no-cpu --no-diag); fi
mkdir -p "$OUT"
PMC=${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY}
timeout -s KILL 240 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d "$OUT/sq" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/bench_sq.log" 2>&1
rc=$?
python3 - "$OUT" <<'PY'
import csv, sys, os, json
d = sys.argv[1]
p = os.path.join(d, "sq", "run_counter_collection.csv")
agg = {}
for r in csv.DictReader(open(p)):
    k = r["Kernel_Name"].replace("bre::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    if "gather" not in k:
        continue
    agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
for k, v in out.items():
    if "SQ_WAVE_CYCLES" in v and v["SQ_WAVE_CYCLES"] > 0:
        v["valu_frac_of_wave_cycles"] = v.get("SQ_ACTIVE_INST_VALU", 0) / v["SQ_WAVE_CYCLES"]
json.dump(out, open(os.path.join(d, "sq_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
PY
exit $rc
