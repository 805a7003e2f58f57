#!/bin/bash
# Round 3b: memory-pipeline counters of the tile kernel (one iteration-0 launch per pass, bench
# --pmc-child) for C2 and C3: TA / TD busy, TCP, VMEM / LDS / VALU instruction counts.  One counter
# group per pass; a pass killed by its time limit ends the script.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r3b/pmc_ta}; mkdir -p $O
pass() { # workload name counters...
  wl=$1; n=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$wl/$n -o run -- \
      python3 bench.py --pmc-child --workload $wl --steps 1 --warmup 0 > $O/${wl}_$n.log 2>&1
  rc=$?
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then echo "pass $wl $n killed ($rc)"; exit 1; fi
  echo "pass $wl $n rc=$rc"
}
for wl in c2 c3; do
  pass $wl ta TA_TA_BUSY_sum GRBM_GUI_ACTIVE || exit 1
  pass $wl td TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
  pass $wl sq SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE || exit 1
done
python3 - $O <<'PY'
import csv, glob, os, sys, json
O = sys.argv[1]
out = {}
for wl in ("c2", "c3"):
    tot = {}
    for f in glob.glob(os.path.join(O, wl, '*', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_gather_tile' in r['Kernel_Name']:
                tot[r['Counter_Name']] = tot.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    out[wl] = tot
    print(wl, json.dumps(tot))
json.dump(out, open(os.path.join(O, "pmc_ta.json"), "w"), indent=1)
PY
