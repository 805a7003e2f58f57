#!/bin/bash
# r2: memory-pipeline counters of the tile kernel (one C2 iteration 0 per pass, bench --pmc-child):
# TA / TD busy, TCP accesses, VMEM / SMEM / SALU instruction counts.  One counter group per pass;
# a pass killed by its time limit ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${EXPLORE_OUT:-pmc_ta}; mkdir -p $O
pass() { # name counters...
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- \
      python3 bench.py --pmc-child --workload ${WL:-c2} --steps 1 --warmup 0 > $O/$n.log 2>&1
  rc=$?
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then echo "pass $n killed ($rc)"; exit 1; fi
  echo "pass $n rc=$rc"
}
pass ta TA_TA_BUSY_sum GRBM_GUI_ACTIVE || exit 1
pass td TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE || exit 1
pass sq SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
python3 - $O <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
tot = {}
for f in glob.glob(os.path.join(O, '*', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_gather_tile' in r['Kernel_Name']:
            tot[r['Counter_Name']] = tot.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
for k in sorted(tot): print(k, tot[k])
PY
