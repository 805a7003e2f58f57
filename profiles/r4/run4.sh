#!/bin/bash
# Round 4 run 4 (via gpurun): where the LDS-beam exact stage loses -- per-phase wave cycles
# (BRE_PHASE_TIMING builds: staging / scan / exact / total) and one SQ + one TA/TD counter pass of
# the iteration-0 launch, for the new kernel and the round-3 kernel, one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run4}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
for n in phase phase_r3; do
  BRE_LIBRARY=$V/libbre_$n.so timeout -k 10 200 python -u profiles/phase_timing.py c2 0 15 > "$OUT/$n.log" 2>&1 \
      || { echo "$n failed"; tail -n 20 "$OUT/$n.log"; exit 1; }
  BRE_LIBRARY=$V/libbre_$n.so timeout -k 10 200 python -u profiles/phase_timing.py c3 0 > "$OUT/${n}_c3.log" 2>&1 \
      || { echo "$n c3 failed"; tail -n 20 "$OUT/${n}_c3.log"; exit 1; }
  echo "== $n"; grep iteration "$OUT/$n.log" "$OUT/${n}_c3.log"
done
pass() { # name lib counters...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/pmc_$n -o run -- \
      python3 bench.py --pmc-child --workload c2 --steps 1 --warmup 0 > $OUT/pmc_$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $n rc=$rc"; exit 1; fi
}
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
TT="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
pass sq_new beam-radiance-estimate-pbrt_amd/libbre.so $SQ
pass tt_new beam-radiance-estimate-pbrt_amd/libbre.so $TT
pass sq_r3 $V/libbre_r3.so $SQ
pass tt_r3 $V/libbre_r3.so $TT
python3 - $OUT <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for tag in ("new", "r3"):
    tot = {}
    for f in glob.glob(os.path.join(O, f'pmc_*_{tag}', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_gather_tile' in r['Kernel_Name']:
                tot[r['Counter_Name']] = tot.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    print(tag, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
