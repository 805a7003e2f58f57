#!/bin/bash
# Round 3b run 7 (via gpurun): knob re-sweep on the current kernel -- work roots S 128 / 512,
# register budgets (occupancy 5 / 7), and for C3 (dense contributions) the transposed-scan threshold
# and RMW rounds 16 / 32.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run7}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base ""


run occ5 "" --occupancy 5
run occ7 "" --occupancy 7
run base2 ""
C3="--workload c3 --steps 1 --warmup 0"
run c3 "" $C3
run c3_t4 "" $C3 --tscan 4
run c3_t8 "" $C3 --tscan 8
run c3_rmw16 rmw16 $C3
run c3_rmw32 rmw32 $C3
run c3_occ5 "" $C3 --occupancy 5
run c3_s128 "" $C3 --split 128
