#!/bin/bash
# Round 4 run 20 (via gpurun): knob check after the 4-wide walk -- work roots S 64 / 128, occupancy
# 5 / 7, transposed-scan threshold 4 / 8 against the defaults (S 256, occupancy 6, tscan 6), C2, one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run20}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
run c2_def
run c2_s128 --split 128
run c2_s64 --split 64
run c2_occ5 --occupancy 5
run c2_occ7 --occupancy 7
run c2_ts4 --tscan 4
run c2_ts8 --tscan 8
run c2_def2
