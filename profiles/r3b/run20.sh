#!/bin/bash
# Round 3b run 20 (via gpurun): knob re-sweep on the closing kernel (the texture-data path now the
# busiest unit): occupancy 5 / 6 (default) / 7, transposed-scan threshold 4 / 6 (default) / 8, C2 and C3.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run20}
mkdir -p "$OUT"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1))"
}
C3="--workload c3 --steps 1 --warmup 0"
run base
run occ5 --occupancy 5
run occ7 --occupancy 7
run ts4 --tscan 4
run ts8 --tscan 8
run c3_base $C3
run c3_occ5 $C3 --occupancy 5
run c3_occ7 $C3 --occupancy 7
run base2
