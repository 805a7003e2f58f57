#!/bin/bash
# Round 5 run 19 (via gpurun): knob re-sweep on the round-5 kernel -- transposed-scan threshold
# (option 108, eighths: default 6) and the tile kernel's occupancy target (option 102: default 6), C2 and C3.
set -o pipefail
OUT=${1:-gpurun_out/r5/run19}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'it0', round(g[0],1), 'it15', round(g[-1],1))"
}
for r in a b; do
  run c2_def_$r
  run c2_t4_$r --tscan 4
  run c2_t8_$r --tscan 8
  run c2_o7_$r --occupancy 7
done
run c3_def --workload c3 --steps 1 --warmup 1
run c3_t4 --workload c3 --steps 1 --warmup 1 --tscan 4
run c3_t8 --workload c3 --steps 1 --warmup 1 --tscan 8
