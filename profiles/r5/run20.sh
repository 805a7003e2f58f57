#!/bin/bash
# Round 5 run 20 (via gpurun): transposed-scan threshold sweep (option 108, eighths) on the round-5 kernel,
# C2 (per-iteration gathers) and C3.
set -o pipefail
OUT=${1:-gpurun_out/r5/run20}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'g', [round(x,1) for x in g])"
}
for t in 6 0 2 3 4 5; do run c2_t$t --tscan $t; done
for t in 6 0 2 3 4 5; do run c3_t$t --workload c3 --steps 1 --warmup 1 --tscan $t; done
run c2_t6_b --tscan 6
run c2_t3_b --tscan 3
run c2_t4_b --tscan 4
