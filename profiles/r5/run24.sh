#!/bin/bash
# Round 5 run 24 (via gpurun): work roots per packet (--split) re-swept with threshold 4, C2 and C3.
set -o pipefail
OUT=${1:-gpurun_out/r5/run24}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'it0-3', [round(x,1) for x in g[:4]], 'it15', round(g[-1],1))"
}
for S in 256 128 512; do run c2_s$S --split $S; done
for S in 256 128 512; do run c3_s$S --workload c3 --steps 1 --warmup 1 --split $S; done
run c2_t3 --tscan 3
run c2_t5 --tscan 5
run c2_s256_b
