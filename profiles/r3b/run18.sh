#!/bin/bash
# Round 3b run 18 (via gpurun): the default bench line with the vector-memory (TA / TD) PMC pass.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run18}
mkdir -p "$OUT"
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
    || { tail -n 30 "$OUT/bench.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('value', round(d['value']), 'frac', r['frac'], {k: r['issue'].get(k) for k in ('td_busy_frac','ta_busy_frac','lds_busy_frac','busiest_unit')})"
