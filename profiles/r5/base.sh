#!/bin/bash
# Round 5 session start (via gpurun): smoke and the driver-shaped bench line (20 steps) on the
# round-4 closing code, to see this round's box.
set -o pipefail
OUT=${1:-gpurun_out/r5/base}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 60 ./profiles/r5/probe/mfma4x4 > "$OUT/mfma4x4.txt" 2>&1; echo "probe rc $?"; tail -n 3 "$OUT/mfma4x4.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -n 30 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
    || { tail -n 30 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log" | cut -c1-400
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])])"
