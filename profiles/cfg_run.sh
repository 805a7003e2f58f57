#!/bin/bash
# One-off measurements of the larger configs at N=1 (C3, then C4), one timed iteration each.
# usage (from the repo root, via gpurun): profiles/cfg_run.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --json-out "$OUT/c3.json" \
    > "$OUT/c3.log" 2>&1 || { echo c3 failed; tail -n 30 "$OUT/c3.log"; exit 1; }
cat "$OUT/c3.json"; echo
timeout -k 10 800 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --no-diag --json-out "$OUT/c4.json" \
    > "$OUT/c4.log" 2>&1 || { echo c4 failed; tail -n 30 "$OUT/c4.log"; exit 1; }
cat "$OUT/c4.json"; echo
