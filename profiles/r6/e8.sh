#!/bin/bash
# Round 6 experiment 8 (via gpurun): the transposed-scan threshold by MaxDistance (option 108 = -1, the new
# default) against the fixed 4 and 5 on C2 (A/B/A/B) and C3; then the tail study (profiles/r6/e7.sh).
set -o pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --no-diag --json-out "$OUT/$n.json" "$@" \
      > "$OUT/$n.log" 2>&1 || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
g = d["gather_ms_per_step"]
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "it0", round(g[0], 1),
      "it15", round(g[15], 1) if len(g) > 15 else None, "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run c2_auto_$r
  run c2_t4_$r --tscan 4
  run c2_t5_$r --tscan 5
done
run c3_auto --workload c3 --steps 1 --warmup 1
run c3_t4 --tscan 4 --workload c3 --steps 1 --warmup 1
bash profiles/r6/e7.sh "$OUT/e7"
