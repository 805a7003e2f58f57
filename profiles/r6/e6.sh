#!/bin/bash
# Round 6 experiment 6 (via gpurun): the transposed-scan threshold re-swept on the round-6 pipeline
# (option 108, eighths: a tile is scanned transposed when on-lanes * 8 < kept beams * t), C2 and C3.
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
  for t in 3 4 5; do run c2_t${t}_$r --tscan $t; done
done
for t in 3 4 5; do run c3_t$t --tscan $t --workload c3 --steps 1 --warmup 1; done
