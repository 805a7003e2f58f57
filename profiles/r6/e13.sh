#!/bin/bash
# Round 6 experiment 13 (via gpurun): coarse sort keys (internal option 121: the tree-order sort on the
# keys' bits [16, 64), the segment sort on [12, 60) -- 6 radix passes each instead of 8) against all
# bits, A/B/A/B on C2 and on an emulated rank of 8, once on C3.
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
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "it0", round(g[0], 1), "last", round(g[-1], 1), "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run c2_fine_$r --coarse-keys 0
  run c2_coarse_$r --coarse-keys 1
  run r8_fine_$r --coarse-keys 0 --emulate-shard 0/8
  run r8_coarse_$r --coarse-keys 1 --emulate-shard 0/8
done
run c3_fine --coarse-keys 0 --workload c3 --steps 1 --warmup 1
run c3_coarse --coarse-keys 1 --workload c3 --steps 1 --warmup 1
