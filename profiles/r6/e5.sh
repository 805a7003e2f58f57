#!/bin/bash
# Round 6 experiment 5 (via gpurun): pipelined contexts at two stream priorities without the fence (the
# higher-priority gather's blocks are dispatched first, the other's fill its tail) against the fence.
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
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "tile", round(d["gather_kernel_ms"], 3),
      "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run fence_$r
  run prio_$r --gather-fence 0 --gather-priority 1
  run fence_e8_$r --emulate-shard 0/8
  run prio_e8_$r --emulate-shard 0/8 --gather-fence 0 --gather-priority 1
done
