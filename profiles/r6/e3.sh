#!/bin/bash
# Round 6 experiment 3 (via gpurun): the one-wave pass chain with and without the tile-kernel fence of
# the pipelined contexts (bre_set_gather_after), against rocPRIM on the chain; N = 1 and an emulated rank
# of 8, A/B/A/B on one box; kernel traces of the default for the gaps between gathers.
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
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "gap", round(d["ms_per_step"] - d["gather_kernel_ms"], 3), "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
trace() { # name args...
  n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$n" -o run -- \
      python3 bench.py --no-cpu --no-pmc --no-legs --no-diag "$@" > "$OUT/tr_$n.log" 2>&1 || { tail -n 20 "$OUT/tr_$n.log"; exit 1; }
  python3 profiles/r6/gap.py "$OUT/tr_$n/run_kernel_trace.csv" "$n"
}
for r in a b; do
  run fence_$r
  run nofence_$r --gather-fence 0
  run rocprim_$r --slot-passes 0 --gather-fence 0
done
for r in a b; do
  run fence_e8_$r --emulate-shard 0/8
  run nofence_e8_$r --emulate-shard 0/8 --gather-fence 0
  run rocprim_e8_$r --emulate-shard 0/8 --slot-passes 0 --gather-fence 0
done
trace fence
trace fence_e8 --emulate-shard 0/8
