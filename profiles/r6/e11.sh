#!/bin/bash
# Round 6 experiment 11 (via gpurun): sparse tile-kernel partials (internal option 120 = 1, the default)
# against every (packet, work root) partial (0), A/B/A/B on C2 and on an emulated rank of 8, and the
# reduce's duration with serial iterations under rocprofv3.
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
      "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run c2_sparse_$r
  run c2_dense_$r --sparse-partials 0
  run r8_sparse_$r --emulate-shard 0/8
  run r8_dense_$r --emulate-shard 0/8 --sparse-partials 0
done
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$v" -o run -- python3 -u bench.py \
      --no-cpu --no-pmc --no-legs --no-diag --pipeline 0 --steps 4 --warmup 1 --sparse-partials $v > "$OUT/tr_$v.log" 2>&1 \
      || { tail -n 20 "$OUT/tr_$v.log"; exit 1; }
  f=$(find "$OUT/tr_$v" -name "*kernel_stats.csv" | head -1)
  grep -E "k_reduce|k_gather_tile" "$f" | cut -c1-60,200-300
done
