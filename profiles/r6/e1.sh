#!/bin/bash
# Round 6 experiment 1 (via gpurun): do the next iteration's passes run inside the gather when their
# workgroups are one wave?  Pipelined C2 bench under a kernel trace, default libbre vs variants.
# usage: bash profiles/r6/e1.sh OUT NAME [NAME ...]
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
run() { # name lib
  n=$1; lib=$2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --no-diag --json-out "$OUT/$n.json" \
      > "$OUT/$n.log" 2>&1 || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "gap", round(d["ms_per_step"] - d["gather_kernel_ms"], 3), "digest", (d.get("film_digest") or {}).get("sha256"))
PY
  BRE_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$n" -o run -- \
      python3 bench.py --no-cpu --no-pmc --no-legs --no-diag > "$OUT/tr_$n.log" 2>&1 || { tail -n 20 "$OUT/tr_$n.log"; exit 1; }
  python3 profiles/r6/gap.py "$OUT/tr_$n/run_kernel_trace.csv" "$n"
}
run def $DEF
for n in "$@"; do run $n $V/libbre_$n.so; done
