#!/bin/bash
# Round 6 experiment 9 (via gpurun): the libm-exact transcendentals (include/bre_fmath.h, round 6) against
# the Cephes-form library of the commit before them (csrc/build/variants/libbre_cephes.so, built from
# 1a8bed9), A/B/A/B on C2 and once on C3 (the smoke grid: logf on every delta-tracking step); and C2
# with serial iterations (the tile kernel alone on the GPU).
set -o pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
OLD=beam-radiance-estimate-pbrt_amd/csrc/build/variants/libbre_cephes.so
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --no-diag --json-out "$OUT/$n.json" "$@" \
      > "$OUT/$n.log" 2>&1 || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
g = d["gather_ms_per_step"]
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "photon", d.get("photon_pass_ms"), "camera", d.get("camera_pass_ms"),
      "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run c2_libm_$r ""
  run c2_cephes_$r $OLD
done
# the tile kernel with no pass chain beside it (serial iterations): what the chain costs the gather
run c2_serial "" --pipeline 0
run c3_libm "" --workload c3 --steps 1 --warmup 1
run c3_cephes $OLD --workload c3 --steps 1 --warmup 1
