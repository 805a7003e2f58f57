#!/bin/bash
# Round 6 experiment 12 (via gpurun): the closing tree against the library of the first closing run
# (1a8bed9: before the libm-exact transcendentals and the sparse partials), and the closing tree with dense
# partials (option 120 = 0), A/B/C/A/B/C on C2, on one box.
set -o pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
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
      "it0", round(g[0], 1), "it15", round(g[-1], 1), "digest", (d.get("film_digest") or {}).get("sha256"))
PY
}
for r in a b; do
  run c2_new_$r ""
  run c2_old_$r $OLD
  run c2_dense_$r "" --sparse-partials 0
done
