#!/bin/bash
# Round 5 same-box A/B (via gpurun): the default libbre against the variant build(s) named after OUT
# (csrc/build/variants/libbre_NAME.so): the gather parity tests on the default build, per-segment sums
# bit for bit against each variant (C2 iterations 0 / 8 / 15), then C2 and C3 timing, A/B/A/B.
# usage: bash profiles/r5/ab.sh OUT NAME [NAME ...]
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_c2_production.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py \
    tests/test_film_determinism_gpu.py ${AB_TESTS:-} > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
BRE_LIBRARY=$DEF timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 \
    || { tail -n 20 "$OUT/bc_def.log"; exit 1; }
for n in "$@"; do
  BRE_LIBRARY=$V/libbre_$n.so timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_$n.npz" c2 > "$OUT/bc_$n.log" 2>&1 \
      || { tail -n 20 "$OUT/bc_$n.log"; exit 1; }
  echo "== def vs $n"; python3 profiles/r5/bitcmp.py cmp "$OUT/bc_def.npz" "$OUT/bc_$n.npz"
  rm -f "$OUT/bc_$n.npz"
done
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); n = sys.argv[2]
c = d.get("counters_last_iteration") or {}
print(n, "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), "gather", round(d["gather_kernel_ms"], 1),
      "it0", round(d["gather_ms_per_step"][0], 1),
      "it15", round(d["gather_ms_per_step"][-1], 1) if len(d["gather_ms_per_step"]) > 15 else None,
      "keep", round(d.get("bundle_keep_frac", 0), 4), "t/q", round(d.get("prefilter_tests_per_queued_pair", 0), 2),
      "| late keep", round(c.get("bundle_keep_frac", 0), 4), "t/q", round(c.get("prefilter_tests_per_queued_pair", 0), 2))
PY
}
C3="--workload c3 --steps 1 --warmup 1"
for r in a b; do
  run c2_def_$r $DEF
  for n in "$@"; do run c2_${n}_$r $V/libbre_$n.so; done
done
run c3_def $DEF $C3
for n in "$@"; do run c3_$n $V/libbre_$n.so $C3; done
