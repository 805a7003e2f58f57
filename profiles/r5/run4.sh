#!/bin/bash
# Round 5 run 4 (via gpurun): directional spread in the packet line reject (BRE_DIR_SPREAD, the
# octagon of the lanes' extents along the common normal) -- per-segment sums bit for bit against the
# build without it, the parity tests, then C2 (counters at iterations 0 and 15) and C3 timing, A/B/A/B.
set -o pipefail
OUT=${1:-gpurun_out/r5/run4}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_c2_production.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
for lib in $DEF $V/libbre_nodir.so; do
  n=$(basename $lib .so)
  BRE_LIBRARY=$lib timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_$n.npz" c2 > "$OUT/bc_$n.log" 2>&1 \
      || { tail -n 20 "$OUT/bc_$n.log"; exit 1; }
done
python3 profiles/r5/bitcmp.py cmp "$OUT/bc_libbre.npz" "$OUT/bc_libbre_nodir.npz"
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); n = sys.argv[2]
c = d.get("counters_last_iteration") or {}
print(n, "value", round(d["value"]), "gather", round(d["gather_kernel_ms"], 1), "it0", round(d["gather_ms_per_step"][0], 1),
      "it15", round(d["gather_ms_per_step"][-1], 1) if len(d["gather_ms_per_step"]) > 15 else None,
      "keep", round(d.get("bundle_keep_frac", 0), 4), "t/q", round(d.get("prefilter_tests_per_queued_pair", 0), 2),
      "| late keep", round(c.get("bundle_keep_frac", 0), 4), "t/q", round(c.get("prefilter_tests_per_queued_pair", 0), 2),
      "leaf/wave", round(c.get("leaf_visits_per_wave", 0), 2))
PY
}
C3="--workload c3 --steps 1 --warmup 1"
run c2_def $DEF
run c2_nodir $V/libbre_nodir.so
run c3_def $DEF $C3
run c3_nodir $V/libbre_nodir.so $C3
run c2_def_b $DEF
run c2_nodir_b $V/libbre_nodir.so
