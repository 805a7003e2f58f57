#!/bin/bash
# Round 4 run 8 (via gpurun): the per-lane tile line reject (option 112 = 1: lanes whose segment line is
# too far from a tile's axis line leave the tile before it is staged) -- option / parity tests, then
# C2 / C3 timing with and without it, the rank-mask variants, the round-3 library; one diag line.
set -o pipefail
OUT=${1:-gpurun_out/r4/run8}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 3 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run c2_new $NEW
run c2_tax $NEW --tile-axis 1
run c2_radd $V/libbre_radd.so
run c2_rr8 $V/libbre_rr8.so
run c2_r3 $V/libbre_r3.so
run c3_new $NEW $C3
run c3_tax $NEW $C3 --tile-axis 1
run c3_r3 $V/libbre_r3.so $C3
run c2_tax2 $NEW --tile-axis 1
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --tile-axis 1 --json-out "$OUT/diag_tax.json" > "$OUT/diag_tax.log" 2>&1 || { tail -n 20 "$OUT/diag_tax.log"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/diag.json" > "$OUT/diag.log" 2>&1 || { tail -n 20 "$OUT/diag.log"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
for n in ("diag", "diag_tax"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    keys = ["leaf_visits_per_wave", "beam_lines_staged_per_wave", "exact_batches_per_wave", "bundle_keep_frac",
            "queued_pairs_per_estimate", "contributions_per_queued_pair", "prefilter_tests_per_queued_pair"]
    print(n, "value", round(d["value"]), {k: round(d[k], 3) for k in keys})
    print(n, "last", {k: round(v, 3) if isinstance(v, float) else v for k, v in d.get("counters_last_iteration", {}).items()})
PY
