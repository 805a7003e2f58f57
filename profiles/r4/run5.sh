#!/bin/bash
# Round 4 run 5 (via gpurun): the round-3 kernel with documented-order accumulation (OR-mask ranks,
# read-modify-write rounds to the end: no LDS float atomics) and the deterministic per-pixel film
# compose -- parity + determinism tests, then C2 / C3 timing against the round-3 library on one box,
# and per-iteration timing of tile leaf 32 (the small-radius lever).
set -o pipefail
OUT=${1:-gpurun_out/r4/run5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_c2_production.py tests/test_radius_layout_gpu.py \
    tests/test_prefilter_options_gpu.py tests/test_film_determinism_gpu.py tests/test_pipeline_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
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
run c2_r3 $V/libbre_r3.so
run c2_leaf32 $NEW --tile-leaf 32
run c3_new $NEW $C3
run c3_r3 $V/libbre_r3.so $C3
run c2_new2 $NEW
run c2_r3b $V/libbre_r3.so
