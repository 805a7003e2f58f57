#!/bin/bash
# Round 4 run 26 (via gpurun): work roots by size-balanced splitting (largest internal root first)
# instead of the breadth-first frontier -- parity tests, then C2 at N = 1 and emulated ranks 0 of 8 / 0 of 4
# against the previous commit's gather object (variant head), C3 at N = 1.
set -o pipefail
OUT=${1:-gpurun_out/r4/run26}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py tests/test_pipeline_gpu.py tests/test_boundary_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])])"
}
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run n1_new $NEW
run n1_head $V/libbre_head.so
run r0of8_new $NEW --emulate-shard 0/8 --pipeline 0
run r0of8_head $V/libbre_head.so --emulate-shard 0/8 --pipeline 0
run r0of4_new $NEW --emulate-shard 0/4 --pipeline 0
run r0of8_new_p1 $NEW --emulate-shard 0/8
run c3_new $NEW --workload c3 --steps 1 --warmup 1
run c3_head $V/libbre_head.so --workload c3 --steps 1 --warmup 1
