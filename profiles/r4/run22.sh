#!/bin/bash
# Round 4 run 22 (via gpurun): the parallel k_roots and block-reduced k_segbox (work roots and the 4-wide
# view now computed in the build) -- per-segment sums bit for bit against the previous commit's gather
# object (variant head) at C2 iterations 0 / 8 and C3; parity tests; C2 at N=1 and an emulated 1/8 rank.
set -o pipefail
OUT=${1:-gpurun_out/r4/run22}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py tests/test_pipeline_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
for w in c2 c3; do
  timeout -k 10 300 python -u profiles/r3b/bitcmp.py dump "$OUT/new_$w.npz" $w > "$OUT/dump_new_$w.log" 2>&1 || { tail -n 20 "$OUT/dump_new_$w.log"; exit 1; }
  BRE_LIBRARY=$V/libbre_head.so timeout -k 10 300 python -u profiles/r3b/bitcmp.py dump "$OUT/head_$w.npz" $w > "$OUT/dump_head_$w.log" 2>&1 || { tail -n 20 "$OUT/dump_head_$w.log"; exit 1; }
  python3 profiles/r3b/bitcmp.py cmp "$OUT/new_$w.npz" "$OUT/head_$w.npz"
done
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2))"
}
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run n1_new $NEW
run n1_head $V/libbre_head.so
run r0of8_new $NEW --emulate-shard 0/8
run r0of8_head $V/libbre_head.so --emulate-shard 0/8
run r0of8_new_p0 $NEW --emulate-shard 0/8 --pipeline 0
