#!/bin/bash
# Round 4 run 33 (via gpurun): the transposed scan with two on-lane segments per step (ILP, queue order
# unchanged) -- sums bit for bit against the previous commit's gather (variant head) at C2 iterations
# 0 / 8 and C3, parity tests, then C2 / C3 timing against head on one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run33}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
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
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run c2_new $NEW
run c2_head $V/libbre_head.so
run c3_new $NEW $C3
run c3_head $V/libbre_head.so $C3
run c2_new2 $NEW
run c2_head2 $V/libbre_head.so
