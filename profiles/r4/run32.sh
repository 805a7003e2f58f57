#!/bin/bash
# Round 4 run 32 (via gpurun): two ranks per read-modify-write round in deep exact batches
# (BRE_PAIR_ROUNDS; threshold BRE_PAIR_MIN 4 in-tree, 2 / 8 variants, off = nopair) -- per-segment sums
# bit for bit against nopair at C2 iterations 0 / 8 and C3, parity tests, C2 / C3 timing on one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run32}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
for w in c2 c3; do
  timeout -k 10 300 python -u profiles/r3b/bitcmp.py dump "$OUT/new_$w.npz" $w > "$OUT/dump_new_$w.log" 2>&1 || { tail -n 20 "$OUT/dump_new_$w.log"; exit 1; }
  BRE_LIBRARY=$V/libbre_nopair.so timeout -k 10 300 python -u profiles/r3b/bitcmp.py dump "$OUT/nopair_$w.npz" $w > "$OUT/dump_nopair_$w.log" 2>&1 || { tail -n 20 "$OUT/dump_nopair_$w.log"; exit 1; }
  python3 profiles/r3b/bitcmp.py cmp "$OUT/new_$w.npz" "$OUT/nopair_$w.npz"
done
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])][:4])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
for w in c2 c3; do
  A=""; [ $w = c3 ] && A=$C3
  run ${w}_new $NEW $A
  run ${w}_nopair $V/libbre_nopair.so $A
  run ${w}_pair2 $V/libbre_pair2.so $A
  run ${w}_pair8 $V/libbre_pair8.so $A
done
run c2_new2 $NEW
