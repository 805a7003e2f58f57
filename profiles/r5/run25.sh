#!/bin/bash
# Round 5 run 23 / 25 (via gpurun): 23: the transposed scan queueing beam by beam (bit columns per lane); 25: the sorted lane chain for deep batches; against
# HEAD's segment-by-segment queueing -- parity tests, sums bit for bit, C2 / C3 at thresholds 4 / 6 / 8.
set -o pipefail
OUT=${1:-gpurun_out/r5/run23}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_c2_production.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 40 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
BASE=$V/libbre_base.so
BRE_LIBRARY=$DEF timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 || exit 1
BRE_LIBRARY=$BASE timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_base.npz" c2 > "$OUT/bc_base.log" 2>&1 || exit 1
python3 profiles/r5/bitcmp.py cmp "$OUT/bc_def.npz" "$OUT/bc_base.npz"; rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'it0-3', [round(x,1) for x in g[:4]], 'it15', round(g[-1],1))"
}
for t in 4 6 8; do
  run c2_def_t$t $DEF --tscan $t
  run c2_base_t$t $BASE --tscan $t
done
for t in 4 6 8; do
  run c3_def_t$t $DEF --workload c3 --steps 1 --warmup 1 --tscan $t
  run c3_base_t$t $BASE --workload c3 --steps 1 --warmup 1 --tscan $t
done
run c2_def_t6_b $DEF --tscan 6
run c2_base_t4_b $BASE --tscan 4
