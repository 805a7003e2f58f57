#!/bin/bash
# Round 5 run 22 (via gpurun): the adaptive transposed-scan threshold build (default tslope 15) against
# HEAD's kernel (fixed threshold 6) on one box: C2 A/B/A/B, C3, and tscan 4 on HEAD's kernel.
set -o pipefail
OUT=${1:-gpurun_out/r5/run22}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'it0-3', [round(x,1) for x in g[:4]], 'it15', round(g[-1],1))"
}
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
BASE=$V/libbre_base.so
BRE_LIBRARY=$DEF timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 || exit 1
BRE_LIBRARY=$BASE timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_base.npz" c2 > "$OUT/bc_base.log" 2>&1 || exit 1
python3 profiles/r5/bitcmp.py cmp "$OUT/bc_def.npz" "$OUT/bc_base.npz"; rm -f "$OUT"/*.npz
for r in a b; do
  run c2_def_$r $DEF
  run c2_base_$r $BASE
  run c2_base_t4_$r $BASE --tscan 4
done
run c3_def $DEF --workload c3 --steps 1 --warmup 1
run c3_base $BASE --workload c3 --steps 1 --warmup 1
run c3_base_t3 $BASE --workload c3 --steps 1 --warmup 1 --tscan 3
