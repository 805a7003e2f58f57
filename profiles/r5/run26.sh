#!/bin/bash
# Round 5 run 26 (via gpurun): the tile kernel built with the compiler's other scheduling strategies
# (max-ilp, max-memory-clause) against the default: sums bit for bit, C2 and C3 timing.
set -o pipefail
OUT=${1:-gpurun_out/r5/run26}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
BRE_LIBRARY=$DEF timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 || exit 1
for n in ilp memc; do
  BRE_LIBRARY=$V/libbre_$n.so timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_$n.npz" c2 > "$OUT/bc_$n.log" 2>&1 || exit 1
  echo "== def vs $n"; python3 profiles/r5/bitcmp.py cmp "$OUT/bc_def.npz" "$OUT/bc_$n.npz"; rm -f "$OUT/bc_$n.npz"
done
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'it0-3', [round(x,1) for x in g[:4]], 'it15', round(g[-1],1))"
}
for r in a b; do
  run c2_def_$r $DEF
  run c2_ilp_$r $V/libbre_ilp.so
  run c2_memc_$r $V/libbre_memc.so
done
run c3_def $DEF --workload c3 --steps 1 --warmup 1
run c3_ilp $V/libbre_ilp.so --workload c3 --steps 1 --warmup 1
run c3_memc $V/libbre_memc.so --workload c3 --steps 1 --warmup 1
