#!/bin/bash
# Round 5 run 26 / 27 (via gpurun): 26: the compiler scheduling strategies; 27: wave priority (s_setprio) while loads issue
# (max-ilp, max-memory-clause) against the default: sums bit for bit, C2 and C3 timing.
set -o pipefail
OUT=${1:-gpurun_out/r5/run26}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
BRE_LIBRARY=$DEF timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 || exit 1
for n in ${VARS:-ilp memc}; do
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
  for n in ${VARS:-ilp memc}; do run c2_${n}_$r $V/libbre_$n.so; done
done
run c3_def $DEF --workload c3 --steps 1 --warmup 1
for n in ${VARS:-ilp memc}; do run c3_$n $V/libbre_$n.so --workload c3 --steps 1 --warmup 1; done
