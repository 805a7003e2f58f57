#!/bin/bash
# Round 4 run 12 (via gpurun): where the last few % vs round 3 go -- the default (tile line reject on,
# queue counted per batch), reject off at run time, the queue count compiled out (nq), also the reject
# compiled out (nqt), both + round 3's accumulation (r3like), the round-3 library; C2, one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run12}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run c2_new $NEW
run c2_notax $NEW --tile-axis 0
run c2_nq $V/libbre_nq.so
run c2_nqt $V/libbre_nqt.so
run c2_r3like $V/libbre_r3like.so
run c2_r3 $V/libbre_r3.so
run c2_new2 $NEW
