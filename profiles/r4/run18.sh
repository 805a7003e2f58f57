#!/bin/bash
# Round 4 run 18 (via gpurun): the packet box reject compiled out (nobox: staging loads no box, more
# beams kept) against the default, C2 / C3, one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run18}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
for w in c2 c3; do
  A=""; [ $w = c3 ] && A=$C3
  run ${w}_new $NEW $A
  run ${w}_nobox $V/libbre_nobox.so $A
done
run c2_new2 $NEW
