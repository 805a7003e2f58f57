#!/bin/bash
# Round 4 run 11 (via gpurun): what the rank costs -- verified ds_or_rtn_b64 ranks (default), the same
# without the order check (rk2), round 3's ds_add_rtn_u32 ranks (rk1), rk1 + 8 rounds + atomics (= round
# 3's accumulation in the current kernel), the round-3 library; C2, one box, timing only.
set -o pipefail
OUT=${1:-gpurun_out/r4/run11}
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
run c2_rk2 $V/libbre_rk2.so
run c2_rk1 $V/libbre_rk1.so
run c2_rk1r8 $V/libbre_rk1r8.so
run c2_r3 $V/libbre_r3.so
run c2_new2 $NEW
run c2_rk1r8b $V/libbre_rk1r8.so
