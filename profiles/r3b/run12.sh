#!/bin/bash
# Round 3b run 12 (via gpurun): exact-stage load ablations (timing only, wrong images) --
# 6: no power load (pw[b]), 7: no SegRec loads (the executing lane's own segment values).
set -o pipefail
OUT=${1:-gpurun_out/r3b/run12}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base ""
run ab6 ab6
run ab7 ab7
C3="--workload c3 --steps 1 --warmup 0"
run c3 "" $C3
run c3_ab6 ab6 $C3
run c3_ab7 ab7 $C3
run base2 ""
