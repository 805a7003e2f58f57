#!/bin/bash
# Round 3b run 16 (via gpurun): packet blocks (map 4) with the exact stage's SegRec from LDS (default
# build) or from global memory (variant pkg) -- where the packet blocks lose their time.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run16}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run map3 ""
run map4 "" --block-map 4
run map4_glob pkg --block-map 4
C3="--workload c3 --steps 1 --warmup 0"
run c3_map4 "" $C3 --block-map 4
run c3_map4_glob pkg $C3 --block-map 4
