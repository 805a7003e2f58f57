#!/bin/bash
# Round 5 run 18 (via gpurun): an emulated rank of 8 at C2 -- work roots per packet (--split) and block
# map (LPT 3 / XCD subtrees 0 / rotated 1), to see what the rank's gather loses above 1/8 of N = 1.
set -o pipefail
OUT=${1:-gpurun_out/r5/run18}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'it0', round(g[0],2), 'it15', round(g[-1],2))"
}
run n1
for r in a b; do
  run e8_s256_m3_$r --emulate-shard 0/8
  run e8_s128_m3_$r --emulate-shard 0/8 --split 128
  run e8_s512_m3_$r --emulate-shard 0/8 --split 512
  run e8_s256_m0_$r --emulate-shard 0/8 --block-map 0
  run e8_s256_m1_$r --emulate-shard 0/8 --block-map 1
done
