#!/bin/bash
# Round 5 run 13 (via gpurun): packet-shard chunk size (--shard-block: packets per chunk dealt
# round-robin) for an emulated rank of 8 at C2, and the N = 1 line for reference.
set -o pipefail
OUT=${1:-gpurun_out/r5/run13}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'over', round(d['ms_per_step']-d['gather_kernel_ms'],2))"
}
run n1
for r in a b; do
  for b in 1 4 16 64; do run e8_b${b}_$r --emulate-shard 0/8 --shard-block $b; done
done
run e8_b16_r3 --emulate-shard 3/8 --shard-block 16
run e8_b1_r3 --emulate-shard 3/8 --shard-block 1
