#!/bin/bash
# Round 5 run 7 (via gpurun): does the two-context pipeline overlap when the gather is several launches?
# (the other stream's passes are dispatched between launches).  C2 at N = 1 and an emulated rank of 8,
# partial cap (option 109) = one launch / ~4 / ~8 launches per gather.
set -o pipefail
OUT=${1:-gpurun_out/r5/run7}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'over', round(d['ms_per_step']-d['gather_kernel_ms'],2))"
}
for r in a b; do
  run n1_one_$r
  run n1_p512_$r --partial-mib 512
  run n1_p256_$r --partial-mib 256
  run e8_one_$r --emulate-shard 0/8
  run e8_p64_$r --emulate-shard 0/8 --partial-mib 64
  run e8_p32_$r --emulate-shard 0/8 --partial-mib 32
done
