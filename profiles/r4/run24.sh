#!/bin/bash
# Round 4 run 24 (via gpurun): packet-shard chunk size (--shard-block B: chunks of B sorted packets dealt
# round-robin to the ranks) for an emulated 1/8 rank of C2, ranks 0 and 7, against N = 1.
set -o pipefail
OUT=${1:-gpurun_out/r4/run24}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2))"
}
run n1
for b in 1 4 16 64; do
  run r0of8_b$b --emulate-shard 0/8 --shard-block $b
  run r7of8_b$b --emulate-shard 7/8 --shard-block $b
done
