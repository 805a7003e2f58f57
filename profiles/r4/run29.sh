#!/bin/bash
# Round 4 run 29 (via gpurun): strong-scaling emulation of the round's final kernel on one GPU -- C2
# ranks 0 of 2 / 4 / 8 and 7 of 8 (bench.py --emulate-shard R/N, pipelined as in the real run), C4 ranks
# 0 and 5 of 8, against N = 1.
set -o pipefail
OUT=${1:-gpurun_out/r4/run29}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2))"
}
run c2_n1
run c2_0of2 --emulate-shard 0/2
run c2_0of4 --emulate-shard 0/4
run c2_0of8 --emulate-shard 0/8
run c2_7of8 --emulate-shard 7/8
run c4_n1 --workload c4 --steps 1 --warmup 0
run c4_0of8 --workload c4 --steps 1 --warmup 0 --emulate-shard 0/8
run c4_5of8 --workload c4 --steps 1 --warmup 0 --emulate-shard 5/8
