#!/bin/bash
# Round 4 run 25 (via gpurun): work roots S = 64 / 128 / 256 for an emulated 1/8 rank of C2 (is the
# rank's excess over 1/8 of the gather the kernel's tail of long (packet, subtree) waves?), and S at N=1.
set -o pipefail
OUT=${1:-gpurun_out/r4/run25}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])])"
}
run n1
for s in 64 128 256; do run r0of8_s$s --emulate-shard 0/8 --split $s --pipeline 0; done
run r0of2 --emulate-shard 0/2 --pipeline 0
run r0of4 --emulate-shard 0/4 --pipeline 0
