#!/bin/bash
# Round 4 run 35 (via gpurun): XCD-aware LPT block map (map 5: XCD x sweeps the subtrees of size rank x mod 8)
# against map 3, C2 at N = 1 and rank 0 of 8, C3.
set -o pipefail
OUT=${1:-gpurun_out/r4/run35}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])][:6])"
}
for m in 3 5; do
  run n1_m$m --block-map $m
  run r0of8_m$m --emulate-shard 0/8 --block-map $m
  run c3_m$m --workload c3 --steps 1 --warmup 1 --block-map $m
done
run n1_m3b --block-map 3
