#!/bin/bash
# Round 4 run 39 (via gpurun): work-root shards with more roots (S = 512 / 1024: each rank of 8 gets
# 64 / 128 of them, so the ranks' shares of the work average out better) -- ranks 0 / 3 / 7 of 8, C2.
set -o pipefail
OUT=${1:-gpurun_out/r4/run39}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])][:4])"
}
for s in 512 1024; do
  for r in 0 3 7; do run s${s}_r${r} --emulate-shard $r/8 --shard-mode roots --split $s; done
done
for r in 1 2 4 5 6; do run s256_r${r} --emulate-shard $r/8 --shard-mode roots; done
