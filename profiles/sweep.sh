#!/bin/bash
# Bench sweep over argument sets (no CPU leg / PMC / counters pass); one JSON per set.
# usage (repo root, via gpurun): profiles/sweep.sh OUTDIR "ARGS1" "ARGS2" ...
set -o pipefail
OUT=${1:-gpurun_out/sweep}
shift || true
mkdir -p "$OUT"
i=0
for a in "$@"; do
  i=$((i + 1))
  timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/s$i.json" $a > "$OUT/s$i.log" 2>&1 \
      || { echo "[$a] failed"; tail -n 20 "$OUT/s$i.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/s$i.json'));print('[$a]', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
done
