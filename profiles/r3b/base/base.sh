#!/bin/bash
# Session re-entry check (via gpurun): production parity tests, C2 bench, C3 one iteration.
set -o pipefail
OUT=${1:-gpurun_out/r3b/base}
mkdir -p "$OUT"
bash profiles/quick.sh "$OUT" || exit 1
timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --json-out "$OUT/c3.json" \
    > "$OUT/c3.log" 2>&1 || { tail -n 30 "$OUT/c3.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('c3 value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1))"
