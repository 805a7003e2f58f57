#!/bin/bash
# Round 3 sweep 1 (via gpurun): with the (start, end) tree order, re-sweep the tile kernel's knobs on
# the C2 bench: leaf tile size, work roots (split), transposed-scan threshold, segment sort key.
set -o pipefail
OUT=${1:-gpurun_out/r3/sweep1}
mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1 \
      || { tail -n 20 "$OUT/$name.log"; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base && run leaf32 --tile-leaf 32 && run split128 --split 128 && run tscan4 --tscan 4 && run tscan8 --tscan 8 \
  && run key0 --sort-key 0 && run base2
