#!/bin/bash
# Round 3 sweep 2 (via gpurun): with the (start, end) tree order, re-sweep the tile kernel's knobs on
# the C2 bench: Hilbert instead of Morton order for the tree (beam key 2) and the segment sort (key 4).
set -o pipefail
OUT=${1:-gpurun_out/r3/sweep2}
mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1 \
      || { tail -n 20 "$OUT/$name.log"; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base && run bk2 --beam-key 2 && run sk4 --sort-key 4 && run both --beam-key 2 --sort-key 4 && run base2
