#!/bin/bash
# Round 3b run 5 (via gpurun): buffer-descriptor loads (default) + the tile axis reject (default) --
# the GPU suite without C4 (parity), then C2 / C3 benches with the tile axis reject on and off.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run5}
mkdir -p "$OUT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not c4" \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'staged/wave', round(d.get('beam_lines_staged_per_wave',0)))"
}
run axis1
run axis0 --tile-axis 0
run axis1b
run c3_axis1 --workload c3 --steps 1 --warmup 0
run c3_axis0 --workload c3 --steps 1 --warmup 0 --tile-axis 0
