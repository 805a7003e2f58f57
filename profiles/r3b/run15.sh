#!/bin/bash
# Round 3b run 15 (via gpurun): packet blocks (block map 4: one 8-wave workgroup per packet, SegRec
# planes in LDS, work roots claimed from an LDS counter) -- tests, then C2 / C3 A/B against map 3.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run15}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_packet_blocks_gpu.py > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run map3
run map4 --block-map 4
run map5 --block-map 5
run map6 --block-map 6
C3="--workload c3 --steps 1 --warmup 0"
run c3_map3 $C3
run c3_map5 $C3 --block-map 5
run c3_map6 $C3 --block-map 6

run map3b
