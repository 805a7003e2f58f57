#!/bin/bash
# Round 3b run 17 (via gpurun): r = dist / MaxDistance through the shared reciprocal for uniform-radius
# sets -- layout tests (bit identity against the division) + parity, then C2 / C3 A/B.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run17}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_radius_layout_gpu.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run rec
run split --split-records 1
C3="--workload c3 --steps 1 --warmup 0"
run c3_rec $C3
run c3_split $C3 --split-records 1
run rec2
run c3_rec2 $C3
