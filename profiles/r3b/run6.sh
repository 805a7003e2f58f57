#!/bin/bash
# Round 3b run 6 (via gpurun): the tile axis reject with the beam loads issued before its test --
# production parity tests, then C2 A/B (on, off, on, off) and C3 A/B.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run6}
mkdir -p "$OUT"
T="tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -n 30 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run axis1
run axis0 --tile-axis 0
run axis1b
run axis0b --tile-axis 0
run c3_axis1 --workload c3 --steps 1 --warmup 0
run c3_axis0 --workload c3 --steps 1 --warmup 0 --tile-axis 0
